# One GPU call: k_trace2's per-XCD-group queue segments (IZPI_TUNE_XCD_SEG, 256) against one
# cursor, on the LDS-BVH configs (C4, C2, C5) and C3; the kernel-variant parity test first.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "kernel_variants" > gpurun_out/t8.log 2>&1 || { tail -30 gpurun_out/t8.log; exit 1; }
tail -2 gpurun_out/t8.log
O=gpurun_out/ab8.log
V="timeout -k 10 300 python tools/variants.py run --frames 2"
: > $O
for c in "C4 --spp 128" "C2 --spp 256" "C5 --spp 32" "C3 --spp 128"; do
  for r in 1 2; do
    $V --config $c base >> $O
    $V --config $c --tune flags=256 base >> $O
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/ab8.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["tune"], d["frame"], d["trace_ms"], d["shade_ms"], d["device_ms"], d["digest"][:8])
PY
