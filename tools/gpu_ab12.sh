# One GPU call: (1) Colour records padded to 48 B (rec6) against 40-B records (base), C4;
# (2) k_accumulate staged through LDS (base) against per-lane strided loads (acc0), C3 / C2:
# the accumulate time is device_ms - trace - shade - tail. Parity tests first.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "c3 or c2 or kernel_variants or accumulate or tiles or chunk or spectral" > gpurun_out/t12.log 2>&1 || { tail -30 gpurun_out/t12.log; exit 1; }
tail -2 gpurun_out/t12.log
O=gpurun_out/ab12.log
V="timeout -k 10 300 python tools/variants.py run --frames 2"
$V --config C4 --spp 128 base rec6 base rec6 base rec6 > $O
$V --config C3 --spp 512 base acc0 base acc0 >> $O
$V --config C2 --spp 256 base acc0 >> $O
python - <<'PY'
import json
for l in open("gpurun_out/ab12.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["variant"], d["frame"], d["slots"], d["trace_ms"], d["shade_ms"], d["device_ms"], round(d["device_ms"] - d["trace_ms"] - d["shade_ms"] - d["tail_ms"], 3), d["digest"][:8])
PY
