# One GPU call: small scenes' primitive records in LDS for shading (base) against global
# loads (flags=256, IZPI_TUNE_NO_PRIM_LDS) inside one process each (tools/ab_inproc.py), and
# against the previous head's library; parity tests of the shading paths first.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_materials.py -x -q --timeout 200 --timeout-method thread -k "kernel_variants or c4 or c5 or c2 or spectral or pbr or glass or metal or dielectric or zero or sphere or normal or texture" > gpurun_out/t9.log 2>&1 || { tail -30 gpurun_out/t9.log; exit 1; }
tail -2 gpurun_out/t9.log
O=gpurun_out/ab9.log
: > $O
for c in "C4 --spp 128" "C5 --spp 32" "C2 --spp 256"; do
  timeout -k 10 300 python tools/ab_inproc.py --config $c --rounds 3 base flags=256 >> $O
done
timeout -k 10 300 python tools/variants.py run --frames 1 --config C4 --spp 128 base head base head >> $O
python - <<'PY'
import json
for l in open("gpurun_out/ab9.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d.get("setting", d.get("variant")), d.get("round", d.get("frame")), d["trace_ms"], d["shade_ms"], d["device_ms"], d["digest"][:8])
PY
