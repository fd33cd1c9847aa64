# One GPU call: light samples read from the staged LDS tables (base) against the global GLight
# load (div = -DIZPI_NO_LRAND_LDS), alternating processes; previous commit (ps) alongside.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_materials.py -x -q --timeout 200 --timeout-method thread -k "gomath or kernel_variants or c4 or c5 or c3 or spectral or pbr or glass or metal or sphere or normal or texture or small_scene or light" > gpurun_out/t11.log 2>&1 || { tail -30 gpurun_out/t11.log; exit 1; }
tail -2 gpurun_out/t11.log
O=gpurun_out/ab11.log
V="timeout -k 10 300 python tools/variants.py run --frames 1"
$V --config C3 --spp 128 base div ps base div ps > $O
$V --config C4 --spp 128 base div ps base div ps >> $O
$V --config C5 --spp 32 base div ps >> $O
$V --config C2 --spp 256 base div ps >> $O
python - <<'PY'
import json
for l in open("gpurun_out/ab11.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["variant"], d["trace_ms"], d["shade_ms"], d["device_ms"], d["digest"][:8])
PY
