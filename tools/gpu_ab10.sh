# One GPU call: shared sin/cos reduction and shared-reciprocal vector division (base) against
# the sin/cos change alone (nodiv) and the previous commit (ps), alternating processes; the
# gomath device test (ops 11-13) and the shading parity tests first.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_materials.py -x -q --timeout 200 --timeout-method thread -k "gomath or kernel_variants or c4 or c5 or c3 or spectral or pbr or glass or metal or sphere or normal or texture or small_scene" > gpurun_out/t10.log 2>&1 || { tail -30 gpurun_out/t10.log; exit 1; }
tail -2 gpurun_out/t10.log
O=gpurun_out/ab10.log
V="timeout -k 10 300 python tools/variants.py run --frames 1"
$V --config C4 --spp 128 base nodiv ps base nodiv ps > $O
$V --config C3 --spp 128 base nodiv ps base nodiv ps >> $O
$V --config C5 --spp 32 base nodiv ps >> $O
python - <<'PY'
import json
for l in open("gpurun_out/ab10.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["variant"], d["trace_ms"], d["shade_ms"], d["device_ms"], d["digest"][:8])
PY
