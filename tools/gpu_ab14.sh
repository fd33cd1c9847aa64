# One GPU call: one texel index for a PBR hit's same-size images (base) against one index per
# lookup (prev), C4 alternating processes; the texture / PBR parity tests first.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_materials.py -x -q --timeout 200 --timeout-method thread -k "pbr or texture or normal or c4 or spectral or small_scene or kernel_variants" > gpurun_out/t14.log 2>&1 || { tail -30 gpurun_out/t14.log; exit 1; }
tail -2 gpurun_out/t14.log
O=gpurun_out/ab14.log
V="timeout -k 10 300 python tools/variants.py run --frames 2"
$V --config C4 --spp 256 base prev base prev base prev > $O
python - <<'PY'
import json
for l in open("gpurun_out/ab14.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["variant"], d["frame"], d["slots"], d["trace_ms"], d["shade_ms"], d["device_ms"], d["digest"][:8])
PY
