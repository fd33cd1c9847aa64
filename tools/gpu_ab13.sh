# One GPU call: no kind words for scenes without path-length rays (base) against the previous
# head (prev), alternating processes; the full GPU parity suite first (parking included).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t13.log 2>&1 || { tail -30 gpurun_out/t13.log; exit 1; }
tail -2 gpurun_out/t13.log
O=gpurun_out/ab13.log
V="timeout -k 10 300 python tools/variants.py run --frames 2"
$V --config C3 --spp 512 base prev base prev base prev > $O
$V --config C4 --spp 256 base prev base prev >> $O
$V --config C2 --spp 256 base prev base prev >> $O
python - <<'PY'
import json
for l in open("gpurun_out/ab13.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["config"], d["variant"], d["frame"], d["slots"], d["trace_ms"], d["shade_ms"], d["device_ms"], round(d["device_ms"] - d["trace_ms"] - d["shade_ms"] - d["tail_ms"], 3), d["digest"][:8])
PY
