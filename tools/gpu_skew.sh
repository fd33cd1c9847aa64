# Shading-time modes: state arrays offset against each other by 4352 B (sk1),
# 33 MB + 4352 B (sk2), 1.3 MB + 4352 B (sk3) against none (base), C3 at 128 spp, each in its
# own process; a 250-GB hog process before the second round (the fast-mode condition).
set -e
mkdir -p gpurun_out
O=gpurun_out/skew.log
V="timeout -k 10 300 python tools/variants.py run --frames 2 --config C3 --spp 128"
$V base sk1 sk2 sk3 base sk1 sk2 sk3 > $O
timeout -k 10 120 python -c "import torch; x = torch.empty(int(250e9) // 8, dtype=torch.float64, device='cuda'); x.fill_(1.0); torch.cuda.synchronize(); print('hog 250 GB')" >> $O
$V sk2 base sk2 base >> $O
python - <<'PY'
import json
for l in open("gpurun_out/skew.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["variant"], d["frame"], d["trace_ms"], d["shade_ms"], d["device_ms"], d["digest"][:8])
    else:
        print(l.strip())
PY
