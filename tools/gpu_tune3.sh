# k_trace2 launch settings re-swept for the ray-in-LDS instance (C3), in one process
# (tools/ab_inproc.py: settings alternate frame by frame, so they share the process's mode).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python tools/ab_inproc.py --config C3 --spp 128 --rounds 3 base prim_weight=24 prim_weight=40 refill_min=16 refill_min=32 trace_chunk=256 trace_chunk=1024 prim_weight=28,refill_min=20 > gpurun_out/tune3.log 2>&1
python - <<'PY'
import json, collections
acc = collections.defaultdict(list)
for l in open("gpurun_out/tune3.log"):
    if l.startswith("{"):
        d = json.loads(l)
        acc[d["setting"]].append((d["trace_ms"], d["digest"]))
for k, v in acc.items():
    print(k, [t for t, _ in v], round(sum(t for t, _ in v) / len(v), 3), set(g for _, g in v))
PY
