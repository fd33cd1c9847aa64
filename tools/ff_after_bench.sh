# One-shot frame right after another large-workspace render process: a C2
# bench process (128 GB of workspace, frames rendered) exits, then a fresh process renders
# its first frame of CONFIG at each wavefront slot budget (tools/first_frame.py).
#   bash tools/ff_after_bench.sh CONFIG "SLOTS..."
set -e
mkdir -p gpurun_out
CFG=${1:-C3}; SLOTS=${2:-"0 134217728 67108864"}
for s in $SLOTS; do
  timeout -k 10 200 python bench.py --config C2 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/ffb_prev.log 2>&1
  timeout -k 10 300 python tools/first_frame.py --config $CFG --frames 2 --slots $s > gpurun_out/ffb_${CFG}_s$s.log 2>&1
  grep '^{"config' gpurun_out/ffb_${CFG}_s$s.log | python -c "
import json, sys
d = json.loads(sys.stdin.read()); f = d['frames']
print(json.dumps({'config': d['config'], 'after': 'C2 bench', 'slots': f[0]['slots'], 'workspace_gb': round(f[0]['workspace_gb'], 1), 'first_wall_ms': round(f[0]['wall_ms'], 1), 'first_alloc_ms': round(f[0]['alloc_ms'], 1), 'steady_wall_ms': round(f[1]['wall_ms'], 1), 'steady_device_ms': round(f[1]['device_ms'], 1), 'setup_s': round(d['setup_s'], 3)}))"
done
# the allocation rate itself after the same kind of process, at once and after a pause
for pause in 0 5; do
  timeout -k 10 200 python bench.py --config C2 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/ffb_prev.log 2>&1
  timeout -k 10 120 python tools/alloc_probe.py --chunks 8 --gb 16 --pause $pause
done
