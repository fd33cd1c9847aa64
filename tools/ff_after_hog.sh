# One-shot frame right after another large-workspace process (BASELINE §4):
# a "hog" process fills HOG_GB of HBM and exits, then a fresh process renders its first
# frame at each wavefront slot budget (tools/first_frame.py); alloc_ms is the host time
# its workspace allocations took (the driver clears VRAM the previous process freed).
#   bash tools/ff_after_hog.sh CONFIG "SLOTS..." [HOG_GB]
set -e
mkdir -p gpurun_out
CFG=${1:-C4}; SLOTS=${2:-"0 67108864 33554432 16777216"}; HOG=${3:-130}
for s in $SLOTS; do
  timeout -k 10 120 python -c "import torch; x = torch.empty(int($HOG * 1e9) // 8, dtype=torch.float64, device='cuda'); x.fill_(1.0); torch.cuda.synchronize(); print('hog', $HOG, 'GB')"
  timeout -k 10 300 python tools/first_frame.py --config $CFG --frames 2 --slots $s > gpurun_out/ffh_${CFG}_s$s.log 2>&1
  grep '^{"config' gpurun_out/ffh_${CFG}_s$s.log | python -c "
import json, sys
d = json.loads(sys.stdin.read()); f = d['frames']
print(json.dumps({'config': d['config'], 'slots': f[0]['slots'], 'workspace_gb': round(f[0]['workspace_gb'], 1), 'first_wall_ms': round(f[0]['wall_ms'], 1), 'first_alloc_ms': round(f[0]['alloc_ms'], 1), 'steady_wall_ms': round(f[1]['wall_ms'], 1), 'steady_device_ms': round(f[1]['device_ms'], 1), 'setup_s': round(d['setup_s'], 3)}))"
done
