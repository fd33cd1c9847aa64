# One GPU call: C2 bench with its reference-tree check (one workspace per process now), then
# C4's bench: C4's first frame shows what the driver had to clear.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config C2 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/ff2_c2.log 2>&1
timeout -k 10 400 python bench.py --config C4 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-reference-check > gpurun_out/ff2_c4.log 2>&1
for f in gpurun_out/ff2_c2.log gpurun_out/ff2_c4.log; do grep '^{' $f | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); dd=d['detail']; print(d['config']['workload'], d['value'], d['ms_per_step'], dd['first_frame_ms'], dd['first_frame_alloc_ms'], dd['hbm_workspace_gb'], (dd.get('reference_tree') or {}).get('image_bitwise_equal'))"; done
