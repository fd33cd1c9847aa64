# One-shot frame cost against the wavefront slot count (C4, C3): a fresh process per slot
# count, first and second frame with their allocation time (tools/first_frame.py).
set -e
mkdir -p gpurun_out
for s in 0 134217728 67108864 33554432; do
  timeout -k 10 200 python tools/first_frame.py --config C4 --frames 2 --slots $s > gpurun_out/ff_c4_s$s.log 2>&1
  grep '^{' gpurun_out/ff_c4_s$s.log | tail -1 | cut -c1-600
done
for s in 0 67108864; do
  timeout -k 10 200 python tools/first_frame.py --config C3 --frames 2 --slots $s > gpurun_out/ff_c3_s$s.log 2>&1
  grep '^{' gpurun_out/ff_c3_s$s.log | tail -1 | cut -c1-600
done
