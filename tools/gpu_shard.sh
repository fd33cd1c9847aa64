# Per-share cost of an 8-way C3 split on one GPU (tools/shard_probe.py) at the default k_tail
# threshold and larger ones, plus one per-pass log of the default.
set -e
mkdir -p gpurun_out
O=gpurun_out/shard_r4.log
: > $O
timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 1,8 >> $O 2>&1
for t in 262144 524288 1048576 2097152; do
  echo "tail_paths $t" >> $O
  timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 1,8 --tail-paths $t >> $O 2>&1
done
timeout -k 10 300 python tools/shard_probe.py --config C3 --worlds 8 --pass-log > gpurun_out/shard_r4_passlog.log 2>&1
grep -v amdgpu.ids $O | tail -40
