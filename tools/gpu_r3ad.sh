set -e
timeout -k 10 200 python tools/shard_probe.py --config C3 --worlds 1,8 > gpurun_out/shard_ad.log 2>&1
timeout -k 10 200 python tools/shard_probe.py --config C3 --worlds 1,8 --tail-paths 200000 >> gpurun_out/shard_ad.log 2>&1
timeout -k 10 200 python tools/shard_probe.py --config C3 --worlds 1,8 --tail-paths 500000 >> gpurun_out/shard_ad.log 2>&1
timeout -k 10 200 python tools/shard_probe.py --config C3 --worlds 1,8 --tail-paths 30000 >> gpurun_out/shard_ad.log 2>&1
