set -e
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/gputests.log 2>&1 || { tail -5 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for v in main nosort; do
  if [ $v != main ]; then cp izpi_amd/_lib/variants/$v.so izpi_amd/_lib/libizpi_gpu.so; fi
  timeout -k 10 200 python tools/tune.py --config C3 --spp 256 --rounds 2 > gpurun_out/ab_c3_$v.log 2>&1
  timeout -k 10 200 python bench.py --config C5 --spp 16 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c5_$v.log 2>&1
done
