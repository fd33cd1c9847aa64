# One GPU call: the parity suite, then a short bench (PMC passes included).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/first_frame.py --frames 2 > gpurun_out/ff.log 2>&1
tail -1 gpurun_out/ff.log
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
