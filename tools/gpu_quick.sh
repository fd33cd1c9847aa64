# One GPU call: smoke, the parity suite, C3 and C5 frames of a fresh renderer.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/first_frame.py --frames 3 > gpurun_out/ff_c3.log 2>&1
grep '^{"wall' gpurun_out/ff_c3.log
timeout -k 10 200 python tools/first_frame.py --config C5 --spp 16 --frames 3 > gpurun_out/ff_c5.log 2>&1
grep '^{"wall' gpurun_out/ff_c5.log
