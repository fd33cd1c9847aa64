set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --config C5 --spp 32 --no-cpu-baseline --no-reference-check > gpurun_out/c5.log 2>&1
grep '^{' gpurun_out/c5.log | tail -1 | python -c "import json,sys;d=json.load(sys.stdin);x=d['detail'];print(d['value'], x['rank0_trace_ms_per_step'], x['rank0_shade_ms_per_step'])"
