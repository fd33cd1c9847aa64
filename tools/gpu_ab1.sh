set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "kernel_variants or dragon or c3_frame or trace_closest" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
V="timeout -k 10 200 python tools/variants.py run --config C3 --spp 128 --frames 2"
O=gpurun_out/ab1.log
$V base > $O; $V --tune flags=128 base >> $O; $V pf >> $O; $V --tune flags=128 pf >> $O; $V base >> $O
cut -c1-400 $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 python tools/pmc_variants.py --config C3 --spp 64 base base@flags=128 pf > gpurun_out/pmc1.log 2>&1 || { tail -30 gpurun_out/pmc1.log; exit 1; }
cat gpurun_out/pmc1.log
