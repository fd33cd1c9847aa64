# One GPU call: FETCH_SIZE calibration on known-byte gathers, then k_trace2's per-class
# bytes past L2 from the shadow-load builds (tools/variants.py build shN -DIZPI_SHADOW=N).
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/fetch_calib.py > gpurun_out/fetch_calib.jsonl 2> gpurun_out/fetch_calib.err || { tail -20 gpurun_out/fetch_calib.err; exit 1; }
cut -c1-300 gpurun_out/fetch_calib.jsonl
timeout -k 10 200 python tools/variants.py run --config C3 --spp 64 --frames 1 base sh0 > gpurun_out/sh_run.log 2>&1 || { tail -20 gpurun_out/sh_run.log; exit 1; }
grep -E "IZPI_SHADOW|trace_ms" gpurun_out/sh_run.log | cut -c1-300
timeout -k 10 900 python tools/pmc_variants.py --config C3 --spp 64 base sh0 sh1 sh2 sh4 > gpurun_out/pmc_sh.log 2>&1 || { tail -30 gpurun_out/pmc_sh.log; exit 1; }
cat gpurun_out/pmc_sh.log
