# One GPU call: k_trace2 / k_shade unit counters (TA, TD, TCP) on C3, shading section
# clocks on C4 and C5, then the first frame after a large process at several budgets.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python tools/pmc_units.py --config C3 --spp 64 > gpurun_out/pmc_units_c3.jsonl 2> gpurun_out/pmc_units_c3.err || { tail -5 gpurun_out/pmc_units_c3.err; exit 1; }
cut -c1-900 gpurun_out/pmc_units_c3.jsonl
timeout -k 10 300 python tools/variants.py run --config C4 --spp 128 --frames 1 base sclk > gpurun_out/sclk_c4.log 2>&1
timeout -k 10 300 python tools/variants.py run --config C5 --spp 32 --frames 1 base sclk > gpurun_out/sclk_c5.log 2>&1
grep -E "IZPI_SHADE|shade_ms" gpurun_out/sclk_c4.log gpurun_out/sclk_c5.log | cut -c1-300
bash tools/ff_after_hog.sh C4 "0 67108864 33554432" 130 > gpurun_out/ffh_c4.log 2>&1
cat gpurun_out/ffh_c4.log
