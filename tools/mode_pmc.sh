#!/bin/bash
# Shading-time modes: the same C3 frame in several fresh processes, each under
# one rocprofv3 --pmc pass of translation / cache counters; k_shade's time tells the mode.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mode
rocprofv3 --list-avail 2>/dev/null | grep -i -E "UTCL|TLB" | head -20 > gpurun_out/mode/avail.txt
cat gpurun_out/mode/avail.txt | head -20
CTRS=${CTRS:-"TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCC_HIT_sum TCC_MISS_sum"}
for i in 1 2 3 4 5; do
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d gpurun_out/mode/p$i -o run -- python3 tools/first_frame.py --config C3 --frames 2 > gpurun_out/mode/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/mode/p$i.log; exit 1; }
  grep '^{"wall' gpurun_out/mode/p$i.log | tail -1
done
