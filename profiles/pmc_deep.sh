#!/bin/bash
# Deeper PMC passes for k_trace2 (one rocprofv3 run per group; stops at the first
# pass that times out). Usage: bash profiles/pmc_deep.sh TAG CONFIG SPP "group1" "group2" ...
TAG=$1; CFG=$2; SPP=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --spp $SPP > $OUT/g$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then exit $rc; fi
done
