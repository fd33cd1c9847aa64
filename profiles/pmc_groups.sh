#!/bin/bash
# PMC counter groups (one rocprofv3 pass each, no tracing domains) on a short bench run.
#   bash profiles/pmc_groups.sh TAG CONFIG SPP
set -e
TAG=${1:-r1}
CFG=${2:-C3}
SPP=${3:-32}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --spp $SPP > $OUT/g$i.log 2>&1
done
ls $OUT/*/
