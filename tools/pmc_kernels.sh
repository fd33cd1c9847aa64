#!/bin/bash
# PMC counter groups (one rocprofv3 --pmc pass each, no tracing) over one C3 frame:
#   bash tools/pmc_kernels.sh TAG [SPP]   -> gpurun_out/pmc_TAG/gN/...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r2}; SPP=${2:-512}; CFG=${CONFIG:-C3}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_FLAT" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 tools/first_frame.py --config $CFG --frames 1 --spp $SPP > $OUT/g$i.log 2>&1 || { echo "group $i failed"; exit 1; }
done
python3 tools/pmc_report.py $OUT > $OUT/report.txt 2>&1; cat $OUT/report.txt
