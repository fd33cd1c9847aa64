#!/bin/bash
# k_accumulate's average duration, default library against variants/base.so (rocprofv3 kernel stats).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base cur; do
  lib=""; [ $v = base ] && lib="$PWD/izpi_amd/_lib/variants/base.so"
  IZPI_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/acc_$v -o run -- python3 tools/first_frame.py --config ${CFG:-C3} --frames 2 > gpurun_out/acc_$v.log 2>&1
  f=$(find gpurun_out/acc_$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(grep -E 'k_accumulate' $f | cut -d, -f1-4)"
done
