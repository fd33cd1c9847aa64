#!/bin/bash
# k_accumulate's average duration, default library against variants/base.so (rocprofv3 kernel stats).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base cur; do
  lib=""; [ $v = base ] && lib="$PWD/izpi_amd/_lib/variants/base.so"
  IZPI_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/acc_$v -o run -- python3 tools/first_frame.py --config ${CFG:-C3} --frames 2 > gpurun_out/acc_$v.log 2>&1
  f=$(find gpurun_out/acc_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r[\"Name\"]: print(sys.argv[3], r[\"Name\"][:40], r[\"Calls\"], r[\"AverageNs\"])" $f ${KERNEL:-k_accumulate} $v
done
