#!/bin/bash
# On the GPU box: time variants (izpi_amd/_lib/variants/*.so) on one config, alternating.
#   VARIANTS="A B" bash tools/vrun.sh CONFIG SPP ROUNDS
CFG=${1:-C3}; SPP=${2:-512}; R=${3:-2}
for r in $(seq 1 $R); do
  for v in ${VARIANTS}; do
    IZPI_LIB_PATH=$PWD/izpi_amd/_lib/variants/$v.so timeout -k 10 300 python tools/first_frame.py --config $CFG --spp $SPP --frames 3 2>&1 | grep '^{"config' | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); f=d['frames'][1:]
print('$v', 'device_ms %.1f trace %.1f shade %.1f hbm %.1f' % tuple(sum(x[k] for x in f)/len(f) for k in ('device_ms','trace_ms','shade_ms','hbm_used_gb')))" || exit 1
  done
done
