#!/bin/bash
# On the GPU box: time variants on one config, alternating, frames 2.. of a fresh renderer.
#   VARIANTS="A B name:IZPI_X=1,IZPI_Y=2" bash tools/vrun.sh CONFIG SPP ROUNDS
# A plain name runs izpi_amd/_lib/variants/NAME.so; "name:ENV=..." runs the default library
# with those environment variables.
CFG=${1:-C3}; SPP=${2:-512}; R=${3:-2}
for r in $(seq 1 $R); do
  for v in ${VARIANTS}; do
    name=${v%%:*}
    if [ "$name" != "$v" ]; then envs=$(echo "${v#*:}" | tr ',' ' '); lib=""; else envs=""; lib="IZPI_LIB_PATH=$PWD/izpi_amd/_lib/variants/$v.so"; fi
    env $lib $envs timeout -k 10 300 python tools/first_frame.py --config $CFG --spp $SPP --frames 3 2>&1 | grep '^{"config' | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); f=d['frames'][1:]
print('$name', 'device_ms %.1f trace %.1f shade %.1f tail %.1f rays %.0f parks %.0f hbm %.1f' % tuple(sum(x[k] for x in f)/len(f) for k in ('device_ms','trace_ms','shade_ms','tail_ms','rays','parks','hbm_used_gb')))" || exit 1
  done
done
