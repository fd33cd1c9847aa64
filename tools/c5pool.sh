for v in "base:IZPI_NOP=1" "div2:IZPI_POOL_DIV=2" "div1:IZPI_POOL_DIV=1" "dense24:IZPI_REC_DENSE=24" "dense32:IZPI_REC_DENSE=32"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 python tools/first_frame.py --config C5 --spp 256 --frames 1 2>&1 | grep '^{"wall' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'device_ms %.0f trace %.0f shade %.0f rays %.3g parks %.3g hbm %.1f' % (d['device_ms'], d['trace_ms'], d['shade_ms'], d['rays'], d['parks'], d['hbm_used_gb']))"
done
