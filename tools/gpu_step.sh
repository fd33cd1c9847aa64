# Run GPU steps in order; stop at the first that ends in anything but success or an
# ordinary test failure (fault, abort, segfault, time limit: nothing more runs on the GPU).
#   bash tools/gpu_step.sh OUTDIR "name:seconds:command" ...
OUT=$1; shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  tail -3 "$OUT/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
done
