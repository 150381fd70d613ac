#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that ends in a
# fault, abort, segfault or time limit (rc not 0/1) stops the chain.
#   tools/gpu_steps.sh OUTDIR "name:seconds:command" ...
OUT=$1; shift
mkdir -p "$OUT"
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "[step] $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.txt" 2>&1
  rc=$?
  echo "[step] $name rc=$rc"
  tail -3 "$OUT/$name.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[step] stopping after rc=$rc"; exit $rc; fi
done
