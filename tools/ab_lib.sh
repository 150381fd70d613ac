#!/bin/bash
# Same-box A/B of two builds of libnas.so (boxes differ by several percent, so
# small changes are compared on one box, alternating): runs
# `bench.py ARGS` ROUNDS times with each library and prints one JSON per run.
# usage (on the GPU box, from the repo root): tools/ab_lib.sh A.so B.so ROUNDS OUTDIR -- ARGS...
set -uo pipefail
A=$1; B=$2; R=$3; OUT=$4; shift 5
LIB=kubernetesnetawarescheduler_amd/libnas.so
mkdir -p "$OUT"
cp "$LIB" "$OUT/orig.so"
for i in $(seq 1 "$R"); do
  for v in A B; do
    if [ $v = A ]; then cp "$A" "$LIB"; else cp "$B" "$LIB"; fi
    timeout -k 10 300 python3 bench.py "$@" > "$OUT/${v}_$i.json" 2>> "$OUT/err.log" || { cp "$OUT/orig.so" "$LIB"; exit 1; }
  done
done
cp "$OUT/orig.so" "$LIB"
