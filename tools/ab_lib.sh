#!/bin/bash
# Same-box A/B(/C...) of builds of libnas.so (boxes differ by several percent,
# so small changes are compared on one box, alternating): runs `bench.py ARGS`
# ROUNDS times with each library and prints one JSON per run, named by the
# library's letter (A_1.json, B_1.json, C_1.json, ...).
# usage (on the GPU box, from the repo root):
#   tools/ab_lib.sh A.so B.so [C.so ...] ROUNDS OUTDIR -- ARGS...
set -uo pipefail
LIBS=()
while [ $# -gt 0 ] && [ "${1%.so}" != "$1" ]; do LIBS+=("$1"); shift; done
R=$1; OUT=$2; shift 3
LIB=kubernetesnetawarescheduler_amd/libnas.so
mkdir -p "$OUT"
cp "$LIB" "$OUT/orig.so"
TAGS=(A B C D E F)
for i in $(seq 1 "$R"); do
  for k in "${!LIBS[@]}"; do
    cp "${LIBS[$k]}" "$LIB"
    timeout -k 10 300 python3 bench.py "$@" > "$OUT/${TAGS[$k]}_$i.json" 2>> "$OUT/err.log" \
      || { cp "$OUT/orig.so" "$LIB"; exit 1; }
  done
done
cp "$OUT/orig.so" "$LIB"
