#!/bin/bash
# Builds tools/mb_aux.hip once per knob setting (here on the CPU) or runs the
# built binaries alternately on the GPU box.
#   build: tools/mb_aux.sh build TAG "-DKNOB=V ..." [TAG "-D..." ...]
#   run:   tools/mb_aux.sh run ROUNDS TAG... (from the repo root; prints lines)
set -euo pipefail
D=$(dirname "$0")
if [ "$1" = build ]; then
  shift
  while [ $# -ge 2 ]; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I/opt/rocm/include -I"$D/.." \
      -I"$D/../../../include" -DMB_TAG="\"$1\"" $2 -o "$D/mb_aux_$1" "$D/mb_aux.hip" &
    shift 2
  done
  wait
else
  R=$2; shift 2
  for i in $(seq 1 "$R"); do
    for t in "$@"; do timeout -k 5 60 "$D/mb_aux_$t" 10000 100000 4; done
  done
fi
