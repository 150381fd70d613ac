#!/bin/bash
# Profiles for the judged bench line (run on the GPU box from the repo root):
#   kernel-trace + stats of the scoring launch (bench --only score), the vote
#   launch (--only vote) and the pipelined placement (--only place), then
#   separate PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass)
#   over the scoring and vote launches for the HBM traffic figure.
# usage: tools/prof_bench.sh OUTDIR
set -euo pipefail
OUT=$(realpath -m "$1")
ROOT=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --no-cpu-baseline"
for only in score vote place; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$only" -o t \
    -- python3 $B --only $only --steps 5 --warmup 1 > "$OUT/trace_$only.json" 2> "$OUT/trace_$only.err"
done
for only in score vote; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pmc_${only}_$pmc" -o p \
      -- python3 $B --only $only --steps 1 --warmup 0 > "$OUT/pmc_${only}_$pmc.log" 2>&1
  done
done
echo done > "$OUT/DONE"
