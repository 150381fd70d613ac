#!/bin/bash
# Profiles for the judged bench line (run on the GPU box from the repo root):
#   kernel-trace + stats of the scoring leg (bench --only score: full-size
#   k_cost_topk launches), the vote leg (--only vote) and the pipelined
#   placement (--only place); then PMC passes over the scoring leg, one
#   counter group per run (gfx950 slot limits): MFMA / wait / clock counters,
#   FETCH_SIZE, WRITE_SIZE (k_fit, k_cost_topk and k_merge HBM bytes).
# usage: tools/prof_bench.sh OUTDIR
set -uo pipefail
OUT=$(realpath -m "$1")
ROOT=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --no-cpu-baseline --no-pmc"
for only in score vote place; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$only" -o t \
    -- python3 $B --only $only --steps 10 --warmup 2 > "$OUT/trace_$only.json" 2> "$OUT/trace_$only.err" \
    || { echo "trace $only failed"; exit 1; }
done
i=0
for pmc in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pmc$i" -o p \
    -- python3 $B --only score --steps 2 --warmup 0 > "$OUT/pmc$i.log" 2>&1 || { echo "pmc $i failed"; exit 1; }
done
echo done > "$OUT/DONE"
