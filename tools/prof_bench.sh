#!/bin/bash
# Profiles for the judged bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command itself (`bench.py --steps 10
#      --warmup 2`, everything the driver's line has except the in-run PMC
#      child, which cannot nest under a profiler), then tools/check_roofline.py:
#      each roofline's HIP-event launch time vs the rocprof mean of the same
#      dispatches;
#   2. marker trace of the placement leg (roctx ranges of the C-ABI entries);
#   3. PMC passes over the scoring leg, one counter group per run (gfx950 slot
#      limits): MFMA busy / wait / LDS / clock counters, FETCH_SIZE, WRITE_SIZE
#      (k_fit, k_cost_topk and k_merge HBM bytes).
# usage: tools/prof_bench.sh OUTDIR
set -uo pipefail
OUT=$(realpath -m "$1")
ROOT=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_bench" -o t \
  -- python3 "$ROOT/bench.py" --no-pmc --steps 10 --warmup 2 > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" \
  || { echo "bench trace failed"; exit 1; }
python3 "$ROOT/tools/check_roofline.py" "$OUT/trace_bench.json" "$OUT/trace_bench/t_kernel_trace.csv" \
  > "$OUT/check_roofline.json"
echo "check_roofline rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$OUT/trace_place" -o t \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-pmc --only place --steps 3 --warmup 1 \
  > "$OUT/trace_place.json" 2> "$OUT/trace_place.err" || { echo "place trace failed"; exit 1; }
B="$ROOT/bench.py --no-cpu-baseline --no-pmc"
i=0
for pmc in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pmc$i" -o p \
    -- python3 $B --only score --steps 2 --warmup 0 > "$OUT/pmc$i.log" 2>&1 || { echo "pmc $i failed"; exit 1; }
done
echo done > "$OUT/DONE"
