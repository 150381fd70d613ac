#!/bin/bash
# Kernel timeline of rank 0 of a G = 8 C3 pass (rehearsal) and the rank-0
# pass time at G = 1, 2, 4, 8 (run on the GPU box from the repo root).
#   tools/rehearse_sweep.sh OUTDIR
set -uo pipefail
OUT=$(realpath -m "$1"); ROOT=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
B="--only place --no-cpu-baseline --no-pmc --no-configs --no-reference-mode"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr8" -o t \
    -- python3 "$ROOT/bench.py" $B --rehearse-world 8 --steps 5 --warmup 2 > "$OUT/g8.json" 2>&1 ) || { echo "trace failed"; exit 1; }
python3 tools/pass_timeline.py "$OUT/tr8" > "$OUT/g8_timeline.txt"
for G in 1 2 4 8; do
  timeout -k 10 120 python3 bench.py $B --rehearse-world $G --steps 30 --warmup 3 > "$OUT/reh$G.json" 2> "$OUT/reh$G.err" || exit 1
  python3 -c "import json; d=json.load(open('$OUT/reh$G.json')); print($G, round(d['ms_per_step'],3), round(d['roofline']['launch_ms'],3))"
done
