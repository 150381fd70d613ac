#!/bin/bash
# PMC passes over the cost kernel microbenchmark (one counter group per run,
# within gfx950's per-block slot limits); run on the GPU box from the repo root.
# usage: tools/pmc_cost.sh OUTDIR [variants]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; V=${2:-a}
mkdir -p "$OUT"
M=kubernetesnetawarescheduler_amd/csrc/tools/mb_cost
i=0
for pmc in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD TA_BUSY_avr TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
  "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o p -- $M 10000 100000 1 ${V} > $OUT/p$i.log 2>&1
done
