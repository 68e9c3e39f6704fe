#!/usr/bin/env bash
# PMC passes (one rocprofv3 run per counter group -- FETCH_SIZE takes 3 of the 4 TCC
# slots and WRITE_SIZE 2, so they never share a pass -- counters only -- no trace
# domains) over one gemm_bench shape.  usage: tools/pmc_passes.sh OUTDIR ONLY PREC
set -euo pipefail
out=$1; only=$2; prec=${3:-fp16x3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM"
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE"
)
i=0
for g in "${groups[@]}"; do
  timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d "$out/p$i" -- \
    python3 tools/gemm_bench.py --eager --reps 20 --only "$only" --prec "$prec" > "$out/p$i.log" 2>&1
  i=$((i+1))
done
