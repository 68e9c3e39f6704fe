#!/usr/bin/env bash
# One rocprofv3 pass per counter group (counters only, no trace domains) over
# isolated forwards; analyse with tools/pmc_ops.py OUTDIR.
# usage: tools/pmc_ops.sh OUTDIR [trace_forward.py args...]
set -euo pipefail
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS"
)
# (TA_*_sum counters made a pass hang past its limit on this pool; left out)
i=0
for g in "${groups[@]}"; do
  if [ "$i" = 0 ]; then extra=(--ops-out "$out/ops.json"); else extra=(); fi
  timeout -k 10 240 rocprofv3 --pmc $g --output-format csv -d "$out/p$i" -- \
    python3 tools/trace_forward.py "${extra[@]}" "$@" > "$out/p$i.log" 2>&1
  i=$((i+1))
done
