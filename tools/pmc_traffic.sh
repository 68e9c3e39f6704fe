#!/usr/bin/env bash
# HBM bytes and MFMA-busy per op of isolated forwards: three rocprofv3 PMC passes
# (FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CU_CYCLES +
# GRBM_GUI_ACTIVE -- counters only, no trace domains; FETCH_SIZE and WRITE_SIZE
# need 3 + 2 of the 4 TCC slots, so they never share a pass), then
# tools/pmc_traffic.py.
# usage: tools/pmc_traffic.sh OUTDIR [trace_forward.py args...]
set -euo pipefail
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -- \
  python3 tools/trace_forward.py --ops-out "$out/ops.json" "$@" > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -- \
  python3 tools/trace_forward.py "$@" > "$out/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$out/mfma" -- python3 tools/trace_forward.py "$@" > "$out/mfma.log" 2>&1
python3 tools/pmc_traffic.py "$out/fetch" "$out/write" "$out/ops.json" --mfma "$out/mfma" -o "$out/traffic.json" \
  --mfma-out "$out/mfma.json"
