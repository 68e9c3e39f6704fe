#!/usr/bin/env bash
# HBM bytes per op of isolated forwards: two rocprofv3 PMC passes (FETCH_SIZE,
# WRITE_SIZE -- counters only, no trace domains), then tools/pmc_traffic.py.
# usage: tools/pmc_traffic.sh OUTDIR [trace_forward.py args...]
set -euo pipefail
out=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -- \
  python3 tools/trace_forward.py --ops-out "$out/ops.json" "$@" > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -- \
  python3 tools/trace_forward.py "$@" > "$out/write.log" 2>&1
python3 tools/pmc_traffic.py "$out/fetch" "$out/write" "$out/ops.json" -o "$out/traffic.json"
