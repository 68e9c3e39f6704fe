#!/bin/bash
# Round-5 profile collection: timed-loop traces + roofline rocprof summaries, then PMC traffic /
# MFMA-busy per op, for the four BASELINE GPU configs (gpurun from the repo root).
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ROUND=r05 timeout -k 10 1000 bash tools/round_profile.sh > gpurun_out/r5_round_profile.log 2>&1 || { tail -30 gpurun_out/r5_round_profile.log; exit 1; }
tail -3 gpurun_out/r5_round_profile.log
timeout -k 10 900 bash tools/profile_round.sh > gpurun_out/r5_pmc.log 2>&1 || { tail -30 gpurun_out/r5_pmc.log; exit 1; }
tail -5 gpurun_out/r5_pmc.log
