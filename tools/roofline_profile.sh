#!/usr/bin/env bash
# Round evidence for bench.py's roofline (run through gpurun from the repo root):
#   1. the default bench line                          -> gpurun_out/rl/bench.json
#   2. rocprofv3 --kernel-trace --stats of the roofline leg for the op the bench line named
#      (bench.py --roofline-only --roofline-op <op>: one warm-up task, then the op's
#      back-to-back launches the bench times)           -> gpurun_out/rl/prof/
#   3. rocprofv3 --kernel-trace --stats of the headline's timed loop (no extras)
#                                                       -> gpurun_out/rl/prof_bench/
# Copy the *_kernel_stats.csv files and tools/trace_ops.py regroupings into profiles/<round>/.
set -euo pipefail
out=gpurun_out/rl
mkdir -p "$out"
timeout -k 10 400 python3 bench.py "$@" > "$out/bench.json" 2> "$out/bench.err"
op=$(python3 -c "import json,sys; print(json.loads(open('$out/bench.json').read().strip().splitlines()[-1])['roofline']['kernel'])")
echo "roofline op: $op"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -- \
  python3 bench.py --roofline-only --roofline-op "$op" > "$out/roofline_only.json" 2> "$out/roofline_only.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_bench" -- \
  python3 bench.py --extras 0 --cpu-seconds 0 > "$out/bench_prof.json" 2> "$out/bench_prof.err"
python3 tools/rocprof_roofline.py "$(ls "$out"/prof/*/*_kernel_stats.csv | head -n 1)" "$op" "$out/roofline_rocprof.json"
