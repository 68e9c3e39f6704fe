#!/usr/bin/env bash
# Which engine carries the e2e path's H2D / D2H copies, and what the HIP copy knobs do to it
# (run through gpurun from the repo root):
#   1. rocprofv3 kernel + memory-copy trace of the e2e leg -> gpurun_out/cp/prof/
#      (SDMA copies appear as memory copies, shader copies as __amd_rocclr_copyBuffer kernels)
#   2. bench.py --extras 0 under each knob setting          -> gpurun_out/cp/<name>.json
set -euo pipefail
out=gpurun_out/cp
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$out/prof" -- \
  python3 bench.py --extras 0 --cpu-seconds 0 > "$out/traced.json" 2> "$out/traced.err"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --extras 0 --cpu-seconds 0 > "$out/$name.json" 2>> "$out/ab.err"
}
run base X=0
run largebar0 ROC_ENABLE_LARGE_BAR=0
run forceblit0 GPU_FORCE_BLIT_COPY_SIZE=0
run blitwg16 DEBUG_CLR_LIMIT_BLIT_WG=16
run base2 X=0
