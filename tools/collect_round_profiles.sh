#!/usr/bin/env bash
# Copy a round's GPU profiling outputs (tools/round4_profile.sh, tools/profile_round.sh) from
# gpurun_out/ into profiles/<round>/ under the names bench.py reads:
#   trace_<cfg>_ops.csv / _kernel_stats.csv   (the timed loop's rocprofv3 trace, per op)
#   roofline_rocprof.json, roofline_<cfg>_kernel_stats.csv  (the roofline op's back-to-back launches)
#   traffic_<cfg>.json, mfma_<cfg>.json        (PMC: HBM bytes and MFMA-busy per op)
# usage: tools/collect_round_profiles.sh r04
set -euo pipefail
r=${1:?round, e.g. r04}
dst=profiles/$r
mkdir -p "$dst"
cp gpurun_out/trace/trace_*_ops.csv gpurun_out/trace/trace_*_kernel_stats.csv "$dst/" 2>/dev/null || true
if [ -f gpurun_out/rl_$r/roofline_rocprof.json ]; then
  cp gpurun_out/rl_$r/roofline_rocprof.json "$dst/roofline_rocprof.json"
  cp gpurun_out/rl_$r/roofline_*_kernel_stats.csv "$dst/" 2>/dev/null || true
fi
for d in gpurun_out/pmc_*; do
  [ -d "$d" ] || continue
  cfg=${d#gpurun_out/pmc_}
  [ -f "$d/traffic.json" ] && cp "$d/traffic.json" "$dst/traffic_${cfg}.json"
  [ -f "$d/mfma.json" ] && cp "$d/mfma.json" "$dst/mfma_${cfg}.json"
done
ls -la "$dst"
