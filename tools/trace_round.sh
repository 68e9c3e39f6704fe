#!/usr/bin/env bash
# rocprofv3 kernel traces of the graph-replayed timed loop, per BASELINE config (run through
# gpurun from the repo root), each regrouped per op with the config's launch table:
#   gpurun_out/trace/<cfg>/...kernel_trace.csv, <cfg>_launches.tsv, trace_<cfg>_ops.csv
# Copy trace_<cfg>_ops.csv (+ the *_kernel_stats.csv) to profiles/<round>/: bench.py's roofline
# takes the op with the largest summed device time from there (bench.trace_ranking).
# usage: tools/trace_round.sh [model:batch:precision ...]
set -euo pipefail
cfgs=("$@")
if [ ${#cfgs[@]} -eq 0 ]; then
  cfgs=(resnet18:8:fp16m bert_base:8:fp16 resnet152:32:fp16x3 vit_l_16:16:fp16)
fi
out=gpurun_out/trace
mkdir -p "$out"
for c in "${cfgs[@]}"; do
  IFS=: read -r model batch prec <<< "$c"
  tag="${model}_bs${batch}_${prec}"
  rm -rf "$out/$tag"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$tag" -- \
    python3 bench.py --loop-only --model "$model" --batch "$batch" --precision "$prec" \
    --launch-table "$out/${tag}_launches.tsv" --steps 20 --warmup 5 > "$out/${tag}_loop.json" 2> "$out/${tag}_loop.err"
  trace=$(ls "$out/$tag"/*/*_kernel_trace.csv | head -n 1)
  python3 tools/trace_ops.py "$trace" --launches "$out/${tag}_launches.tsv" --csv "$out/trace_${tag}_ops.csv" --top 12
  cp "$(ls "$out/$tag"/*/*_kernel_stats.csv | head -n 1)" "$out/trace_${tag}_kernel_stats.csv"
  rm -rf "$out/$tag"  # the raw trace (tens of MB) stays on the box
done
