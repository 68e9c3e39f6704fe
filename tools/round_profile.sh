#!/usr/bin/env bash
# Roofline evidence of a round (ROUND=r06 by default) for every BASELINE GPU config (run through gpurun from the repo root):
#   1. tools/trace_round.sh: rocprofv3 kernel trace of each config's graph-replayed timed loop,
#      regrouped per op (gpurun_out/trace/trace_<cfg>_ops.csv + kernel stats);
#   2. the trace CSVs copied into profiles/$ROUND/ of this (scratch) tree, so bench.py's roofline
#      picks each config's op from them (bench.trace_ranking) -- copy them into the repo too;
#   3. per config, rocprofv3 --kernel-trace --stats of `bench.py --roofline-only` for the top op
#      of its trace (the back-to-back launches the bench line times) -> gpurun_out/rl_$ROUND/
#      roofline_rocprof.json (tools/rocprof_roofline.py) + roofline_<cfg>_kernel_stats.csv.
# usage: ROUND=r06 bash tools/round_profile.sh
set -euo pipefail
ROUND=${ROUND:-r06}
export TMPDIR=/tmp
cfgs=(resnet18:8:fp16m bert_base:8:fp16 resnet152:32:fp16x3 vit_l_16:16:fp16)
if [ "${SKIP_TRACE:-0}" != 1 ]; then  # SKIP_TRACE=1: the committed profiles/$ROUND traces pick the ops
  mkdir -p gpurun_out/trace
  bash tools/trace_round.sh "${cfgs[@]}" > gpurun_out/trace/log.txt 2>&1
  mkdir -p profiles/$ROUND
  cp gpurun_out/trace/trace_*_ops.csv profiles/$ROUND/
fi
out=gpurun_out/rl_$ROUND
mkdir -p "$out"
for c in "${cfgs[@]}"; do
  IFS=: read -r model batch prec <<< "$c"
  tag="${model}_bs${batch}_${prec}"
  op=$(python3 - "$tag" "$ROUND" <<'EOF'
import csv, sys
rows = [r for r in csv.DictReader(open(f"profiles/{sys.argv[2]}/trace_{sys.argv[1]}_ops.csv")) if r["op"]]
rows.sort(key=lambda r: -float(r["total_us"]))
print(rows[0]["op"].split("|")[0])
EOF
)
  echo "== $tag: $op"
  rm -rf "$out/$tag"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$tag" -- \
    python3 bench.py --roofline-only --roofline-op "$op" --model "$model" --batch "$batch" --precision "$prec" \
    > "$out/${tag}_roofline.json" 2> "$out/${tag}_roofline.err"
  stats=$(ls "$out/$tag"/*/*_kernel_stats.csv | head -n 1)
  ktrace=$(ls "$out/$tag"/*/*_kernel_trace.csv | head -n 1)
  python3 tools/rocprof_roofline.py "$stats" "$op" "$out/roofline_rocprof.json" "$ktrace"
  cp "$stats" "$out/roofline_${tag}_kernel_stats.csv"
  rm -rf "$out/$tag"
done
echo done
