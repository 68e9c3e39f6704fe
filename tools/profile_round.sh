#!/usr/bin/env bash
# Round profile collection on the GPU box (run through gpurun from the repo root):
#   * HBM traffic + MFMA-busy per op for the four BASELINE GPU configs (tools/pmc_traffic.sh:
#     separate FETCH_SIZE / WRITE_SIZE / MFMA-busy PMC passes, counters only);
#   * results land in gpurun_out/pmc_<model>_bs<B>_<prec>/{traffic,mfma}.json; copy them to
#     profiles/<round>/{traffic,mfma}_<model>_bs<B>_<prec>.json (bench.py reads the newest round).
# usage: tools/profile_round.sh [config ...]   config = model:batch:precision
set -euo pipefail
cfgs=("$@")
if [ ${#cfgs[@]} -eq 0 ]; then
  cfgs=(resnet18:8:fp16m bert_base:8:fp16 resnet152:32:fp16x3 vit_l_16:16:fp16)
fi
for c in "${cfgs[@]}"; do
  IFS=: read -r model batch prec <<< "$c"
  out="gpurun_out/pmc_${model}_bs${batch}_${prec}"
  echo "== $model bs$batch $prec -> $out"
  bash tools/pmc_traffic.sh "$out" --model "$model" --batch "$batch" --precision "$prec" --iters 12 > "$out.txt" 2>&1 \
    || { echo "pmc pass failed for $c"; tail -20 "$out.txt"; exit 1; }
  tail -3 "$out.txt"
done
