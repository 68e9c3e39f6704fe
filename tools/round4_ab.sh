#!/usr/bin/env bash
# Round-4 A/B runs on one GPU (four worker streams, interleaved rounds in one process each):
#   ViT-L bs16 fp16: defaults vs no split-K anywhere (gemm256's new slices included) vs no LN fold
#   BERT-base bs8 fp16: defaults vs no LN fold
#   ResNet-18 bs8 fp16m: defaults vs the plain tap walk (SPI_GEMM_WIN=0) vs plan target T 96 / 192
#   H2D: SDMA copies vs worker-stream copies (C4, C5: the configs SPI_H2D_AUTO sends to the stream)
# usage: bash tools/round4_ab.sh [OUTDIR]   (default gpurun_out/ab)
set -euo pipefail
out=${1:-gpurun_out/ab}
mkdir -p "$out"
sweep() {  # name secs args...
  local n=$1 t=$2; shift 2
  echo "== $n" >&2
  timeout -k 10 "$t" python3 -u tools/policy_sweep.py "$@" > "$out/$n.log" 2>&1
}
sweep vit 420 --model vit_l_16 --batch 16 --precision fp16 --steps 10 --rounds 3 \
  --policy base= --policy nosplit=SPI_GEMM_MAXSPLIT=1 --policy nofold=SPI_LN_FOLD=0
sweep bert 300 --model bert_base --batch 8 --precision fp16 --rounds 3 \
  --policy base= --policy nofold=SPI_LN_FOLD=0
sweep r18 300 --model resnet18 --batch 8 --precision fp16m --rounds 3 \
  --policy base= --policy nowin=SPI_GEMM_WIN=0 --policy t96=SPI_GEMM_POLICY=tput:96 \
  --policy t192=SPI_GEMM_POLICY=tput:192
sweep r152 300 --model resnet152 --batch 32 --precision fp16x3 --steps 10 --rounds 3 \
  --policy base= --policy nowin=SPI_GEMM_WIN=0
for m in resnet152 vit_l_16; do
  echo "== sdma $m" >&2
  ROUNDS=2 timeout -k 10 300 python3 -u tools/sdma_ab.py "$m" > "$out/sdma_$m.log" 2>&1
done
echo done >&2
