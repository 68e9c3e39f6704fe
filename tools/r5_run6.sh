#!/bin/bash
# Round-5: ViT LayerNorm fold re-measure, ResNet-18 weight-resident conv A/B.
set -o pipefail
O=gpurun_out/r5/${1:-g}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 3 \
  --policy "default=" --policy "fold=SPI_LN_FOLD=1" > $O/vit_fold.txt 2>&1 || { tail -30 $O/vit_fold.txt; exit 1; }
grep inf/s $O/vit_fold.txt
timeout -k 10 300 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 3 \
  --policy "default=" --policy "nowres=SPI_CONV_WRES=0" > $O/r18_wres.txt 2>&1 || { tail -30 $O/r18_wres.txt; exit 1; }
grep inf/s $O/r18_wres.txt
