#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-n}
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
for v in "SPI_STEM_PR_EXP=0" "SPI_STEM_PR_EXP=1" "SPI_STEM_PR_EXP=2" "SPI_STEM_FUSED=0"; do
env $v timeout -k 10 300 python -u tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 8 \
  --policy "run=" > $O/r152.txt 2>&1 || { tail -30 $O/r152.txt; exit 1; }
echo "$v $(grep inf/s $O/r152.txt)"
done
done
