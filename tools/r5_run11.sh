#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-l}
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
for v in "SPI_EXP_SPLIT4=3" "SPI_EXP_SPLIT4=2" "SPI_EXP_SPLIT4=4" "SPI_EXP_SPLIT4=6" "SPI_EXP_SPLIT3=3" "SPI_EXP_SPLIT3=4" "SPI_EXP_SPLIT2=2"; do
env $v timeout -k 10 200 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 2 \
  --policy "run=" > $O/r18.txt 2>&1 || { tail -30 $O/r18.txt; exit 1; }
echo "$v $(grep inf/s $O/r18.txt)"
done
done
