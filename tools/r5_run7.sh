#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-h}
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in "SPI_STEM_PR_EXP=0" "SPI_STEM_PR_EXP=1" "SPI_STEM_PR_EXP=2" "SPI_STEM_PR_EXP=0" "SPI_STEM_PR_EXP=1" "SPI_STEM_PR_EXP=2"; do
env $v timeout -k 10 200 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 2 \
  --policy "$v=" > $O/r18.txt 2>&1 || { tail -30 $O/r18.txt; exit 1; }
grep inf/s $O/r18.txt
done
