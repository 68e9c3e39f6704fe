#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-bertplan}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= \
  --policy p128x64=SPI_GEMM_PLAN=128,64,3,1 --policy p128x128=SPI_GEMM_PLAN=128,128,2,1 --policy p64=SPI_GEMM_PLAN=64,64,4,1 > $O/bert.txt 2>&1 || { tail -30 $O/bert.txt; exit 1; }
grep -v amdgpu.ids $O/bert.txt | grep "inf/s"
