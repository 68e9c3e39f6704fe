#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-vitsplit}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --policy base= \
  --policy split2=SPI_GEMM_256_LONGK=48,1024,2 --policy split2k2048=SPI_GEMM_256_LONGK=48,2048,2 > $O/vit.txt 2>&1 || { tail -30 $O/vit.txt; exit 1; }
grep -v amdgpu.ids $O/vit.txt | grep "inf/s"
