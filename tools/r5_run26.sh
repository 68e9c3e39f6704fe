#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-stemab}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 3 --policy base= \
  --policy unfused=SPI_STEM_FUSED=0 --policy halo128=SPI_GEMM_HALO_CFG=56:128,a > $O/r18.txt 2>&1 || { tail -30 $O/r18.txt; exit 1; }
grep -v amdgpu.ids $O/r18.txt | grep "inf/s"
