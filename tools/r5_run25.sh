#!/bin/bash
# ViT-L: gemm256 routing of the wide GEMMs (QKV 156 / FFN1 208 tiles) re-measured on the round-5 kernels.
set -o pipefail
O=gpurun_out/r5/${1:-vit256}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --policy base= \
  --policy min0=SPI_GEMM_256_MIN=0 --policy min200=SPI_GEMM_256_MIN=200 --policy min160=SPI_GEMM_256_MIN=160 > $O/vit.txt 2>&1 || { tail -30 $O/vit.txt; exit 1; }
grep -v amdgpu.ids $O/vit.txt | grep "inf/s"
timeout -k 10 900 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 3 --policy base= \
  --policy split2=SPI_GEMM_MAXSPLIT=2 --policy split1=SPI_GEMM_MAXSPLIT=1 > $O/r18.txt 2>&1 || { tail -30 $O/r18.txt; exit 1; }
grep -v amdgpu.ids $O/r18.txt | grep "inf/s"
