#!/bin/bash
# Re-validate older plan decisions for C3 / C4 / C5 on the round-5 kernels (four streams, one process per model).
set -o pipefail
O=gpurun_out/r5/${1:-revalidate}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {
  local tag=$1; shift
  timeout -k 10 900 python -u tools/policy_sweep.py "$@" > $O/$tag.txt 2>&1 || { tail -30 $O/$tag.txt; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids $O/$tag.txt | grep "inf/s"
}
run vit --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --policy base= --policy longk0=SPI_GEMM_256_LONGK=0 \
  --policy g128=SPI_GEMM_256_MIN=128,64 --policy g128b2=SPI_GEMM_256_MIN=128,64,2
run r152 --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --policy base= --policy win0=SPI_GEMM_WIN=0 \
  --policy halo0=SPI_GEMM_HALO_CFG=0 --policy split1=SPI_GEMM_MAXSPLIT=1
run bert --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy g128=SPI_GEMM_256_MIN=128,64 \
  --policy longk0=SPI_GEMM_256_LONGK=0
