# 4-stage ring threshold (SPI_GEMM_ST4_MIN) across models, four streams
set -euo pipefail
out=gpurun_out/st4; mkdir -p $out
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy s32= --policy s24=SPI_GEMM_ST4_MIN=24 --policy s16=SPI_GEMM_ST4_MIN=16 > $out/bert.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 3 --policy s32= --policy s24=SPI_GEMM_ST4_MIN=24 --policy s16=SPI_GEMM_ST4_MIN=16 > $out/r18.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 6 --policy s32= --policy s24=SPI_GEMM_ST4_MIN=24 > $out/r152.log 2>&1
