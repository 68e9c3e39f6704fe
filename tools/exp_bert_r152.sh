# BERT-base with 8-wave attention workgroups (SPI_ATTN_SWAP=2); ResNet-152 bs32 under smaller plan targets
set -euo pipefail
out=gpurun_out/br; mkdir -p $out
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy a8=SPI_ATTN_SWAP=2 > $out/bert.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 6 --policy base= --policy t96=SPI_GEMM_POLICY=tput:96 --policy t64=SPI_GEMM_POLICY=tput:64 > $out/r152.log 2>&1
