# gemm256 long-K rule (SPI_GEMM_256_LONGK, default 48,1024) vs off; PMC traffic of the headline after the round's plan changes
set -euo pipefail
out=gpurun_out/longk; mkdir -p $out
timeout -k 10 300 python3 tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 6 --policy longk= --policy off=SPI_GEMM_256_LONGK=0 > $out/vit.log 2>&1
bash tools/profile_round.sh resnet18:8:fp16m > $out/pmc.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy a8=SPI_ATTN_SWAP=2 > $out/bert.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 6 --policy base= --policy t96=SPI_GEMM_POLICY=tput:96 --policy t64=SPI_GEMM_POLICY=tput:64 > $out/r152.log 2>&1
