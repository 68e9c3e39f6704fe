# gemm256 for smaller grids (SPI_GEMM_256_MIN): fewer CUs per GEMM at ~1.7x the per-CU rate -- four-stream A/B
set -euo pipefail
out=gpurun_out/g256min; mkdir -p $out
timeout -k 10 300 python3 tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 6 --policy base= --policy m48=SPI_GEMM_256_MIN=48 --policy m32=SPI_GEMM_256_MIN=32 > $out/vit.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy m48=SPI_GEMM_256_MIN=48 --policy m32=SPI_GEMM_256_MIN=32 --policy m24=SPI_GEMM_256_MIN=24 > $out/bert.log 2>&1
timeout -k 10 200 python3 tools/gemm_bench.py --model-epi --only vit --envs ";SPI_GEMM_256_MIN=48" > $out/gb_vit.log 2>&1
SPI_ATTN_SWAP=3 timeout -k 10 200 python3 tools/loaded_ops.py --model vit_l_16 --precision fp16 --batch 16 > $out/vit_ops_attn4w.log 2>&1
timeout -k 10 200 python3 tools/loaded_ops.py --model vit_l_16 --precision fp16 --batch 16 > $out/vit_ops_attn8w.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 6 --policy a4=SPI_ATTN_SWAP=3 --policy a8=SPI_ATTN_SWAP=1 > $out/vit_attn.log 2>&1
