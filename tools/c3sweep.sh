set -o pipefail
O=gpurun_out/c3sweep; mkdir -p $O
timeout -k 10 500 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --steps 20 --rounds 2 --policy base= --policy g256_32=SPI_GEMM_256_MIN=32 --policy g256_12=SPI_GEMM_256_MIN=12 > $O/c3.log 2>&1 &&
timeout -k 10 200 python -u tools/gemm_bench.py --model-epi --epi-variants --only bert --envs 'SPI_GEMM_256_MIN=128;SPI_GEMM_256_MIN=12' > $O/gb_bert.log 2>&1
