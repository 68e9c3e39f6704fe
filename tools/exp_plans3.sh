# Plan knobs after the joint pair plan: ring depth (SPI_GEMM_ST4_MIN), no 128x128 tiles (SPI_GEMM_NO128SQ),
# halo kinds on the 28 / 14-wide maps (SPI_GEMM_HALO_CFG) -- four-stream throughput, same process per model
set -euo pipefail
out=gpurun_out/p3; mkdir -p $out
timeout -k 10 300 python3 tools/gemm_bench.py --model-epi --only bert --envs ";SPI_GEMM_ST4_MIN=32;SPI_GEMM_NO128SQ=1;SPI_GEMM_NO128SQ=1&SPI_GEMM_ST4_MIN=32" > $out/gb_bert.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy st4_32=SPI_GEMM_ST4_MIN=32 --policy nosq=SPI_GEMM_NO128SQ=1 --policy nosq_st4=SPI_GEMM_NO128SQ=1\&SPI_GEMM_ST4_MIN=32 --policy st3_8=SPI_GEMM_ST3_MIN=8 > $out/bert.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 3 --policy base= --policy halo28_14=SPI_GEMM_HALO_CFG=28:64,a\;14:64,a\;0:0 --policy halo14=SPI_GEMM_HALO_CFG=14:64,a\;0:0 --policy halo28=SPI_GEMM_HALO_CFG=28:64,a\;0:0 --policy st3_8=SPI_GEMM_ST3_MIN=8 > $out/r18.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 6 --policy base= --policy st4_32=SPI_GEMM_ST4_MIN=32 --policy nosq=SPI_GEMM_NO128SQ=1 > $out/vit.log 2>&1
