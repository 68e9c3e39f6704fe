# 128x64 split-K plans (SPI_GEMM_SPLIT128=1) and the 4-stage rule (SPI_GEMM_ST4_MIN) -- parity, isolated layers, four streams
set -euo pipefail
out=gpurun_out/s128; mkdir -p $out
SPI_GEMM_SPLIT128=1 timeout -k 10 250 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py tests/test_serving_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python3 tools/gemm_bench.py --model-epi --envs ";SPI_GEMM_SPLIT128=1" > $out/gb.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 3 --policy base= --policy s128=SPI_GEMM_SPLIT128=1 > $out/r18.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy s128=SPI_GEMM_SPLIT128=1 --policy st4off=SPI_GEMM_ST4_MIN=1000000 > $out/bert.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 6 --policy base= --policy s128=SPI_GEMM_SPLIT128=1 --policy st4off=SPI_GEMM_ST4_MIN=1000000 > $out/r152.log 2>&1
