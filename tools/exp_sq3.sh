# 3-stage ring for dense fp16 128x128 tiles (SPI_GEMM_SQ_STAGES=3): isolated GEMMs, parity, four streams
set -euo pipefail
out=gpurun_out/sq3; mkdir -p $out
timeout -k 10 300 python3 tools/gemm_bench.py --model-epi --only vit --envs ";SPI_GEMM_SQ_STAGES=3" > $out/gb_vit.log 2>&1
timeout -k 10 300 python3 tools/gemm_bench.py --model-epi --only bert --envs ";SPI_GEMM_SQ_STAGES=3" > $out/gb_bert.log 2>&1
SPI_GEMM_SQ_STAGES=3 timeout -k 10 250 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 6 --policy base= --policy sq3=SPI_GEMM_SQ_STAGES=3 > $out/vit.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy sq3=SPI_GEMM_SQ_STAGES=3 > $out/bert.log 2>&1
timeout -k 10 200 python3 tools/loaded_ops.py --model bert_base --precision fp16 > $out/bert_ops.log 2>&1
