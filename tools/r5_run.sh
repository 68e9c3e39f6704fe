#!/bin/bash
# Round-5 GPU session helper: gemm256 128-row tiles -- op tests, isolated shapes, four-stream models.
set -o pipefail
O=gpurun_out/r5/${1:-a}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm256" \
  tests/test_parity_gpu.py::test_transformer_layernorm_fold_on_gemm256 tests/test_parity_gpu.py::test_transformer_layernorm_fold \
  "tests/test_parity_gpu.py::test_bert_base_seq128_bs8" tests/test_runtime_gpu.py -s > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -E "LN fold|bert-base|p50 coal|passed|failed" $O/tests.txt
timeout -k 10 200 python -u tools/gemm_bench.py --model-epi --only "t_" --reps 50 \
  --envs "SPI_GEMM_256_MIN=128,0;SPI_GEMM_256_MIN=128,1,3;SPI_GEMM_256_MIN=128,1,2;SPI_GEMM_256_MIN=1,0" > $O/gemm.txt 2>&1 || { tail -30 $O/gemm.txt; exit 1; }
grep gemm $O/gemm.txt
timeout -k 10 300 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 \
  --policy "old=SPI_GEMM_256_MIN=128,0" --policy "b3=SPI_GEMM_256_MIN=128,64,3" --policy "b2=SPI_GEMM_256_MIN=128,64,2" \
  --policy "g256=SPI_GEMM_256_MIN=36,0" > $O/bert.txt 2>&1 || { tail -30 $O/bert.txt; exit 1; }
cat $O/bert.txt
timeout -k 10 400 python -u tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 \
  --policy "old=SPI_GEMM_256_MIN=128,0" --policy "b3=SPI_GEMM_256_MIN=128,64,3" --policy "b2=SPI_GEMM_256_MIN=128,64,2" > $O/vit.txt 2>&1 || { tail -30 $O/vit.txt; exit 1; }
cat $O/vit.txt
timeout -k 10 300 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16m --rounds 2 \
  --policy "fp16m=" > $O/bert_f16m.txt 2>&1 || { tail -30 $O/bert_f16m.txt; exit 1; }
cat $O/bert_f16m.txt
