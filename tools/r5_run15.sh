#!/bin/bash
# Window kind with two K groups (SPI_GEMM_WIN=2 / 3): op + model parity, four-stream A/B,
# timed-loop traces per variant.
set -o pipefail
O=gpurun_out/r5/${1:-kg}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "window_kind or window_kgroups or resnet18_full_bs8" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 600 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 3 \
  --policy base= --policy w2=SPI_GEMM_WIN=2 --policy w3=SPI_GEMM_WIN=3 > $O/sweep_r18.txt 2>&1 || { tail -30 $O/sweep_r18.txt; exit 1; }
grep -v amdgpu.ids $O/sweep_r18.txt | tail -8
for w in 1 3 2; do
  SPI_GEMM_WIN=$w timeout -k 10 400 bash tools/trace_round.sh resnet18:8:fp16m > $O/trace_w$w.log 2>&1 || { tail -30 $O/trace_w$w.log; exit 1; }
  cp gpurun_out/trace/trace_resnet18_bs8_fp16m_ops.csv $O/trace_w${w}_ops.csv
done
head -5 $O/trace_w1_ops.csv $O/trace_w3_ops.csv $O/trace_w2_ops.csv
timeout -k 10 600 python -u tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 \
  --policy base= --policy w2=SPI_GEMM_WIN=2 --policy w3=SPI_GEMM_WIN=3 > $O/sweep_r152.txt 2>&1 || { tail -30 $O/sweep_r152.txt; exit 1; }
grep -v amdgpu.ids $O/sweep_r152.txt | tail -8
