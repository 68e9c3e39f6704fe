#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-k}
mkdir -p $O
export PYTHONUNBUFFERED=1
SPI_EXP_W128=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_parity_gpu.py -k "resnet18" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in "SPI_EXP_W128=" "SPI_EXP_W128=0" "SPI_EXP_W128=2" "SPI_EXP_W128=4" "SPI_EXP_W128=" "SPI_EXP_W128=0" "SPI_EXP_W128=2" "SPI_EXP_W128=4"; do
env $v timeout -k 10 200 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 2 \
  --policy "run=" > $O/r18.txt 2>&1 || { tail -30 $O/r18.txt; exit 1; }
echo "$v $(grep inf/s $O/r18.txt)"
done
for v in "SPI_EXP_ST4MIN=32" "SPI_EXP_ST4MIN=1000" "SPI_EXP_ST4MIN=32" "SPI_EXP_ST4MIN=1000"; do
env $v timeout -k 10 200 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 2 \
  --policy "run=" > $O/bert.txt 2>&1 || { tail -30 $O/bert.txt; exit 1; }
echo "$v $(grep inf/s $O/bert.txt)"
done
