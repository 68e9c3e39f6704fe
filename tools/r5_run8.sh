#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-i}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/loaded_ops.py --model resnet18 --precision fp16m > $O/r18_ops.txt 2>&1 || { tail -30 $O/r18_ops.txt; exit 1; }
cat $O/r18_ops.txt
timeout -k 10 300 python -u tools/loaded_ops.py --model vit_l_16 --precision fp16 --batch 16 > $O/vit_ops.txt 2>&1 || { tail -30 $O/vit_ops.txt; exit 1; }
cat $O/vit_ops.txt
timeout -k 10 300 python -u tools/loaded_ops.py --model bert_base --precision fp16 > $O/bert_ops.txt 2>&1 || { tail -30 $O/bert_ops.txt; exit 1; }
cat $O/bert_ops.txt
