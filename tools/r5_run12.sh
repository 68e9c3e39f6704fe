#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-m}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u tools/loaded_ops.py --model resnet152 --precision fp16x3 --batch 32 > $O/r152_ops.txt 2>&1 || { tail -30 $O/r152_ops.txt; exit 1; }
cat $O/r152_ops.txt
