#!/bin/bash
# fp16 vs fp16m ResNet-18 per-op cost (isolated and under the four-stream load).
set -o pipefail
O=gpurun_out/r5/${1:-f16m}
mkdir -p $O
export PYTHONUNBUFFERED=1
for p in fp16 fp16m; do
  timeout -k 10 300 python -u tools/op_table.py --model resnet18 --precision $p --batch 8 > $O/ops_$p.txt 2>&1 || { tail -20 $O/ops_$p.txt; exit 1; }
  grep -v amdgpu.ids $O/ops_$p.txt
done
