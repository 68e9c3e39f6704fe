#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-host}
mkdir -p $O
export PYTHONUNBUFFERED=1
for m in resnet18:8:fp16m bert_base:8:fp16; do
  IFS=: read -r model batch prec <<< "$m"
  timeout -k 10 300 python -u tools/host_enqueue_probe.py --model $model --batch $batch --precision $prec > $O/$model.txt 2>&1 || { tail -20 $O/$model.txt; exit 1; }
  grep -v amdgpu.ids $O/$model.txt
done
