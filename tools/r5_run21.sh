#!/bin/bash
# Per-op isolated / loaded tables for C3 and C5.
set -o pipefail
O=gpurun_out/r5/${1:-optab}
mkdir -p $O
export PYTHONUNBUFFERED=1
for m in bert_base:8:fp16 vit_l_16:16:fp16; do
  IFS=: read -r model batch prec <<< "$m"
  timeout -k 10 400 python -u tools/op_table.py --model $model --precision $prec --batch $batch > $O/ops_$model.txt 2>&1 || { tail -20 $O/ops_$model.txt; exit 1; }
  grep -v amdgpu.ids $O/ops_$model.txt
done
timeout -k 10 600 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 3 \
  --policy base= --policy nowres=SPI_CONV_WRES=0 > $O/sweep_wres.txt 2>&1 || { tail -30 $O/sweep_wres.txt; exit 1; }
grep -v amdgpu.ids $O/sweep_wres.txt | tail -4
