#!/bin/bash
# Weight-resident 64->64 conv vs the window-kind implicit GEMM (SPI_CONV_WRES=0) across ResNet loads.
set -o pipefail
O=gpurun_out/r5/${1:-wres}
mkdir -p $O
export PYTHONUNBUFFERED=1
for m in resnet18:8:fp16m resnet18:8:fp16 resnet18:1:fp16m resnet152:32:fp16 resnet152:8:fp16; do
  IFS=: read -r model batch prec <<< "$m"
  timeout -k 10 600 python -u tools/policy_sweep.py --model $model --batch $batch --precision $prec --rounds 3 \
    --policy base= --policy nowres=SPI_CONV_WRES=0 > $O/sweep_${model}_bs${batch}_$prec.txt 2>&1 || { tail -30 $O/sweep_${model}_bs${batch}_$prec.txt; exit 1; }
  echo "== $m"; grep -v amdgpu.ids $O/sweep_${model}_bs${batch}_$prec.txt | tail -2
done
