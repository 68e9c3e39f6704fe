#!/bin/bash
# wres auto rule: parity (ResNet + wres op tests) and A/B against the old rule (SPI_CONV_WRES=2).
set -o pipefail
O=gpurun_out/r5/${1:-wres2}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resnet or weight_resident or window_kind" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for m in resnet18:8:fp16m resnet18:1:fp16m; do
  IFS=: read -r model batch prec <<< "$m"
  timeout -k 10 600 python -u tools/policy_sweep.py --model $model --batch $batch --precision $prec --rounds 3 \
    --policy auto= --policy always=SPI_CONV_WRES=2 > $O/sweep_${model}_bs${batch}.txt 2>&1 || { tail -30 $O/sweep_${model}_bs${batch}.txt; exit 1; }
  echo "== $m"; grep -v amdgpu.ids $O/sweep_${model}_bs${batch}.txt | tail -2
done
