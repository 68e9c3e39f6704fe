#!/bin/bash
# Ring depth threshold (3 stages from 8 / 12 / 16 k-steps): loop-only rates, separate processes, interleaved.
set -o pipefail
O=gpurun_out/r5/${1:-st3}
mkdir -p $O
export PYTHONUNBUFFERED=1
for m in resnet18:8:fp16m bert_base:8:fp16 resnet152:32:fp16x3; do
  IFS=: read -r model batch prec <<< "$m"
  for rep in 1 2; do
    for v in base st3_8 st3_12; do
      lib=""; [ $v != base ] && lib=tools/libspi_$v.so
      SPI_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --loop-only --model $model --batch $batch --precision $prec --steps 20 --warmup 5 > $O/${model}_${v}_$rep.json 2> $O/${model}_${v}_$rep.err || { tail -20 $O/${model}_${v}_$rep.err; exit 1; }
      echo "$model $v $rep $(python3 -c "import json;print(json.load(open('$O/${model}_${v}_$rep.json'))['value'])")"
    done
  done
done
