#!/bin/bash
# Throughput vs worker streams (loop only): is the four-stream load CU-bound or latency-bound?
set -o pipefail
O=gpurun_out/r5/${1:-streams}
mkdir -p $O
export PYTHONUNBUFFERED=1
for m in resnet18:8:fp16m bert_base:8:fp16 vit_l_16:16:fp16; do
  IFS=: read -r model batch prec <<< "$m"
  for w in 1 2 4 6 8; do
    timeout -k 10 200 python -u bench.py --loop-only --model $model --batch $batch --precision $prec --workers $w --steps 20 --warmup 5 > $O/${model}_w$w.json 2> $O/${model}_w$w.err || { tail -20 $O/${model}_w$w.err; exit 1; }
    echo "$model workers=$w $(cat $O/${model}_w$w.json)"
  done
done
