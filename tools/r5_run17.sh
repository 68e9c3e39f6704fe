#!/bin/bash
# Worker streams x HIP hardware queues (loop only): where the >4-stream collapse comes from.
set -o pipefail
O=gpurun_out/r5/${1:-queues}
mkdir -p $O
export PYTHONUNBUFFERED=1
for wq in 4:5 4:6 4:8 4:16 5:7 5:18 6:6 6:8 6:20 8:8 8:24; do
  IFS=: read -r w q <<< "$wq"
  timeout -k 10 200 python -u bench.py --loop-only --model resnet18 --batch 8 --precision fp16m --workers $w --hw-queues $q --steps 20 --warmup 5 > $O/w${w}_q$q.json 2> $O/w${w}_q$q.err || { tail -20 $O/w${w}_q$q.err; exit 1; }
  echo "workers=$w queues=$q $(cat $O/w${w}_q$q.json)"
done
