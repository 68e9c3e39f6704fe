#!/bin/bash
# fp16m stem with hi + lo weights on the fp16 image: ResNet-18 parity + per-op + loop rate.
set -o pipefail
O=gpurun_out/r5/${1:-stem}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "resnet18 or stem" -s > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
grep -E "fp16m.*err=|fused vs unfused" $O/tests.txt
timeout -k 10 300 python -u tools/op_table.py --model resnet18 --precision fp16m --batch 8 > $O/ops_fp16m.txt 2>&1 || { tail -20 $O/ops_fp16m.txt; exit 1; }
grep -v amdgpu.ids $O/ops_fp16m.txt
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --loop-only --model resnet18 --batch 8 --precision fp16m --steps 20 --warmup 5 > $O/loop$i.json 2> $O/loop$i.err || { tail -20 $O/loop$i.err; exit 1; }
  cat $O/loop$i.json
done
