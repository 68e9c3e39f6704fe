#!/bin/bash
# fp16m FC on plain fp16 weights (variant): ResNet-18 parity (printed errors) + C2 loop rate.
set -o pipefail
O=gpurun_out/r5/${1:-fc16}
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in fc16; do
  timeout -k 10 300 env SPI_HIP_LIB=tools/libspi_$v.so python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k "resnet18" > $O/tests_$v.txt 2>&1 || { tail -30 $O/tests_$v.txt; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.txt)"; grep -E "fp16m.*err=" $O/tests_$v.txt
done
for rep in 1 2 3; do
  for v in base fc16; do
    lib=""; [ $v != base ] && lib=tools/libspi_$v.so
    SPI_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --loop-only --model resnet18 --batch 8 --precision fp16m --steps 20 --warmup 5 > $O/r18_${v}_$rep.json 2> $O/r18_${v}_$rep.err || { tail -20 $O/r18_${v}_$rep.err; exit 1; }
    echo "r18 $v $rep $(python3 -c "import json;print(json.load(open('$O/r18_${v}_$rep.json'))['value'])")"
  done
done
