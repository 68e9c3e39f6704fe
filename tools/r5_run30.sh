#!/bin/bash
# ViT-L attention: 8-wave (default for S > 128) vs 4-wave workgroups, loop-only, interleaved processes.
set -o pipefail
O=gpurun_out/r5/${1:-attn4}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 env SPI_HIP_LIB=tools/libspi_attn4.so python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "vit" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do
  for v in base attn4; do
    lib=""; [ $v = attn4 ] && lib=tools/libspi_attn4.so
    SPI_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --loop-only --model vit_l_16 --batch 16 --precision fp16 --steps 10 --warmup 3 > $O/vit_${v}_$rep.json 2> $O/vit_${v}_$rep.err || { tail -20 $O/vit_${v}_$rep.err; exit 1; }
    echo "vit $v $rep $(python3 -c "import json;print(json.load(open('$O/vit_${v}_$rep.json'))['value'])")"
  done
done
