#!/bin/bash
# gemm256 fp16-park epilogue: op + ViT parity, per-launch timeline, ViT loop rate vs the previous build.
set -o pipefail
O=gpurun_out/r5/${1:-epi16}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm256 or vit or layernorm_fold" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
SPI_HIP_LIB=tools/libspi_g256tl.so timeout -k 10 300 python -u tools/g256_timeline.py > $O/g256_tl.txt 2>&1 || { tail -30 $O/g256_tl.txt; exit 1; }
grep -v amdgpu.ids $O/g256_tl.txt
for rep in 1 2; do
  for v in new old; do
    lib=""; [ $v = old ] && lib=tools/libspi_ab_old.so
    SPI_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --loop-only --model vit_l_16 --batch 16 --precision fp16 --steps 10 --warmup 3 > $O/vit_${v}_$rep.json 2> $O/vit_${v}_$rep.err || { tail -20 $O/vit_${v}_$rep.err; exit 1; }
    echo "vit $v $rep $(python3 -c "import json;print(json.load(open('$O/vit_${v}_$rep.json'))['value'])")"
  done
done
