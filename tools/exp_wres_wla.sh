# Weight-resident conv: weights streamed 3 taps ahead (SPI_CONV_WRES_WLA=3) vs all up front
set -euo pipefail
out=gpurun_out/wla; mkdir -p $out
SPI_CONV_WRES_WLA=3 timeout -k 10 250 python -u -m pytest tests/test_ops_gpu.py -k weight_resident tests/test_parity_gpu.py tests/test_serving_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python3 tools/gemm_bench.py --only l1_3x3 --envs ";SPI_CONV_WRES_WLA=3;;SPI_CONV_WRES_WLA=3" > $out/gb.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 4 --policy base= --policy wla3=SPI_CONV_WRES_WLA=3 > $out/r18.log 2>&1
