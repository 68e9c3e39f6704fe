# Weight-resident conv: several bands per workgroup on one halo buffer (SPI_CONV_WRES_NBUF=1, BPW=2/3)
set -euo pipefail
out=gpurun_out/wmb; mkdir -p $out
SPI_CONV_WRES_NBUF=1 SPI_CONV_WRES_BPW=2 timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -k weight_resident -x -q --timeout 120 --timeout-method thread > $out/tests_bpw2.log 2>&1
SPI_CONV_WRES_NBUF=1 SPI_CONV_WRES_BPW=3 timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -k weight_resident -x -q --timeout 120 --timeout-method thread > $out/tests_bpw3.log 2>&1
timeout -k 10 200 python3 tools/gemm_bench.py --only l1_3x3 --envs ";SPI_CONV_WRES_NBUF=1&SPI_CONV_WRES_BPW=2;SPI_CONV_WRES_NBUF=1&SPI_CONV_WRES_BPW=3" > $out/gb.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 4 --policy base= --policy b2=SPI_CONV_WRES_NBUF=1\&SPI_CONV_WRES_BPW=2 --policy b3=SPI_CONV_WRES_NBUF=1\&SPI_CONV_WRES_BPW=3 > $out/r18.log 2>&1
