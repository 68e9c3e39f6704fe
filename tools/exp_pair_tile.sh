# GEMM phase stamps (diagnostic build) + the joint pair plan with 128x64 pair tiles (SPI_GEMM_PAIR_JOINT=2)
set -euo pipefail
out=gpurun_out/pt; mkdir -p $out
timeout -k 10 200 python3 tools/gemm_stamps.py tools/libspi_stamps.so > $out/stamps.log 2>&1
SPI_GEMM_PAIR_JOINT=2 timeout -k 10 200 python -u -m pytest tests/test_parity_gpu.py tests/test_serving_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
SPI_GEMM_PAIR_JOINT=2 timeout -k 10 120 python3 tools/op_profile.py --model resnet18 --precision fp16m > $out/ops_j2.log 2>&1
timeout -k 10 400 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 4 --policy j1= --policy j2=SPI_GEMM_PAIR_JOINT=2 --policy j2_t96=SPI_GEMM_PAIR_JOINT=2\&SPI_GEMM_POLICY=tput:96 --policy t96=SPI_GEMM_POLICY=tput:96 > $out/sweep.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 6 --policy j1= --policy j2=SPI_GEMM_PAIR_JOINT=2 > $out/r152.log 2>&1
