# Joint split-K plan for grouped pairs (SPI_GEMM_PAIR_JOINT): parity, per-op times, four-stream A/B, PMC traffic
set -euo pipefail
out=gpurun_out/pj; mkdir -p $out
SPI_GEMM_PAIR_JOINT=1 timeout -k 10 200 python -u -m pytest tests/test_parity_gpu.py tests/test_serving_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
SPI_GEMM_PAIR_JOINT=1 timeout -k 10 120 python3 tools/op_profile.py --model resnet18 --precision fp16m > $out/ops_joint.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 4 --policy base= --policy joint=SPI_GEMM_PAIR_JOINT=1 --policy joint_t128=SPI_GEMM_PAIR_JOINT=1\&SPI_GEMM_POLICY=tput:128 > $out/sweep.log 2>&1
SPI_GEMM_PAIR_JOINT=1 bash tools/pmc_traffic.sh $out/pmc_joint --model resnet18 --precision fp16m --batch 8 > $out/pmc.log 2>&1
