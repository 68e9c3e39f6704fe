# XCD-local split-K reduction A/B: parity of the split-K / conv / model tests with it on,
# isolated split-K layers, four-stream ResNet-18 fp16m / fp16x3 and ResNet-152 bs32.
set -o pipefail
O=gpurun_out/${1:-split_local}; mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py tests/test_serving_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 &&
$T 200 python -u tools/gemm_bench.py --only l3 --envs 'SPI_GEMM_SPLIT_LOCAL=1;SPI_GEMM_SPLIT_LOCAL=0' > $O/gb_l3.log 2>&1 &&
$T 200 python -u tools/gemm_bench.py --only l4 --envs 'SPI_GEMM_SPLIT_LOCAL=1;SPI_GEMM_SPLIT_LOCAL=0' > $O/gb_l4.log 2>&1 &&
$T 400 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 3 --policy local=SPI_GEMM_SPLIT_LOCAL=1 --policy wt=SPI_GEMM_SPLIT_LOCAL=0 > $O/r18_fp16m.log 2>&1 &&
$T 400 python -u tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --steps 6 --rounds 2 --policy local=SPI_GEMM_SPLIT_LOCAL=1 --policy wt=SPI_GEMM_SPLIT_LOCAL=0 > $O/r152.log 2>&1
