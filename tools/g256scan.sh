# gemm256 fixed cost vs k-loop: ViT-L FFN1's 3152 x 4096 over K, both pipelines; GELU cost.
set -o pipefail
O=gpurun_out/${1:-g256scan}; mkdir -p $O
T="timeout -k 10"
$T 200 python -u tools/gemm_bench.py --kscan 3152x4096 --envs 'SPI_G256_PIPE=1;SPI_G256_PIPE=0' > $O/kscan.log 2>&1 &&
$T 200 python -u tools/gemm_bench.py --kscan 4096x4096 --envs 'SPI_G256_PIPE=1' > $O/kscan_sq.log 2>&1 &&
$T 200 python -u tools/gemm_bench.py --model-epi --epi-variants --only vit_ff1 --envs 'SPI_G256_PIPE=1;SPI_G256_PIPE=0' > $O/gelu.log 2>&1
