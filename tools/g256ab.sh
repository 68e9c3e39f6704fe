# gemm256 A/B on one GPU box: parity of the GEMM / transformer cases under each pipeline,
# isolated model-epilogue GEMM timings and four-stream C5 (ViT-L/16 bs16 fp16).
# usage: bash tools/g256ab.sh OUTDIR
set -o pipefail
O=gpurun_out/${1:-g256ab}; mkdir -p $O
T="timeout -k 10"
for P in 1 0; do
  SPI_G256_PIPE=$P $T 300 python -u -m pytest tests/test_ops_gpu.py -k "gemm256 or gemm_ or transformer or vit or bert" -x -q --timeout 120 --timeout-method thread > $O/tests_pipe$P.log 2>&1 || exit 1
done
$T 200 python -u tools/gemm_bench.py --model-epi --only vit --envs 'SPI_G256_PIPE=1;SPI_G256_PIPE=0' > $O/gb_vit.log 2>&1 &&
$T 200 python -u tools/gemm_bench.py --only sq4096 --envs 'SPI_G256_PIPE=1;SPI_G256_PIPE=0' > $O/gb_sq.log 2>&1 &&
$T 400 python -u tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --steps 10 --rounds 2 --policy pipe1=SPI_G256_PIPE=1 --policy pipe0=SPI_G256_PIPE=0 > $O/c5.log 2>&1
