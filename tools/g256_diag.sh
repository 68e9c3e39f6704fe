# gemm256 diagnostic variants on the transformer shapes: normal, L2-resident operands, no DMA in the loop
mkdir -p gpurun_out
for d in 0 1 2; do echo "diag $d"; SPI_G256_DIAG=$d timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -E "vit|sq" || exit 1; done > gpurun_out/g256_diag.txt
