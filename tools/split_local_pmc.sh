# HBM traffic per op (PMC) of ResNet-18 bs8 fp16m with the XCD-local split-K reduction on / off
set -euo pipefail
for L in 1 0; do
  SPI_GEMM_SPLIT_LOCAL=$L bash tools/pmc_traffic.sh gpurun_out/pmc_local$L --model resnet18 --precision fp16m --batch 8
done
