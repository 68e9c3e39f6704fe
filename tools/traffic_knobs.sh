# Per-op PMC traffic of ResNet-18 bs8 fp16m under GEMM plan knobs (split-K off, plain XCD order)
set -e
for v in "SPI_GEMM_MAXSPLIT=1" "SPI_GEMM_XCD2D=0"; do
  name=$(echo "$v" | tr '=' '_')
  env $v bash tools/pmc_traffic.sh "gpurun_out/tk_$name" --model resnet18 --batch 8 --precision fp16m --iters 12 > "gpurun_out/tk_$name.txt" 2>&1
done
