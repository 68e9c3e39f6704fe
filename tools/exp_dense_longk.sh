# BERT-base FFN2 (K = 3072) on fewer, larger tiles (SPI_GEMM_DENSE_LONGK_T): four-stream A/B
set -euo pipefail
out=gpurun_out/dlk; mkdir -p $out
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy base= --policy t96=SPI_GEMM_DENSE_LONGK_T=2048,96 --policy t48=SPI_GEMM_DENSE_LONGK_T=2048,48 > $out/bert.log 2>&1
