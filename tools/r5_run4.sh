#!/bin/bash
# Round-5: BERT per-op times, fused vs unfused QKV + attention.
set -o pipefail
O=gpurun_out/r5/${1:-e}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/loaded_ops.py --model bert_base --precision fp16 > $O/ops_fused.txt 2>&1 || { tail -30 $O/ops_fused.txt; exit 1; }
cat $O/ops_fused.txt
SPI_QKV_ATTN=0 timeout -k 10 300 python -u tools/loaded_ops.py --model bert_base --precision fp16 > $O/ops_unfused.txt 2>&1 || { tail -30 $O/ops_unfused.txt; exit 1; }
cat $O/ops_unfused.txt
for w in 1 2 3 4; do
  timeout -k 10 200 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 2 --workers $w \
    --policy "w$w=" > $O/bert_w$w.txt 2>&1 || { tail -30 $O/bert_w$w.txt; exit 1; }
  grep "inf/s" $O/bert_w$w.txt
  timeout -k 10 200 python -u tools/policy_sweep.py --model resnet18 --batch 8 --precision fp16m --rounds 2 --workers $w \
    --policy "r18w$w=" > $O/r18_w$w.txt 2>&1 || { tail -30 $O/r18_w$w.txt; exit 1; }
  grep "inf/s" $O/r18_w$w.txt
done
