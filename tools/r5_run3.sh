#!/bin/bash
# Round-5: fused QKV + attention (BERT) -- tests, loaded ops, four-stream A/B.
set -o pipefail
O=gpurun_out/r5/${1:-d}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_parity_gpu.py -k "qkv_attention_fused or bert or layernorm_fold" -s > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "fused S|LN fold|bert|passed|failed" $O/tests.txt
timeout -k 10 300 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 \
  --policy "unfused=SPI_QKV_ATTN=0" --policy "fused=" > $O/bert.txt 2>&1 || { tail -30 $O/bert.txt; exit 1; }
cat $O/bert.txt
