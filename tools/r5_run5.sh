#!/bin/bash
# Round-5: fused QKV + attention ring depth A/B.
set -o pipefail
O=gpurun_out/r5/${1:-f}
mkdir -p $O
export PYTHONUNBUFFERED=1
for st in 3 2; do
SPI_QKV_STG=$st timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_parity_gpu.py -k "qkv_attention_fused or bert_base" -s > $O/tests$st.txt 2>&1 || { tail -40 $O/tests$st.txt; exit 1; }
grep -E "fused S|bert|passed|failed" $O/tests$st.txt
done
for v in "SPI_QKV_ATTN=0" "SPI_QKV_STG=3" "SPI_QKV_STG=2" "SPI_QKV_ATTN=0" "SPI_QKV_STG=3" "SPI_QKV_STG=2"; do
env $v timeout -k 10 200 python -u tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 2 \
  --policy "$v=" > $O/bert.txt 2>&1 || { tail -30 $O/bert.txt; exit 1; }
grep inf/s $O/bert.txt
done
