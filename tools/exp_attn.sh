# Swapped-orientation fp16 attention (SPI_ATTN_SWAP=1, P in registers, V by ds_read_b64_tr_b16) vs round 2
set -euo pipefail
out=gpurun_out/attn; mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -k "attention or layernorm" -x -q --timeout 120 --timeout-method thread > $out/ops_tests.log 2>&1
timeout -k 10 250 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_torchscript_gpu.py -x -q --timeout 120 --timeout-method thread > $out/model_tests.log 2>&1
SPI_ATTN_SWAP=0 timeout -k 10 200 python3 tools/loaded_ops.py --model bert_base --precision fp16 > $out/bert_ops_old.log 2>&1
timeout -k 10 200 python3 tools/loaded_ops.py --model bert_base --precision fp16 > $out/bert_ops_new.log 2>&1
SPI_ATTN_SWAP=0 timeout -k 10 200 python3 tools/loaded_ops.py --model vit_l_16 --precision fp16 --batch 16 > $out/vit_ops_old.log 2>&1
timeout -k 10 200 python3 tools/loaded_ops.py --model vit_l_16 --precision fp16 --batch 16 > $out/vit_ops_new.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 --policy old=SPI_ATTN_SWAP=0 --policy new=SPI_ATTN_SWAP=1 > $out/bert.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 6 --policy old=SPI_ATTN_SWAP=0 --policy new=SPI_ATTN_SWAP=1 > $out/vit.log 2>&1
