mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_parity_gpu.py tests/test_fullsize_gpu.py -k "attention or bert or vit" > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
bash tools/ab_model.sh tools/libspi_ab_base.so starpu-inference-server_amd/libspi_hip.so 3 --model bert_base --precision fp16 --steps 10 > gpurun_out/ab_attn.txt 2>&1
bash tools/ab_model.sh tools/libspi_ab_base.so starpu-inference-server_amd/libspi_hip.so 2 --model vit_l_16 --batch 16 --precision fp16 --steps 4 >> gpurun_out/ab_attn.txt 2>&1
