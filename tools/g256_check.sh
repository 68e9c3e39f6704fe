# gemm256: parity tests, then transformer-shape timings under each schedule and with it off,
# then the ViT-L bs16 four-stream A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm256 or gemm_bias" > gpurun_out/t_g256.log 2>&1 || { tail -30 gpurun_out/t_g256.log; exit 1; }
SPI_G256_SCHED=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "gemm256" >> gpurun_out/t_g256.log 2>&1 || { tail -30 gpurun_out/t_g256.log; exit 1; }
for v in "SPI_G256_SCHED=1" "SPI_G256_SCHED=0" "SPI_GEMM_256_MIN=0"; do echo "$v"; env $v timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -E "vit|sq" || exit 1; done > gpurun_out/gb_256.txt
timeout -k 10 400 python tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 --steps 4 --policy base= --policy old=SPI_GEMM_256_MIN=0 > gpurun_out/sw_vit256.txt 2>&1
