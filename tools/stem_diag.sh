# Fused-stem timing: tests, then stem_bench (normal and fill-only), then the four-stream A/B.
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_parity_gpu.py -k "stem" > gpurun_out/t_stem.log 2>&1 || { tail -30 gpurun_out/t_stem.log; exit 1; }
for d in 0 2; do echo "diag $d"; SPI_STEM_DIAG=$d timeout -k 10 60 python tools/stem_bench.py 2>&1 | grep rows || exit 1; done > gpurun_out/stem_diag.txt
timeout -k 10 300 python tools/policy_sweep.py --precision fp16m --rounds 3 --policy auto= --policy pr1=SPI_STEM_PR=1 --policy unfused=SPI_STEM_FUSED=0 > gpurun_out/sw_stem.txt 2>&1
