#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-j}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/gemm_bench.py --kscan 3152x4096 --reps 30 > $O/kscan_4096.txt 2>&1 || { tail -30 $O/kscan_4096.txt; exit 1; }
grep kscan $O/kscan_4096.txt
timeout -k 10 300 python -u tools/gemm_bench.py --kscan 3152x1024 --reps 30 > $O/kscan_1024.txt 2>&1 || { tail -30 $O/kscan_1024.txt; exit 1; }
grep kscan $O/kscan_1024.txt
