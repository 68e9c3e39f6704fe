#!/bin/bash
set -o pipefail
O=gpurun_out/r5/${1:-o}
mkdir -p $O
export PYTHONUNBUFFERED=1
SPI_HIP_LIB=tools/libspi_g256tl.so timeout -k 10 300 python -u tools/g256_timeline.py > $O/g256_tl.txt 2>&1 || { tail -30 $O/g256_tl.txt; exit 1; }
grep -v amdgpu.ids $O/g256_tl.txt
