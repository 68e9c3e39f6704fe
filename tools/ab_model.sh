#!/usr/bin/env bash
# Same-box A/B of two library builds on the four-stream model throughput: alternate
# processes (tools/policy_sweep.py) with SPI_HIP_LIB=A and B, `rounds` times each.
# usage: tools/ab_model.sh LIB_A LIB_B ROUNDS [policy_sweep args...]
set -euo pipefail
a=$1; b=$2; n=$3; shift 3
for i in $(seq 1 "$n"); do
  for lib in "$a" "$b"; do
    echo -n "$(basename "$lib") "
    SPI_HIP_LIB=$lib timeout -k 10 200 python tools/policy_sweep.py --rounds 1 "$@" 2>&1 | grep "inf/s"
  done
done
