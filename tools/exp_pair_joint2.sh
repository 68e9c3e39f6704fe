# Joint pair plan + plan target T across the four configs (four-stream throughput, same process per model)
set -euo pipefail
out=gpurun_out/pj2; mkdir -p $out
P="--policy base= --policy joint=SPI_GEMM_PAIR_JOINT=1 --policy joint_t128=SPI_GEMM_PAIR_JOINT=1&SPI_GEMM_POLICY=tput:128 --policy joint_t160=SPI_GEMM_PAIR_JOINT=1&SPI_GEMM_POLICY=tput:160 --policy joint_s3=SPI_GEMM_PAIR_JOINT=1&SPI_GEMM_MAXSPLIT=3"
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 4 $P > $out/r18.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet152 --batch 32 --precision fp16x3 --rounds 2 --steps 6 $P > $out/r152.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model bert_base --batch 8 --precision fp16 --rounds 3 $P > $out/bert.log 2>&1
