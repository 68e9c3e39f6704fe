set -e
mkdir -p gpurun_out/exp1
timeout -k 10 120 python3 tools/op_profile.py --model resnet18 --precision fp16m > gpurun_out/exp1/ops_base.log 2>&1
SPI_GEMM_PAIR=0 timeout -k 10 120 python3 tools/op_profile.py --model resnet18 --precision fp16m > gpurun_out/exp1/ops_pair0.log 2>&1
SPI_GEMM_MAXSPLIT=1 timeout -k 10 120 python3 tools/op_profile.py --model resnet18 --precision fp16m > gpurun_out/exp1/ops_split1.log 2>&1
timeout -k 10 300 python3 tools/policy_sweep.py --model resnet18 --precision fp16m --rounds 3 --policy base= --policy pair0=SPI_GEMM_PAIR=0 --policy split1=SPI_GEMM_MAXSPLIT=1 --policy split2=SPI_GEMM_MAXSPLIT=2 --policy st4=SPI_GEMM_STAGES=4 --policy t128=SPI_GEMM_POLICY=tput:128 > gpurun_out/exp1/sweep.log 2>&1
