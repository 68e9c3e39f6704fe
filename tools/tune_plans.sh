# Sweep SPI_GEMM_PLAN="bm,bn,stages,splits" over layer shapes (tools/gemm_bench.py).
mkdir -p gpurun_out
run() { SPI_GEMM_PLAN="$1" timeout -k 10 120 python tools/gemm_bench.py --only "$2" --prec "${3:-fp16}" 2>/dev/null | grep -E "conv|gemm"; }
for sh in l1_3x3 stem; do for plan in "" "128,64,2,2" "128,64,3,2" "128,64,2,3"; do echo "== $sh [$plan]"; run "$plan" $sh; done; done
for sh in l2_3x3 l2_3x3s2; do for plan in "" "128,128,2,2" "128,128,2,4" "128,64,2,2" "128,64,3,4"; do echo "== $sh [$plan]"; run "$plan" $sh; done; done
for sh in l3_3x3 l4_3x3; do for plan in "" "128,128,2,4" "128,128,2,8" "128,128,2,12" "128,128,2,16" "128,64,3,8"; do echo "== $sh [$plan]"; run "$plan" $sh; done; done
for sh in bert_out bert_ff2 bert_qkv; do for plan in "" "128,128,2,2" "128,64,3,2" "64,64,3,2"; do echo "== $sh [$plan]"; run "$plan" $sh; done; done
