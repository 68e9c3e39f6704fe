# BERT-base bs8 GEMMs under forced plans (bm,bn,stages,splits), isolated, model epilogues
set -o pipefail
O=gpurun_out/${1:-bert_plans}; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_bench.py --model-epi --only bert --plans ';64,64,3,1;64,64,4,1;128,64,3,1;128,64,3,2;128,64,3,4;128,128,2,1;128,128,2,2;128,128,2,4;64,64,3,2' > $O/plans.log 2>&1
