#!/bin/bash
# Round-5: the tests r5_run.sh b deselected, ViT 128-row routing by K, a default bench line.
set -o pipefail
O=gpurun_out/r5/${1:-c}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_parity_gpu.py::test_transformer_layernorm_fold "tests/test_parity_gpu.py::test_bert_base_seq128_bs8" \
  tests/test_runtime_gpu.py -s > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
grep -E "LN fold|bert-base|p50 coal|passed|failed" $O/tests.txt
timeout -k 10 400 python -u tools/policy_sweep.py --model vit_l_16 --batch 16 --precision fp16 --rounds 2 \
  --policy "old=SPI_GEMM_256_MIN=128,0" --policy "outproj128=SPI_GEMM_256_MIN=128,64,3,0,1024" --policy "both128=SPI_GEMM_256_MIN=128,64,3" \
  --policy "ffn2_128=SPI_GEMM_256_MIN=128,64,3,2048" > $O/vit.txt 2>&1 || { tail -30 $O/vit.txt; exit 1; }
cat $O/vit.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d.get('e2e_summary'))
for k,v in d.get('extras',{}).items():
    if isinstance(v,dict) and 'value' in v: print(k, v.get('value'), v.get('p50_latency_ms'))
ci=d.get('extras',{}).get('ci_perf_resnet152_schedule',{})
print('ci', ci.get('value'), ci.get('p50_latency_ms'), ci.get('p50_queue_ms'), 'tuned', ci.get('mi355x_tuned',{}).get('value'), ci.get('mi355x_tuned',{}).get('p50_latency_ms'), ci.get('mi355x_tuned',{}).get('rejected'))
"
