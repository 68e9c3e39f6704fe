#!/bin/bash
# Round-5 checkpoint on one box: the whole GPU suite, smoke, the default bench line.
set -o pipefail
O=gpurun_out/r5/${1:-full}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('C2', d['value'], 'frac', d['roofline'].get('frac'), d['roofline'].get('kernel'), 'e2e', d.get('e2e_summary'))
for k,v in d.get('extras',{}).items():
    if isinstance(v,dict) and 'value' in v: print(k, v.get('value'), v.get('p50_latency_ms'))
ci=d.get('extras',{}).get('ci_perf_resnet152_schedule',{})
print('ci tuned', ci.get('mi355x_tuned',{}).get('value'), ci.get('mi355x_tuned',{}).get('p50_latency_ms'))
"
