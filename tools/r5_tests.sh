#!/bin/bash
# The GPU suite + smoke on the committed tree (no bench).
set -o pipefail
O=gpurun_out/r5/${1:-tests}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 200 python -u bench.py --loop-only --model resnet18 --batch 8 --precision fp16m --steps 20 --warmup 5 > $O/loop.json 2> $O/loop.err && cat $O/loop.json
