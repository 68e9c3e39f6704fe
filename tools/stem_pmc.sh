#!/usr/bin/env bash
# PMC passes over the fused stem (tools/stem_bench.py, one precision / rows config), one
# rocprofv3 run per counter group, counters only; prints per-counter means over its dispatches.
# usage: tools/stem_pmc.sh OUTDIR [fp16m:1]
set -euo pipefail
out=$1; only=${2:-fp16m:1}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU"
)
i=0
for g in "${groups[@]}"; do
  STEM_ONLY=$only timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$out/p$i" -- \
    python3 tools/stem_bench.py > "$out/p$i.log" 2>&1
  i=$((i+1))
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "stem_pool" in row.get("Kernel_Name", ""):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:32s} mean {sum(v) / len(v):16.1f}  ({len(v)} records)")
PY
