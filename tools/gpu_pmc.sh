#!/bin/bash
# GPU-box script: PMC counter passes (kernel-trace only; no sys/runtime trace).
# usage: bash tools/gpu_pmc.sh <tag> "<counters pass1>" ["<counters pass2>" ...] -- [bench args]
set -o pipefail
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do PASSES+=("$1"); shift; done
[ "$1" == "--" ] && shift
i=0
for C in "${PASSES[@]}"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- python3 $ROOT/bench.py --no-cpu-baseline "$@" > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -20 $OUT/pmc$i.log; exit 1; }
done
for f in $(find $OUT -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r.get("Kernel_Name", "")
    if "j2t" not in k: continue
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k[:60])
    for c, v in sorted(d.items()):
        print("  %-28s mean/dispatch %.4g  (n=%d)" % (c, sum(v)/len(v), len(v)))
PY
done
