# flat kernel instruction-fetch counters (one --pmc pass each)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fl5}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
k=0
for ctrs in "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $O/pmc$k -o run -- python3 $GRAFT_REPO_ROOT/tools/fltime_n.py 65536 > $O/pmc$k.log 2>&1 || { tail -5 $O/pmc$k.log; exit 1; }
  f=$(find $O/pmc$k -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    kn = r["Kernel_Name"][:40]
    acc[kn][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(kn, r["Counter_Name"])] += 1
for kn, d in acc.items():
    print(kn, {c: round(v / cnt[(kn, c)]) for c, v in d.items()})
PY
done
echo done
