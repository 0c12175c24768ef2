# C3 wave kernel: phase cycles (DG_WPROF build) + SQ instruction counters
set -o pipefail
T=${TAG:-r3b}
O=gpurun_out/$T
mkdir -p $O
ROOT=$(pwd)
DG_ALLOW_STALE=1 DG_LIB_PATH=$ROOT/dynamicgo_amd/libdgj2t_wprof.so timeout -k 10 200 python -u tools/wprof.py c3 > $O/wprof_c3.log 2>&1 || { tail -20 $O/wprof_c3.log; exit 1; }
tail -12 $O/wprof_c3.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH --kernel-trace --output-format csv -d $ROOT/$O/pmc1 -o run -- python3 $ROOT/bench.py --config c3 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/pmc1.log 2>&1 || { tail -5 $ROOT/$O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR --kernel-trace --output-format csv -d $ROOT/$O/pmc2 -o run -- python3 $ROOT/bench.py --config c3 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/pmc2.log 2>&1 || { tail -5 $ROOT/$O/pmc2.log; exit 1; }
cd $ROOT
for f in $(find $O/pmc1 $O/pmc2 -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r.get("Kernel_Name", "")
    if "wave" not in k: continue
    agg[k[:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("  %-24s max/dispatch %.5g" % (c, max(v)))
PY
done
echo done
