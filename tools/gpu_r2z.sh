set -o pipefail
export DG_FLAT=1 DG_ALLOW_STALE=1
ROOT=$(pwd)
cd /tmp
for v in "" _stop1 _stop2; do
timeout -s KILL 90 env DG_LIB_PATH=$ROOT/dynamicgo_amd/libdgj2t$v.so rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d $ROOT/gpurun_out/r2z$v -o run -- python3 $ROOT/tools/fltime.py c2 > $ROOT/gpurun_out/r2z$v.log 2>&1 || { tail -5 $ROOT/gpurun_out/r2z$v.log; exit 1; }
python3 - $ROOT/gpurun_out/r2z$v/run_counter_collection.csv "$v" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if "flat" not in r["Kernel_Name"]: continue
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2] or "full", " ".join("%s=%.4g" % (c[3:], sum(v)/len(v)) for c, v in sorted(agg.items())))
PY
done
