# A/B of library variants on ONE box (tools/build_variants.py builds them as
# dynamicgo_amd/libdgj2t_<name>.so), interleaved, REPS rounds:
#   VARIANTS="libdgj2t_base libdgj2t" CONFIGS="c2 c3" O=gpurun_out/x bash tools/gpu_ab.sh
# MODE=bench (default): bench.py lines (value, the dominant kernel's ms)
# MODE=kstats: rocprofv3 --kernel-trace --stats over tools/ablate.py (CONFIGS: c2 c3 c3small c3big)
# TESTS="tests/test_gpu_flat.py ...": run those GPU tests first (the default library)
set -o pipefail
O=${O:-gpurun_out/ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
ROOT=$(pwd)
for rep in ${REPS:-1 2 3}; do
for v in ${VARIANTS:-libdgj2t}; do
for c in ${CONFIGS:-c2}; do
  if [ "${MODE:-bench}" = kstats ]; then
    (cd /tmp && export TMPDIR=/tmp && DG_ALLOW_STALE=1 DG_LIB_PATH=$ROOT/dynamicgo_amd/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/${v}_${c}_$rep -o run -- python3 $ROOT/tools/ablate.py $c > $ROOT/$O/${v}_${c}_$rep.log 2>&1) || { tail -20 $O/${v}_${c}_$rep.log; exit 1; }
    python3 -c '
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], sys.argv[3], " ".join("%s=%.2fus" % (r["Name"].split("(")[0].split("<")[0][-22:], float(r["AverageNs"])/1e3) for r in rows if "j2t" in r["Name"] or "t2j" in r["Name"]))' $O/${v}_${c}_$rep/run_kernel_stats.csv $v $c
  else
    DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/$v.so timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/${v}_${c}_$rep.json 2> $O/${v}_${c}_$rep.err || { tail -5 $O/${v}_${c}_$rep.err; exit 1; }
    python -c 'import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],sys.argv[3],d["value"],d["ms_per_step"],d["config"].get("serial_gbs"),d["roofline"]["kernel_ms"])' $O/${v}_${c}_$rep.json $v $c
  fi
done; done; done
