# r4p: t2j LDS output groups -- flush by call (main) vs inline whole-group stores (ginl); pair stores (safe-no-jout tree) for reference
set -o pipefail
O=gpurun_out/r4p
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],d["config"].get("serial_gbs"))'
export DG_ALLOW_STALE=1
for v in main ginl; do
  if [ $v = main ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t.so; else export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so; fi
  for c in t2j-c2 t2j-c3; do
    timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/${c}_$v.json 2> $O/${c}_$v.err || { tail -20 $O/${c}_$v.err; exit 1; }
    python -c "$J" $O/${c}_$v.json
  done
done
export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_ginl.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_t2j.py -x -q --timeout 120 --timeout-method thread > $O/gputest_ginl.log 2>&1 || { tail -40 $O/gputest_ginl.log; exit 1; }
tail -1 $O/gputest_ginl.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw -o run -- python3 -u bench.py --config t2j-c2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcw.log 2>&1 || { tail -20 $O/pmcw.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf -o run -- python3 -u bench.py --config t2j-c2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcf.log 2>&1 || { tail -20 $O/pmcf.log; exit 1; }
find $O -name "*counter_collection.csv"
