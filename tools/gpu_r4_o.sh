# r4o: t2j JSON through 64-byte LDS groups -- parity (t2j suite) and t2j-c2/c3 speed and write traffic
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],d["config"].get("serial_gbs"))'
for c in t2j-c2 t2j-c3; do
  timeout -k 10 400 python -u bench.py --config $c > $O/${c}.json 2> $O/${c}.err || { tail -20 $O/${c}.err; exit 1; }
  python -c "$J" $O/${c}.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in t2j-c2 t2j-c3; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcw_$c.log 2>&1 || { tail -20 $O/pmcw_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcf_$c.log 2>&1 || { tail -20 $O/pmcf_$c.log; exit 1; }
done
find $O -name "*counter_collection.csv"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_t2j-c2 -o run -- python3 -u bench.py --config t2j-c2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/kt_t2j-c2.log 2>&1 || { tail -20 $O/kt_t2j-c2.log; exit 1; }
find $O -name "*kernel_stats.csv"
