# r4f: GPU tests, benches (c2 c3 c5 t2j-c2 t2j-c3; agg with its CPU baseline), kernel stats, t2j PMC traffic
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for c in c2 c3 c5 t2j-c2 t2j-c3; do
  E=--no-e2e; [ $c = c2 ] && E=
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline $E > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d.get('e2e_host'))"
done
timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg.json').read().strip().splitlines()[-1]);print('agg',d['value'],d['cpu_baseline'] and (d['cpu_baseline']['value'], d['cpu_baseline']['share']),[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50']) for r in d['config']['runs']])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c5 t2j-c2 t2j-c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/kt_$c.log 2>&1 || { tail -20 $O/kt_$c.log; exit 1; }
done
for c in t2j-c2 t2j-c3; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcf_$c.log 2>&1 || { tail -20 $O/pmcf_$c.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcw_$c.log 2>&1 || { tail -20 $O/pmcw_$c.log; exit 1; }
done
find $O -name "*stats.csv" -o -name "*counter_collection.csv"
