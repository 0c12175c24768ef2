# r4e: GPU tests (all), then C5 / agg / t2j-c3 benches + kernel stats, aggregator runtime trace
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
for c in c5 t2j-c3 t2j-c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u bench.py --config agg --steps 5 --warmup 2 --no-cpu-baseline > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg.json').read().strip().splitlines()[-1]);print('agg',d['value'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['us_per_batch']) for r in d['config']['runs']])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c5kt -o c5 -- python3 -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/c5kt.log 2>&1 || { tail -20 $O/c5kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/t3kt -o t2jc3 -- python3 -u bench.py --config t2j-c3 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/t3kt.log 2>&1 || { tail -20 $O/t3kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/aggkt -o agg -- python3 -u bench.py --config agg --steps 3 --warmup 1 --no-cpu-baseline > $O/aggkt.log 2>&1 || { tail -20 $O/aggkt.log; exit 1; }
timeout -k 10 300 rocprofv3 --runtime-trace --stats -d $O/aggrt -o agg -- python3 -u bench.py --config agg --steps 3 --warmup 1 --no-cpu-baseline > $O/aggrt.log 2>&1 || { tail -20 $O/aggrt.log; exit 1; }
find $O -name "*stats.csv"
