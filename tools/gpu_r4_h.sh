# r4h: aggregator breakdown over the timed steps only; e2e zero-copy check and a kernel + copy timeline
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg.json').read().strip().splitlines()[-1]);print('agg',d['value'],d['cpu_baseline'] and d['cpu_baseline']['share']['msgs_per_s'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50'],r['us_per_batch']) for r in d['config']['runs']])"
DG_PIPE_DEBUG=1 timeout -k 10 200 python -u tools/e2e_trace.py 4 5 > $O/e2e.log 2>&1 || { tail -20 $O/e2e.log; exit 1; }
cat $O/e2e.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/e2etr -o run -- python3 -u tools/e2e_trace.py 4 3 > $O/e2etr.log 2>&1 || { tail -20 $O/e2etr.log; exit 1; }
find $O -name "*.csv"
