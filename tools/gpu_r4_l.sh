# r4l: pack counts overflows (no status scan), t2j wave threshold 256, drive blocks on the oldest call again
set -o pipefail
O=gpurun_out/r4l
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],(d.get("e2e_host") or {}).get("sweep_gbs"))'
A="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('agg',d['value'],d['cpu_baseline'] and d['cpu_baseline']['share']['msgs_per_s'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50'],r['us_per_batch']) for r in d['config']['runs'][:2]])"
timeout -k 10 200 python -u tools/e2e_trace.py 4 5 > $O/e2e.log 2>&1 && DG_PIPE_STAGED=1 timeout -k 10 200 python -u tools/e2e_trace.py 4 5 > $O/e2e_staged.log 2>&1 || { tail -20 $O/e2e.log; exit 1; }
grep chunks $O/e2e.log; grep chunks $O/e2e_staged.log
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_e2e.json 2> $O/c2_e2e.err || { tail -20 $O/c2_e2e.err; exit 1; }
python -c "$J" $O/c2_e2e.json
timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "$A" $O/agg.json
for w in 256; do
  DG_T2J_WAVE_MIN=$w timeout -k 10 300 python -u bench.py --config t2j-c3 --steps 10 --warmup 3 --no-cpu-baseline > $O/t3_$w.json 2> $O/t3_$w.err || { tail -20 $O/t3_$w.err; exit 1; }
  python -c "$J" $O/t3_$w.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/e2etr -o run -- python3 -u tools/e2e_trace.py 4 3 > $O/e2etr.log 2>&1 || { tail -20 $O/e2etr.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/e2etr1 -o run -- python3 -u tools/e2e_trace.py 1 3 > $O/e2etr1.log 2>&1 || { tail -20 $O/e2etr1.log; exit 1; }
find $O -name "*.csv"
