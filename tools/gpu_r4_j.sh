# r4j: aggregator buffers at the parts' cap bound; e2e timeline after the device cursor; t2j-c3 wave threshold below 512
set -o pipefail
O=gpurun_out/r4j
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_agg.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],(d.get("e2e_host") or {}).get("sweep_gbs"))'
A="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('agg',d['value'],d['cpu_baseline'] and d['cpu_baseline']['share']['msgs_per_s'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50'],r['us_per_batch']) for r in d['config']['runs'][:2]])"
timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "$A" $O/agg.json
DG_AGG_RING=16 timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 --no-cpu-baseline > $O/agg16.json 2> $O/agg16.err || { tail -20 $O/agg16.err; exit 1; }
python -c "$A" $O/agg16.json
for w in 256 384; do
  DG_T2J_WAVE_MIN=$w timeout -k 10 300 python -u bench.py --config t2j-c3 --steps 10 --warmup 3 --no-cpu-baseline > $O/t3_$w.json 2> $O/t3_$w.err || { tail -20 $O/t3_$w.err; exit 1; }
  python -c "$J" $O/t3_$w.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/e2etr -o run -- python3 -u tools/e2e_trace.py 4 3 > $O/e2etr.log 2>&1 || { tail -20 $O/e2etr.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/e2etr1 -o run -- python3 -u tools/e2e_trace.py 1 3 > $O/e2etr1.log 2>&1 || { tail -20 $O/e2etr1.log; exit 1; }
find $O -name "*.csv"
