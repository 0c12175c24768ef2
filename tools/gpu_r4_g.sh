# r4g: GPU tests; C2 A/B against the round-3 tree (r3ref/); e2e zero copy on/off; agg breakdown; t2j-c2 traffic
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],d["roofline"].get("traffic"),(d.get("e2e_host") or {}).get("sweep_gbs"))'
for rep in 1 2; do
  (cd r3ref && timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e) > $O/c2_r3_$rep.json 2> $O/c2_r3_$rep.err || { tail -20 $O/c2_r3_$rep.err; exit 1; }
  python -c "$J" $O/c2_r3_$rep.json
  timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/c2_r4_$rep.json 2> $O/c2_r4_$rep.err || { tail -20 $O/c2_r4_$rep.err; exit 1; }
  python -c "$J" $O/c2_r4_$rep.json
done
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_e2e.json 2> $O/c2_e2e.err || { tail -20 $O/c2_e2e.err; exit 1; }
python -c "$J" $O/c2_e2e.json
DG_NO_ZERO_COPY=1 timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_e2e_nozc.json 2> $O/c2_e2e_nozc.err || { tail -20 $O/c2_e2e_nozc.err; exit 1; }
python -c "$J" $O/c2_e2e_nozc.json
timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg.json').read().strip().splitlines()[-1]);print('agg',d['value'],d['cpu_baseline'] and d['cpu_baseline']['share']['msgs_per_s'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50'],r['us_per_batch']) for r in d['config']['runs'][:1]])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
(cd r3ref && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../$O/kt_c2_r3 -o run -- python3 -u bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1) > $O/kt_c2_r3.log 2>&1 || { tail -20 $O/kt_c2_r3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c2 -o run -- python3 -u bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/kt_c2.log 2>&1 || { tail -20 $O/kt_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_t2j-c2 -o run -- python3 -u bench.py --config t2j-c2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcw_t2j-c2.log 2>&1 || { tail -20 $O/pmcw_t2j-c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_t2j-c2 -o run -- python3 -u bench.py --config t2j-c2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcf_t2j-c2.log 2>&1 || { tail -20 $O/pmcf_t2j-c2.log; exit 1; }
find $O -name "*kernel_stats.csv" -o -name "*counter_collection.csv"
