# aggregator sweep: ring depth and each thread's share of a batch (window / div)
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
A="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50']) for r in d['config']['runs'][:2]])"
for ring in 16 32; do
  for div in 4 2 8; do
    DG_AGG_RING=$ring DG_BENCH_AGG_SHARE_DIV=$div timeout -k 10 300 python -u bench.py --config agg --steps 5 --warmup 2 --no-cpu-baseline > $O/agg_${ring}_$div.json 2> $O/agg_${ring}_$div.err || { tail -20 $O/agg_${ring}_$div.err; exit 1; }
    python -c "$A" $O/agg_${ring}_$div.json
  done
done
