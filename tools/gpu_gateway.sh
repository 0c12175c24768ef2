# gateway-shape aggregator runs (bench.py --config agg), per min_fill divisor and worker count
# usage: O=gpurun_out/r5y4 FILLS="8 0" WORKERS="16 12" bash tools/gpu_gateway.sh
O=${O:-gpurun_out/gateway}; mkdir -p $O
for wk in ${WORKERS:-16}; do
for f in ${FILLS:-8}; do
DG_BENCH_GW_WORKERS=$wk DG_BENCH_GW_FILL_DIV=$f timeout -k 10 300 python -u bench.py --config agg --no-cpu-baseline > $O/agg_w${wk}_f$f.json 2> $O/agg_w${wk}_f$f.err || { tail -5 $O/agg_w${wk}_f$f.err; exit 1; }
python - $O/agg_w${wk}_f$f.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d["value"])
for r in d["config"]["gateway_runs"]: print(" ", r["callers"], r["os_threads"], r["min_fill"], r["msgs_per_s"], r["msgs_per_s_best"], r["lat_us_p50"], r["avg_batch"], r["us_per_batch"]["flusher_wait_free"], r["us_per_batch"]["flusher_wait_seal"], r["worker_ns_per_call"])
PY
done
done
