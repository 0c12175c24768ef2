# A/B of aggregator library variants on the gateway shape (bench.py --config agg), interleaved
# usage: VARIANTS="libdgj2t libdgj2t_gwp8" bash tools/gpu_gw_ab.sh
O=${O:-gpurun_out/gwab}; mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-libdgj2t}; do
  DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/$v.so timeout -k 10 300 python -u bench.py --config agg --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
  python - $O/${v}_$rep.json $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], [(r["callers"], r["msgs_per_s"], r["msgs_per_s_best"], r["worker_ns_per_call"]["in_wait"]) for r in d["config"]["gateway_runs"]])
PY
done; done
