# r4m: t2j variants -- walkers per wave (T2W_MPT 16/32/64) and non-temporal JSON pair stores; traffic of the latter
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],d["config"].get("serial_gbs"))'
export DG_ALLOW_STALE=1
for v in main mpt32 mpt64p ntp; do
  if [ $v = main ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t.so; else export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so; fi
  for c in t2j-c3 t2j-c2; do
    timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/${c}_$v.json 2> $O/${c}_$v.err || { tail -20 $O/${c}_$v.err; exit 1; }
    python -c "$J" $O/${c}_$v.json
  done
done
export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_ntp.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmcw_nt -o run -- python3 -u bench.py --config t2j-c2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcw_nt.log 2>&1 || { tail -20 $O/pmcw_nt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcf_nt -o run -- python3 -u bench.py --config t2j-c2 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/pmcf_nt.log 2>&1 || { tail -20 $O/pmcf_nt.log; exit 1; }
find $O -name "*counter_collection.csv"
unset DG_LIB_PATH DG_ALLOW_STALE
A="import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('agg',d['value'],d['cpu_baseline'] and d['cpu_baseline']['share']['msgs_per_s'],[ (r['threads'],r['msgs_per_s'],r['avg_batch'],r['lat_us_p50'],r['us_per_batch']['ns_per_call_in_submit'],r['us_per_batch']['ns_per_call_in_wait']) for r in d['config']['runs'][:2]])"
timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_e2e.json 2> $O/c2_e2e.err || { tail -20 $O/c2_e2e.err; exit 1; }
python -c "import json,sys;d=json.loads(open('$O/c2_e2e.json').read().strip().splitlines()[-1]);print('c2',d['value'],d['e2e_host']['sweep_gbs'])"
timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
python -c "$A" $O/agg.json
DG_HOST_NUMA=1 timeout -k 10 400 python -u bench.py --config agg --steps 5 --warmup 2 > $O/agg_numa.json 2> $O/agg_numa.err || { tail -20 $O/agg_numa.err; exit 1; }
python -c "$A" $O/agg_numa.json
