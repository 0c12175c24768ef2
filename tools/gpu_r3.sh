# round-3 measurement pass: GPU parity suite, smoke, every bench config, rocprof
# kernel stats and FETCH/WRITE traffic for every config (traffic_<cfg>.json)
# (profiles and counters: one batch at a time, --inflight 1, the leg the roofline is priced on)
# usage: TAG=r3a [SKIP_TESTS=1] [CONFIGS="c2 c3"] [NO_PMC=1] bash tools/gpu_r3.sh
set -o pipefail
T=${TAG:-r3a}
O=gpurun_out/$T
mkdir -p $O
( while sleep 30; do date >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
CONFIGS=${CONFIGS:-"c2 c2s c2x c1 c3 c4 c5 t2j-c2 t2j-c3"}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
[ -z "$SKIP_BENCH" ] && for c in $CONFIGS; do
  ST=20; [ $c = c5 ] && ST=5
  timeout -k 10 500 python -u bench.py --config $c --steps $ST $BENCH_ARGS > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['unit'],d['ms_per_step'],d['roofline']['frac'],(d.get('cpu_baseline') or {}).get('value'))"
done
[ -n "$NO_PROF" ] && exit 0
ROOT=$(pwd)
case " $CONFIGS " in *" c5 "*)  # the C5 batch generated once, outside the profiler (its worker pool)
  timeout -k 10 300 python3 -c "import bench; bench.c5_shared_arena(bench.CONFIGS['c5'][1], 45, 1.0, bench.gen_workers())" || exit 1
  export DG_C5_CACHE=1
  trap "kill $HB 2>/dev/null; python3 -c 'import bench; bench.release_c5_cache()'" EXIT;;
esac
cd /tmp && export TMPDIR=/tmp
[ -z "$SKIP_PROF" ] && for c in $CONFIGS; do
  ST=10; W=3; [ $c = c5 ] && { ST=3; W=1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_$c -o $c -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --no-e2e --inflight 1 --steps $ST --warmup $W > $ROOT/$O/prof_$c.log 2>&1 || exit 1
  head -4 $ROOT/$O/prof_$c/${c}_kernel_stats.csv
done
[ -n "$NO_PMC" ] && exit 0
for c in $CONFIGS; do
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/$O/pmcf_$c -o run -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --no-e2e --inflight 1 --steps 3 --warmup 1 > $ROOT/$O/pmcf_$c.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/$O/pmcw_$c -o run -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --no-e2e --inflight 1 --steps 3 --warmup 1 > $ROOT/$O/pmcw_$c.log 2>&1 || exit 1
  case $c in c3|c4|c5) K=j2t_wave_kernel;; t2j-c3) K=t2j_wave_kernel;; t2j-*) K=t2j_kernel;; *) K=j2t_flat_kernel;; esac
  python3 $ROOT/tools/traffic.py $(find $ROOT/$O/pmcf_$c -name '*counter_collection.csv') $(find $ROOT/$O/pmcw_$c -name '*counter_collection.csv') $K $ROOT/$O/traffic_$c.json > $ROOT/$O/traffic_$c.log || exit 1; head -c 300 $ROOT/$O/traffic_$c.log; echo
done
echo done
