# round-2 measurement pass: GPU parity suite, smoke, every bench config, rocprof stats, PMC traffic
set -o pipefail
T=${TAG:-r2f}
O=gpurun_out/$T
mkdir -p $O
# heartbeat: long silent steps (C5 generation under rocprof) must not look hung
( while sleep 30; do date >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ -n "$ONLY_PROF" ]; then SKIP_MAIN=1; fi
if [ -z "$SKIP_MAIN" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { tail -20 $O/c2_bench.err; exit 1; }
tail -c 600 $O/c2_bench.json; echo
for c in c2s c2x c3 c4 c1 t2j-c2 t2j-c3; do
  timeout -k 10 400 python -u bench.py --config $c --no-e2e > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['unit'],d['ms_per_step'],d['roofline']['frac'],(d.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 600 python -u bench.py --config c5 --no-e2e --steps 5 > $O/c5_bench.json 2> $O/c5_bench.err || { tail -20 $O/c5_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c5_bench.json').read().strip().splitlines()[-1]);print('c5',d['value'],d['ms_per_step'],d['roofline']['frac'])"
fi
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
[ -z "$SKIP_MAIN" ] && for c in c2 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_$c -o $c -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --no-e2e --steps 10 > $ROOT/$O/prof_$c.log 2>&1 || exit 1
  head -4 $ROOT/$O/prof_$c/${c}_kernel_stats.csv
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof_c5 -o c5 -- python3 $ROOT/bench.py --config c5 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/prof_c5.log 2>&1 || exit 1
head -5 $ROOT/$O/prof_c5/c5_kernel_stats.csv
for c in c2 c3; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/$O/pmcf_$c -o run -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/pmcf_$c.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/$O/pmcw_$c -o run -- python3 $ROOT/bench.py --config $c --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/pmcw_$c.log 2>&1 || exit 1
done
echo done
