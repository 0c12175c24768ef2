# round-3 quick check: GPU parity suite, smoke, C2 + C3 bench lines
set -o pipefail
T=${TAG:-r3a}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in ${CFGS:-c2 c3}; do
  timeout -k 10 400 python -u bench.py --config $c ${BENCH_ARGS} > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['unit'],d['ms_per_step'],d['roofline']['frac'],(d.get('cpu_baseline') or {}).get('value'),(d.get('e2e_host') or {}).get('value'))"
done
echo done
