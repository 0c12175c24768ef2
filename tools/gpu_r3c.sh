# aggregator + pipeline tests, aggregator bench, C-pipeline e2e sweep (c2, c3)
set -o pipefail
O=gpurun_out/${TAG:-r3c}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_agg.py -x -v --timeout 120 --timeout-method thread > $O/agg_tests.log 2>&1 || { tail -30 $O/agg_tests.log; exit 1; }
tail -1 $O/agg_tests.log
timeout -k 10 400 python -u bench.py --config agg --steps 10 > $O/agg_bench.json 2> $O/agg_bench.err || { tail -20 $O/agg_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg_bench.json').read().strip().splitlines()[-1]);print('agg',d['value'],d['config']['runs'],(d.get('cpu_baseline') or {}).get('value'))"
[ -n "$NO_E2E" ] && exit 0
for c in c2 c3; do
timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/${c}_e2e.json 2> $O/${c}_e2e.err || { tail -20 $O/${c}_e2e.err; exit 1; }
python -c "import json;d=json.loads(open('$O/${c}_e2e.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['e2e_host'])"
done
