# r3y part 2: rocprof kernel stats + FETCH/WRITE traffic of every config (serial leg), aggregator bench, e2e sweep
set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 400 python -u bench.py --config agg --steps 10 > $O/agg_bench.json 2> $O/agg_bench.err || { tail -20 $O/agg_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg_bench.json').read().strip().splitlines()[-1]);print('agg',d['value'],(d.get('cpu_baseline') or {}).get('value'))"
for c in c2 c3; do
timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/${c}_e2e.json 2> $O/${c}_e2e.err || { tail -20 $O/${c}_e2e.err; exit 1; }
python -c "import json;d=json.loads(open('$O/${c}_e2e.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['e2e_host'])"
done
TAG=r3y SKIP_TESTS=1 SKIP_BENCH=1 bash tools/gpu_r3.sh
