# round-3 final pass at HEAD: rocprof + FETCH/WRITE traffic for the configs whose kernels changed since r3y
# (copied into profiles/ on the box so the bench lines cite them), then the GPU suite, smoke and every bench
set -o pipefail
T=${TAG:-r3z}
O=gpurun_out/$T
mkdir -p $O
TAG=$T SKIP_TESTS=1 SKIP_BENCH=1 CONFIGS="${PMC_CONFIGS:-c2 t2j-c2 t2j-c3}" bash tools/gpu_r3.sh || exit 1
for c in ${PMC_CONFIGS:-c2 t2j-c2 t2j-c3}; do cp $O/traffic_$c.json profiles/traffic_$c.json || exit 1; done
TAG=$T NO_PROF=1 bash tools/gpu_r3.sh || exit 1
timeout -k 10 400 python -u bench.py --config agg --steps 10 > $O/agg_bench.json 2> $O/agg_bench.err || { tail -20 $O/agg_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/agg_bench.json').read().strip().splitlines()[-1]);print('agg',d['value'],(d.get('cpu_baseline') or {}).get('value'))"
echo final-done
