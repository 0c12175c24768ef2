# t2j wave path: GPU t2j tests, t2j benches, then the aggregator tests + bench
set -o pipefail
O=gpurun_out/${TAG:-r3g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_t2j.py -x -v --timeout 120 --timeout-method thread > $O/t2j_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/t2j_tests.log | tail -30; exit 1; }
tail -1 $O/t2j_tests.log
for c in t2j-c3 t2j-c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}_bench.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['config']['ok_msgs_rank0'])"
done
TAG=$TAG NO_E2E=1 bash tools/gpu_r3c.sh
