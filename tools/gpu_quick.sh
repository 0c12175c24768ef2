# quick check after a kernel change: parity tests for the touched kernels, then bench lines (no CPU baseline / e2e)
# usage: O=gpurun_out/r5x TESTS="tests/test_gpu_flat.py" CONFIGS="c2 c2s c3" bash tools/gpu_quick.sh
set -o pipefail
O=${O:-gpurun_out/quick}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c 'import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],d["config"]["exact_path_msgs_per_step"])' $O/${c}_bench.json
done
