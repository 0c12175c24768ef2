# t2j GPU tests + t2j bench after a t2j kernel change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_t2j.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2jq_test.log 2>&1 || { tail -40 gpurun_out/t2jq_test.log; exit 1; }
tail -1 gpurun_out/t2jq_test.log
for c in t2j-c2 t2j-c3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/t2jq_$c.json 2> gpurun_out/t2jq_$c.err || { tail -5 gpurun_out/t2jq_$c.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'])" gpurun_out/t2jq_$c.json $c
done
