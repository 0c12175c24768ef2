# quick check after a wave-kernel change: wave + parity GPU tests, C3/C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wvq_test.log 2>&1 || { tail -40 gpurun_out/wvq_test.log; exit 1; }
tail -1 gpurun_out/wvq_test.log
for c in c3 c5 c4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/wvq_$c.json 2> gpurun_out/wvq_$c.err || { tail -5 gpurun_out/wvq_$c.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'])" gpurun_out/wvq_$c.json $c
done
