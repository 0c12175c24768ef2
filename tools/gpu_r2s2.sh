set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2s2.log 2>&1 || { tail -30 gpurun_out/r2s2.log; exit 1; }
tail -2 gpurun_out/r2s2.log
for c in c5 c4; do
timeout -k 10 400 python -u bench.py --config $c --no-e2e --no-cpu-baseline --steps 5 > gpurun_out/r2s2_$c.json 2> gpurun_out/r2s2_$c.err || { tail -20 gpurun_out/r2s2_$c.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2s2_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'])"
done
