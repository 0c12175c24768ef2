# wave kernel: GPU tests (wave + parity + flat), then C3/C5/C4 bench lines
set -o pipefail
T=${TAG:-wv}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
for c in ${CFGS:-c3}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e --steps 10 > $O/${c}.json 2> $O/${c}.err || { tail -20 $O/${c}.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${c}.json').read().strip().splitlines()[-1]);c=d['config'];print('$c',d['value'],d['unit'],d['ms_per_step'],d['roofline']['frac'],'bails',c['exact_path_msgs_per_step'])"
done
