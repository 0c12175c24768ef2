# flat kernel iteration: its parity tests, the batch-size sweep, the C2 bench line
set -o pipefail
T=${TAG:-fl}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 200 python -u tools/fltime_n.py > $O/fltime.log 2>&1 || { tail -20 $O/fltime.log; exit 1; }
cat $O/fltime.log
timeout -k 10 400 python -u bench.py --config c2 > $O/c2_bench.json 2> $O/c2_bench.err || { tail -20 $O/c2_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c2_bench.json').read().strip().splitlines()[-1]);print('c2',d['value'],d['unit'],d['ms_per_step'],d['roofline'])"
echo done
