# in-flight API: tests + bench at depth 1/2/3/4 (C2), 2 (C3, C4)
set -o pipefail
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py -k "inflight or iters" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for d in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --config c2 --no-cpu-baseline --no-e2e --inflight $d > $O/c2_$d.json 2> $O/c2_$d.err || { tail -20 $O/c2_$d.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/c2_$d.json')); print('c2 d=$d', d['value'], d['ms_per_step'], d['config']['serial_gbs'], d['roofline']['kernel_ms'])"
done
for c in c3 c4 c2s; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['config']['serial_gbs'], d['roofline']['kernel_ms'])"
done
echo done
