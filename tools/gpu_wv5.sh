# GPU suite + C2..C5 bench after a wave-kernel change
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wv5_gputest.log 2>&1 || { tail -40 gpurun_out/wv5_gputest.log; exit 1; }
tail -2 gpurun_out/wv5_gputest.log
for c in c3 c4 c5 c2; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/wv5_$c.json 2> gpurun_out/wv5_$c.err || { tail -5 gpurun_out/wv5_$c.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'])" gpurun_out/wv5_$c.json $c
done
