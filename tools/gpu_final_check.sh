# round-end rehearsal: the whole GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/fc_gputest.log 2>&1 || { tail -40 gpurun_out/fc_gputest.log; exit 1; }
tail -1 gpurun_out/fc_gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fc_smoke.log 2>&1 || { cat gpurun_out/fc_smoke.log; exit 1; }
tail -1 gpurun_out/fc_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/fc_bench.json 2> gpurun_out/fc_bench.err || { tail -20 gpurun_out/fc_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/fc_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
