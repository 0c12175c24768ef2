set -o pipefail
for c in c2 c2s c3; do
timeout -k 10 300 python -u bench.py --config $c --no-e2e --no-cpu-baseline > gpurun_out/r2p2_$c.json 2> gpurun_out/r2p2_$c.err || { tail -20 gpurun_out/r2p2_$c.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2p2_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['config']['per_rank_kernel_ms'])"
done
