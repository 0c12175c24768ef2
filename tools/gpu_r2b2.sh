set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b2_gputest.log 2>&1 || { tail -40 gpurun_out/r2b2_gputest.log; exit 1; }
tail -2 gpurun_out/r2b2_gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b2_smoke.log 2>&1 || { cat gpurun_out/r2b2_smoke.log; exit 1; }
tail -1 gpurun_out/r2b2_smoke.log
for c in c2 c2s c2x; do
timeout -k 10 300 python -u bench.py --config $c --no-e2e --no-cpu-baseline > gpurun_out/r2b2_$c.json 2> gpurun_out/r2b2_$c.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/r2b2_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['config']['per_rank_kernel_ms'],d['config']['exact_path_msgs_per_step'],d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r2b2_prof_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r2b2_prof_c2.log 2>&1 || exit 1
head -4 $GRAFT_REPO_ROOT/gpurun_out/r2b2_prof_c2/c2_kernel_stats.csv
