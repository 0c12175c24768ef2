set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r2q_gputest.log 2>&1 || { tail -30 gpurun_out/r2q_gputest.log; exit 1; }
tail -3 gpurun_out/r2q_gputest.log
timeout -k 10 300 python -u bench.py --no-e2e > gpurun_out/r2q_c2.json 2> gpurun_out/r2q_c2.err || exit 1
cat gpurun_out/r2q_c2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2q_prof_c2 -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r2q_prof_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r2q_prof_c3 -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --no-cpu-baseline --no-e2e --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/r2q_prof_c3.log 2>&1 || exit 1
echo done
