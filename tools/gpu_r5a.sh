# r5a: new GPU tests (dist / t2j base / shifted arena), flat-kernel SQ counters, c2 kernel trace
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_t2j.py::test_response_base tests/test_gpu_agg.py -v --timeout 120 --timeout-method thread > $O/newtests.log 2>&1; echo "newtests rc=$?" >> $O/newtests.log
tail -3 $O/newtests.log
O=$O CONFIGS="c2 c2s" timeout -k 10 500 bash tools/gpu_sqinsts.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c2 -o run -- python3 -u bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --inflight 1 > $O/kt_c2.log 2>&1
