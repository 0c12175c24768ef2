set -o pipefail
mkdir -p gpu_out_tmp gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_t2j.py -v --timeout 120 --timeout-method thread > gpurun_out/r2g_t2j.log 2>&1
rc=$?
tail -30 gpurun_out/r2g_t2j.log
exit $rc
