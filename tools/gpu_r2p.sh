set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_http.py -q --timeout 120 --timeout-method thread > gpurun_out/r2p.log 2>&1
rc=$?
tail -15 gpurun_out/r2p.log
exit $rc
