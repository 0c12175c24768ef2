set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2n_gputest.log 2>&1
rc=$?
tail -5 gpurun_out/r2n_gputest.log
exit $rc
