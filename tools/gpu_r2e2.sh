set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_streams.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2e2.log 2>&1 || { tail -30 gpurun_out/r2e2.log; exit 1; }
tail -2 gpurun_out/r2e2.log
timeout -k 10 120 python -u tools/wvtime.py 2>&1 | grep us/step || exit 1
