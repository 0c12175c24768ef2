set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_streams.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qf.log 2>&1 || { tail -30 gpurun_out/qf.log; exit 1; }
tail -2 gpurun_out/qf.log
timeout -k 10 120 python -u tools/fltime.py c2 2>&1 | grep us/step || exit 1
timeout -k 10 120 python -u tools/fltime.py c2s 2>&1 | grep us/step || exit 1
