set -o pipefail
O=gpurun_out/${TAG:-fl7}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
VARIANTS="_fpw2 _fpw2i32 _i32" SIZES="12288 65536" bash tools/gpu_flv.sh
