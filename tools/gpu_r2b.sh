set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests -m gpu > gpurun_out/r2b/tests.log 2>&1; rc=$?; tail -15 gpurun_out/r2b/tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_exp.sh r2b "|c2|20" "|c2x|20" "|c2s|20" "DG_WAVE_MIN=0|c2|10" "|c3|10" "DG_WAVE_MIN=1000000|c3|5" "DG_WAVE_MIN=1000000 DG_SMALL_MPW=32|c3|5" "DG_WAVE_MIN=1000000 DG_SMALL_MPW=16|c3|5"
