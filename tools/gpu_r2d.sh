set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r2d/tests.log 2>&1; rc=$?; tail -15 gpurun_out/r2d/tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_exp.sh r2d "|c2|20" "|c2x|20" "|c2s|20" "|c3|10" "|c5|5"
