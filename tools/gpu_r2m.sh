set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r2m_flat.log 2>&1 || { tail -30 gpurun_out/r2m_flat.log; exit 1; }
tail -2 gpurun_out/r2m_flat.log
bash tools/gpu_exp.sh r2m "|c2|20" "|c2s|20" || exit 1
DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so DG_ALLOW_STALE=1 timeout -k 10 200 python tools/flprof.py c2
