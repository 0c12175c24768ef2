set -o pipefail
export DG_ALLOW_STALE=1 DG_FLAT=1
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so python -u tools/flprof.py c2 > gpurun_out/r2t_flprof.log 2>&1 || exit 1
cat gpurun_out/r2t_flprof.log
