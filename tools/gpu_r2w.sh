set -o pipefail
timeout -k 10 120 env DG_FLAT=1 DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof2.so python -u tools/flprof2.py c2 > gpurun_out/r2w.log 2>&1 || exit 1
cat gpurun_out/r2w.log
