set -o pipefail
export DG_ALLOW_STALE=1
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so python -u tools/flprof.py c2 > gpurun_out/r2r_flprof.log 2>&1 || exit 1
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so python -u tools/flprof.py c2s >> gpurun_out/r2r_flprof.log 2>&1 || exit 1
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t_fprof.so python -u tools/fprof.py c2 > gpurun_out/r2r_fprof.log 2>&1 || exit 1
timeout -k 10 200 env DG_FLAT=1 python -u bench.py --no-e2e --no-cpu-baseline > gpurun_out/r2r_flat_c2.json 2>&1 || exit 1
cat gpurun_out/r2r_flprof.log gpurun_out/r2r_fprof.log
