set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2a2_flat.log 2>&1 || { tail -30 gpurun_out/r2a2_flat.log; exit 1; }
tail -2 gpurun_out/r2a2_flat.log
export DG_FLAT=1 DG_ALLOW_STALE=1
for v in "" _wpe6; do
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u tools/fltime.py c2 2>&1 | grep us/step || exit 1
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u tools/fltime.py c2s 2>&1 | grep us/step || exit 1
done
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so python -u tools/flprof.py c2 2>&1 | grep -v amdgpu.ids || exit 1
