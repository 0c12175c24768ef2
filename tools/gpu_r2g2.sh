set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_wave.py tests/test_gpu_parity.py tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g2.log 2>&1 || { tail -30 gpurun_out/r2g2.log; exit 1; }
tail -2 gpurun_out/r2g2.log
export DG_ALLOW_STALE=1
for v in "" _ch16 _ch64; do
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u tools/wvtime.py 2>&1 | grep us/step || exit 1
done
