set -o pipefail
L=dynamicgo_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r2k_flat.log 2>&1 || { tail -20 gpurun_out/r2k_flat.log; exit 1; }
tail -2 gpurun_out/r2k_flat.log
bash tools/gpu_exp.sh r2k "|c2|20" "DG_NO_FLAT=1|c2|20" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fwpe4.so|c2|20" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fw8.so|c2|20" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fw2.so|c2|20" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fwpe2.so|c2|20" "|c2x|20" "|c2s|20" "|c1|20"
