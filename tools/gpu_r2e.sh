set -o pipefail
L=dynamicgo_amd
bash tools/gpu_exp.sh r2e "|c3|10" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w2s.so|c3|10" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w3.so|c3|10" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w4.so|c3|10" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w3.so|c5|5" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w4.so|c5|5"
