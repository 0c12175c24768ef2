set -o pipefail
L=dynamicgo_amd
bash tools/gpu_exp.sh r2f "|c3|10" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w5.so|c3|10" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_w4g.so|c3|10" "|c5|5" "|c4|5"
