set -o pipefail
L=dynamicgo_amd
bash tools/gpu_exp.sh r2l "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fwpe4.so|c2|20" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fwpe5.so|c2|20" "DG_ALLOW_STALE=1 DG_LIB_PATH=$L/libdgj2t_fwpe6.so|c2|20"
