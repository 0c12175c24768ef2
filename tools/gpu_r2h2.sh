set -o pipefail
export DG_ALLOW_STALE=1
timeout -k 10 200 python -u tools/dbg_d3.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 env DG_LIB_PATH=dynamicgo_amd/libdgj2t_head.so python -u tools/dbg_d3.py 2>&1 | grep -v amdgpu.ids
