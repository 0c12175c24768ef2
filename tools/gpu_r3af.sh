# flat kernel: task-cap hardening (base), then the 16-byte-chunk build that overflowed the cap before
set -o pipefail
O=gpurun_out/r3af
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py > $O/t_base.log 2>&1 || { tail -30 $O/t_base.log; exit 1; }
echo "base $(tail -1 $O/t_base.log)"
timeout -k 10 120 python -u tools/twostream.py 1 60 2>&1 | grep -v amdgpu.ids | tail -2
export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_c16.so DG_ALLOW_STALE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py > $O/t_c16.log 2>&1 || { tail -30 $O/t_c16.log; exit 1; }
echo "c16 $(tail -1 $O/t_c16.log)"
