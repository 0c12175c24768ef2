# flat kernel chunk-task size: 32 (HEAD) vs 24 vs 16 (+ inline 8)
set -o pipefail
O=gpurun_out/r3ae
mkdir -p $O
for v in "" c16 c24 c16i8 ""; do
  if [ -n "$v" ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1; else unset DG_LIB_PATH; fi
  echo "== ${v:-base}"
  timeout -k 10 120 python -u tools/twostream.py 1 60 2>&1 | grep -v amdgpu.ids | tail -3
done
for v in c16 c24 c16i8; do
  export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; exit 1; }
  echo "$v $(tail -1 $O/t_$v.log)"
done
