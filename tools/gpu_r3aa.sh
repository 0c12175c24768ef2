# flat kernel: field-to-wave assignment (w + 4h vs snake)
set -o pipefail
O=gpurun_out/r3aa
mkdir -p $O
for v in "" p1 "" p1; do
  if [ -n "$v" ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1; else unset DG_LIB_PATH; fi
  echo "== ${v:-base}"
  timeout -k 10 120 python -u tools/twostream.py 1 60 2>&1 | grep -v amdgpu.ids
done
export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_p1.so DG_ALLOW_STALE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py > $O/test_p1.log 2>&1 || { tail -30 $O/test_p1.log; exit 1; }
tail -1 $O/test_p1.log
