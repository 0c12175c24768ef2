# flat kernel block shape: 4 waves x 2 fields (HEAD) vs 6 x 1 vs 8 x 1
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
for v in "" fl6 fl8; do
  if [ -n "$v" ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1; fi
  echo "== ${v:-base}"
  timeout -k 10 120 python -u tools/twostream.py 1 40 > $O/t_${v:-base}.log 2>&1 || { tail -20 $O/t_${v:-base}.log; exit 1; }
  cat $O/t_${v:-base}.log | grep -v amdgpu.ids
  timeout -k 10 120 python -u tools/twostream.py 2 40 > $O/t2_${v:-base}.log 2>&1 || { tail -20 $O/t2_${v:-base}.log; exit 1; }
  cat $O/t2_${v:-base}.log | grep -v amdgpu.ids
done
for v in fl6 fl8; do
  export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py tests/test_gpu_parity.py -k "flat or full_batch or shuffled or golden" > $O/test_$v.log 2>&1 || { tail -30 $O/test_$v.log; exit 1; }
  tail -3 $O/test_$v.log
done
echo done
