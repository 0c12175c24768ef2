# flat kernel: numbers parsed after the size barrier (df) vs in the parse phase (HEAD default)
set -o pipefail
O=gpurun_out/r3ah
mkdir -p $O
export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_df.so DG_ALLOW_STALE=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py tests/test_gpu_parity.py -k "flat or full_batch or shuffled or golden or jsconv or fuzz" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
echo "tests $(tail -1 $O/t.log)"
for v in df "" df ""; do
  if [ -n "$v" ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1; else unset DG_LIB_PATH; fi
  echo "== ${v:-head}"
  timeout -k 10 120 python -u tools/twostream.py 1 60 2>&1 | grep -v amdgpu.ids | tail -2
done
