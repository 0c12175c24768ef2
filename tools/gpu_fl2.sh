# flat kernel variants: parity, batch-size sweep per variant, phase profile
set -o pipefail
O=gpurun_out/${TAG:-fl2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for v in "" _fpw2; do
  echo "variant $v"
  DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t$v.so timeout -k 10 200 python -u tools/fltime_n.py > $O/fltime$v.log 2>&1 || { tail -20 $O/fltime$v.log; exit 1; }
  grep us/step $O/fltime$v.log
done
DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_flprof.so timeout -k 10 200 python -u tools/flprof.py c2 > $O/flprof.log 2>&1 || { tail -20 $O/flprof.log; exit 1; }
cat $O/flprof.log
echo done
