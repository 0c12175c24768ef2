# flat kernel phase profile at HEAD + two-stream C2
set -o pipefail
O=gpurun_out/r3r
mkdir -p $O
DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_flprof.so timeout -k 10 200 python -u tools/flprof.py c2 > $O/flprof.log 2>&1 || { tail -20 $O/flprof.log; exit 1; }
cat $O/flprof.log
timeout -k 10 200 python -u tools/twostream.py 2 40 > $O/two.log 2>&1 || { tail -20 $O/two.log; exit 1; }
cat $O/two.log
echo done
