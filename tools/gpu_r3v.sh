set -o pipefail
O=gpurun_out/r3v
mkdir -p $O
DG_ALLOW_STALE=1 DG_LIB_PATH=$(pwd)/dynamicgo_amd/libdgj2t_t2wprof.so timeout -k 10 200 python -u tools/t2wprof.py > $O/t2wprof.log 2>&1 || { tail -20 $O/t2wprof.log; exit 1; }
cat $O/t2wprof.log
