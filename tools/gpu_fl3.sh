# flat kernel: per-kernel durations at 12288 and 65536 messages, phase profile
set -o pipefail
O=gpurun_out/${TAG:-fl3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof12k -o run -- python3 -u tools/fltime_n.py 12288 > $O/p12.log 2>&1 || { tail -20 $O/p12.log; exit 1; }
grep us/step $O/p12.log
find $O/prof12k -name "*kernel_stats.csv" -exec cat {} \;
DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_flprof.so timeout -k 10 200 python -u tools/flprof.py c2 > $O/flprof.log 2>&1 || { tail -20 $O/flprof.log; exit 1; }
cat $O/flprof.log
echo done
