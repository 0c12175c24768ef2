set -o pipefail
O=gpurun_out/${TAG:-r3h}
mkdir -p $O
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o t2j -- python3 $ROOT/bench.py --config t2j-c3 --no-cpu-baseline --steps 5 --warmup 2 > $ROOT/$O/prof.log 2>&1 || { tail -20 $ROOT/$O/prof.log; exit 1; }
head -8 $ROOT/$O/prof/t2j_kernel_stats.csv
