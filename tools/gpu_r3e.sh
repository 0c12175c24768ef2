set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 120 python -u tools/e2e_trace.py 4 5 > $O/e2e_plain.log 2>&1 || { tail -20 $O/e2e_plain.log; exit 1; }
cat $O/e2e_plain.log
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $ROOT/$O/trace -o run -- python3 $ROOT/tools/e2e_trace.py 4 3 > $ROOT/$O/e2e_trace.log 2>&1 || { tail -20 $ROOT/$O/e2e_trace.log; exit 1; }
ls $ROOT/$O/trace/*
