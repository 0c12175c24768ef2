set -o pipefail
O=gpurun_out/dbgagg2; mkdir -p $O
REPS=15 timeout -k 10 300 python -u tools/dbg_agg.py > $O/out.log 2>&1; rc=$?
tail -40 $O/out.log
exit $rc
