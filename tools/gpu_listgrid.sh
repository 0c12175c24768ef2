#!/bin/bash
# GPU-box script: list-pass kernel duration vs its grid (DG_LIST_BLOCKS), C2.
set -o pipefail
ROOT=$(pwd)
export TMPDIR=/tmp
for LB in 1 4 16; do
  cd /tmp && DG_LIST_BLOCKS=$LB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/lg$LB -o run -- python3 $ROOT/tools/ablate.py c2 > $ROOT/gpurun_out/lg$LB.log 2>&1 || { echo "lb $LB failed"; tail -5 $ROOT/gpurun_out/lg$LB.log; exit 1; }
  echo "== list blocks $LB"; tail -1 $ROOT/gpurun_out/lg$LB.log
  find $ROOT/gpurun_out/lg$LB -name "*kernel_stats.csv" -exec grep -h "j2t_" {} \; | cut -d, -f1-4
done
