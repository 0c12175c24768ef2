#!/bin/bash
# GPU-box script: parity suite, then C2 ablate timing and C2/C5 bench lines (no CPU baseline).
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python tools/ablate.py c2 || exit 1
for CFG in c2 c5; do
  timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --no-e2e --steps 20 > $OUT/$CFG.json 2> $OUT/$CFG.err || { tail -5 $OUT/$CFG.err; exit 1; }
  head -c 400 $OUT/$CFG.json; echo
done
