#!/bin/bash
# round-2 GPU check: parity tests, default bench, C5 at N=1 and N=2 (two
# ranks sharing the one GPU over gloo), C3 bench.
set -o pipefail
OUT=gpurun_out/${1:-r2a}
mkdir -p $OUT
export TMPDIR=/tmp DG_LOG_LIB=1
echo "== tests" >&2
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
echo "== bench default" >&2
timeout -k 10 300 python bench.py > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
head -c 3000 $OUT/c2.json; echo
echo "== c5 n=1" >&2
timeout -k 10 300 python bench.py --config c5 --steps 5 --no-e2e > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
head -c 1500 $OUT/c5.json; echo
echo "== c5 n=2 gloo shared gpu" >&2
DG_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --config c5 --steps 5 --no-e2e > $OUT/c5n2.json 2> $OUT/c5n2.err || { tail -20 $OUT/c5n2.err; exit 1; }
head -c 1500 $OUT/c5n2.json; echo
echo "== c3" >&2
timeout -k 10 300 python bench.py --config c3 --steps 10 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
head -c 1500 $OUT/c3.json; echo
