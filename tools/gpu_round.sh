#!/bin/bash
# GPU-box script: parity tests, C2 bench (+CPU baseline, e2e) with rocprof stats,
# C2 HBM traffic (2 PMC passes), C3/C4/C5 bench lines. Output under gpurun_out/$1.
set -o pipefail
TAG=${1:-round}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*" >&2; }
step tests
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
step pmc
for C in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_$C -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
cd $ROOT
python3 tools/traffic.py $(find $OUT/pmc_FETCH_SIZE -name "*counter_collection.csv") $(find $OUT/pmc_WRITE_SIZE -name "*counter_collection.csv") j2t_small_kernel $OUT/traffic_c2.json && cp $OUT/traffic_c2.json profiles/ || exit 1
step bench-c2
bash tools/gpu_bench.sh $TAG/c2 --config c2 > $OUT/c2.txt 2>&1 || { cat $OUT/c2.txt; exit 1; }
for CFG in c3 c4 c5; do
  step bench-$CFG
  timeout -k 10 400 python bench.py --config $CFG --no-cpu-baseline --steps 10 > $OUT/$CFG.json 2> $OUT/$CFG.err || { tail -5 $OUT/$CFG.err; exit 1; }
done
head -c 2000 $OUT/c2.txt; echo; for CFG in c3 c4 c5; do head -c 600 $OUT/$CFG.json; echo; done
step rocprof-c5
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5prof -o run -- python3 $ROOT/bench.py --config c5 --no-cpu-baseline --no-e2e --steps 10 > $OUT/c5prof.json 2> $OUT/c5prof.err || { echo "rocprof c5 failed"; exit 1; }
find $OUT/c5prof -name "*kernel_stats.csv" -exec head -5 {} \;
