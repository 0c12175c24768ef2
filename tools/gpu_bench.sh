#!/bin/bash
# GPU-box script: bench + rocprofv3 kernel-trace summary. Output under gpurun_out/.
# usage: bash tools/gpu_bench.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $ROOT/bench.py "$@" --no-cpu-baseline --no-e2e > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \;
