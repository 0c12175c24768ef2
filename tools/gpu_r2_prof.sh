#!/bin/bash
# GPU-box script (round 2): rocprof kernel stats + HBM traffic (FETCH/WRITE in
# separate --pmc passes) for the dominant kernel of each config, copied to
# profiles/ as r2_<tag>_<cfg>_kernel_stats.csv and traffic_<cfg>.json.
# usage: bash tools/gpu_r2_prof.sh <tag> <cfg>:<kernel-substring> ...
set -o pipefail
TAG=$1; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for spec in "$@"; do
  CFG=${spec%%:*}; K=${spec#*:}
  echo "== $CFG ($K)" >&2
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$CFG -o run -- python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --no-e2e --steps 10 --warmup 2 > $OUT/stats_$CFG.json 2> $OUT/stats_$CFG.err || { echo "stats $CFG failed"; tail -5 $OUT/stats_$CFG.err; exit 1; }
  for C in FETCH_SIZE WRITE_SIZE; do
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${CFG}_$C -o run -- python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $OUT/pmc_${CFG}_$C.log 2>&1 || { echo "pmc $CFG $C failed"; tail -5 $OUT/pmc_${CFG}_$C.log; exit 1; }
  done
  cd $ROOT
  python3 tools/traffic.py $(find $OUT/pmc_${CFG}_FETCH_SIZE -name "*counter_collection.csv") $(find $OUT/pmc_${CFG}_WRITE_SIZE -name "*counter_collection.csv") $K $OUT/traffic_$CFG.json || exit 1
  cp $OUT/traffic_$CFG.json profiles/traffic_$CFG.json
  cp $(find $OUT/stats_$CFG -name "*kernel_stats.csv") profiles/${TAG}_${CFG}_kernel_stats.csv
  head -4 profiles/${TAG}_${CFG}_kernel_stats.csv | cut -c1-200
done
