#!/bin/bash
# round-2 experiments: bench lines for configs / env variants, no CPU baseline.
# usage: bash tools/gpu_exp.sh <tag> "<ENV=.. ENV=..>|<config>|<steps>" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  IFS='|' read -r envs cfg steps <<< "$spec"
  echo "== $i: [$envs] $cfg" >&2
  env $envs timeout -k 10 240 python bench.py --config $cfg --steps ${steps:-10} --no-cpu-baseline --no-e2e > $OUT/e$i.json 2> $OUT/e$i.err || { echo "exp $i failed"; tail -5 $OUT/e$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$OUT/e$i.json').read().strip().splitlines()[-1])
print('$i', '[$envs]', '$cfg', 'GB/s', d['value'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'], 'exact', d['config']['exact_path_msgs_per_step'])
"
done
