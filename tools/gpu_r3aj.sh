# t2j bench: 1 vs 2 batches in flight
set -o pipefail
O=gpurun_out/r3aj
mkdir -p $O
for c in t2j-c2 t2j-c3; do for d in 1 2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e --inflight $d > $O/${c}_$d.json 2> $O/${c}_$d.err || { tail -20 $O/${c}_$d.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/${c}_$d.json')); print('$c d=$d', d['value'], d['ms_per_step'], d['config']['serial_gbs'])"
done; done
