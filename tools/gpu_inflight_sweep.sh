# batches in flight for the timed steps (bench --inflight)
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"])'
for c in c2 t2j-c2 c3; do
  for k in 2 3 4; do
    timeout -k 10 300 python -u bench.py --config $c --steps 40 --warmup 5 --no-cpu-baseline --no-e2e --inflight $k > $O/${c}_$k.json 2> $O/${c}_$k.err || { tail -20 $O/${c}_$k.err; exit 1; }
    python -c "$J" $O/${c}_$k.json
  done
done
