# r4r: C5 / C3 routing knobs by environment (wave_min, wave_occ, list_blocks)
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"])'
for e in "X=0" "DG_WAVE_MIN=256" "DG_WAVE_MIN=1024" "DG_WAVE_OCC=5" "DG_LIST_BLOCKS=64"; do
  for c in c5 c3; do
    env $e timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/${c}_${e}.json 2> $O/${c}_${e}.err || { tail -20 $O/${c}_${e}.err; exit 1; }
    python -c "$J" $O/${c}_${e}.json
  done
done
