# r4n: t2j wave kernel beside the lane pass (DG_T2J_OVERLAP 1 vs 0)
set -o pipefail
O=gpurun_out/r4n
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_t2j.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"],d["config"].get("serial_gbs"))'
for ov in 1 0; do
  for c in t2j-c3 t2j-c2; do
    DG_T2J_OVERLAP=$ov timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $O/${c}_$ov.json 2> $O/${c}_$ov.err || { tail -20 $O/${c}_$ov.err; exit 1; }
    python -c "$J" $O/${c}_$ov.json
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_t3 -o run -- python3 -u bench.py --config t2j-c3 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/kt_t3.log 2>&1 || { tail -20 $O/kt_t3.log; exit 1; }
find $O -name "*kernel_stats.csv"
