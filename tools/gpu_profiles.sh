# round profiles: GPU suite, smoke, every bench line, kernel stats (rocprofv3 --stats)
# usage: O=gpurun_out/r5z bash tools/gpu_profiles.sh   (traffic: tools/gpu_traffic.sh)
set -o pipefail
O=${O:-gpurun_out/prof}
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"] and d["roofline"].get("kernel_ms"),(d.get("e2e_host") or {}).get("sweep_gbs"))'
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { tail -20 $O/c2_bench.err; exit 1; }
python -c "$J" $O/c2_bench.json
for c in ${CONFIGS:-c1 c2s c2x c3 c4 c5 t2j-c2 t2j-c3 agg}; do
  timeout -k 10 900 python -u bench.py --config $c > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c "$J" $O/${c}_bench.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c2 c3 c4 c5 t2j-c2 t2j-c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$c -o run -- python3 -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/kt_$c.log 2>&1 || { tail -20 $O/kt_$c.log; exit 1; }
done
find $O -name "*kernel_stats.csv"
