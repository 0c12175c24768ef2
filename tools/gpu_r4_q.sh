# r4q: round-end state -- GPU suite, smoke, default bench line, t2j lines (pair stores restored)
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
( while sleep 20; do echo "[hb $(date +%T)]" >> $O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"] and d["roofline"].get("kernel_ms"),d["config"].get("serial_gbs"),(d.get("e2e_host") or {}).get("sweep_gbs"))'
timeout -k 10 600 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { tail -20 $O/c2_bench.err; exit 1; }
python -c "$J" $O/c2_bench.json
for c in t2j-c2 t2j-c3; do
  timeout -k 10 400 python -u bench.py --config $c > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
  python -c "$J" $O/${c}_bench.json
done
