# Round profiles on one GPU box (run from the repo root under gpurun):
#   O=gpurun_out/r7z bash tools/gpu_profiles.sh
# Steps (each switchable; all on by default):
#   TESTS=1    the GPU suite (pytest -m gpu) and smoke()
#   BENCH=1    every bench line (CONFIGS), JSON under $O/<config>_bench.json
#   KSTATS=1   rocprofv3 --kernel-trace --stats of the serial leg (KCONFIGS)
#   TRAFFIC=1  HBM bytes per launch of the dominant kernel: FETCH_SIZE,
#              WRITE_SIZE and the L2 read requests by size, one PMC pass each
#              (MI355X_MICROARCH.md: <= 4 TCC counters per pass), then
#              tools/traffic.py -> $O/traffic_<config>.json (TCONFIGS)
#   SQ=0       SQ instruction / cycle counters (SQCONFIGS, PASSES="insts cycles lds vmem")
# C5's 1M-message batch is generated once outside the profiler and mapped by
# the profiled runs (bench.py DG_C5_CACHE): a fork pool under rocprofv3 did
# not finish in 120 s (r6z).
set -o pipefail
O=${O:-gpurun_out/prof}
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/$O
( while sleep 20; do echo "[hb $(date +%T)]" >> $ROOT/$O/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
cd $ROOT
J='import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d.get("roofline") or {};print(sys.argv[1],d["value"],d["ms_per_step"],r.get("kernel"),r.get("kernel_ms"),r.get("frac"),(d.get("e2e_host") or {}).get("value"))'
c5_cache() { timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; bench.c5_shared_arena(1 << 20, 45, 1.0, bench.gen_workers())" || exit 1; export DG_C5_CACHE=1; }
c5_release() { python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; bench.release_c5_cache()"; unset DG_C5_CACHE; }
kern() { case $1 in c1|c2|c2s|c2x) echo j2t_flat_kernel;; c3|c4|c5) echo j2t_wave_kernel;; t2j-c2) echo t2j_kernel;; t2j-c3) echo t2j_wave_kernel;; esac; }

if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
  tail -1 $O/gputest.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  for c in ${CONFIGS:-c2 c1 c2s c2x c3 c4 c5 t2j-c2 t2j-c3 agg}; do
    timeout -k 10 900 python -u bench.py --config $c > $O/${c}_bench.json 2> $O/${c}_bench.err || { tail -20 $O/${c}_bench.err; exit 1; }
    python -c "$J" $O/${c}_bench.json
  done
fi
cd /tmp && export TMPDIR=/tmp
if [ "${KSTATS:-1}" = 1 ]; then
  for c in ${KCONFIGS:-c2 c3 c4 c5 t2j-c2 t2j-c3}; do
    [ $c = c5 ] && c5_cache
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/kt_$c -o run -- python3 -u $ROOT/bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $ROOT/$O/kt_$c.log 2>&1 || { tail -20 $ROOT/$O/kt_$c.log; exit 1; }
    [ $c = c5 ] && c5_release
  done
  find $ROOT/$O -name "*kernel_stats.csv"
fi
if [ "${TRAFFIC:-1}" = 1 ]; then
  for c in ${TCONFIGS:-c2 c2s c2x c1 c3 c4 c5 t2j-c2 t2j-c3}; do
    [ $c = c5 ] && c5_cache
    i=0
    for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/$O/tr_${c}_$i -o run -- python3 -u $ROOT/bench.py --config $c --steps ${TR_STEPS:-2} --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $ROOT/$O/tr_${c}_$i.log 2>&1 || { tail -20 $ROOT/$O/tr_${c}_$i.log; exit 1; }
    done
    python3 $ROOT/tools/traffic.py $ROOT/$O/tr_${c}_1/run_counter_collection.csv $ROOT/$O/tr_${c}_2/run_counter_collection.csv $(kern $c) $ROOT/$O/traffic_$c.json $ROOT/$O/tr_${c}_3/run_counter_collection.csv > /dev/null || exit 1
    python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d["hbm_bytes_per_launch"],d.get("hbm_bytes_per_launch_by_request_size"))' $ROOT/$O/traffic_$c.json $c
    [ $c = c5 ] && c5_release
  done
fi
if [ "${SQ:-0}" = 1 ]; then
  for c in ${SQCONFIGS:-c2 c3}; do
    for pass in ${PASSES:-insts cycles}; do
      case $pass in
        insts) PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" ;;
        cycles) PMC="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY" ;;
        lds) PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES" ;;
        vmem) PMC="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES" ;;
      esac
      timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $ROOT/$O/sq_${pass}_$c -o run -- python3 -u $ROOT/bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $ROOT/$O/sq_${pass}_$c.log 2>&1 || { tail -20 $ROOT/$O/sq_${pass}_$c.log; exit 1; }
    done
  done
fi
echo profiles done
