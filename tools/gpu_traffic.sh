# HBM traffic per launch, per config: FETCH_SIZE, WRITE_SIZE and the L2 read
# requests by size (TCC_EA0_RDREQ_32B/_64B/_128B), each its own PMC pass
# (MI355X_MICROARCH.md: <= 4 TCC counters per pass; FETCH_SIZE uses 3)
# usage: O=gpurun_out/r5x CONFIGS="c2 c3" bash tools/gpu_traffic.sh
set -o pipefail
O=${O:-gpurun_out/traffic}
mkdir -p $O
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
kern() { case $1 in c1|c2|c2s|c2x) echo j2t_flat_kernel;; c3|c4|c5) echo j2t_wave_kernel;; t2j-c2) echo t2j_kernel;; t2j-c3) echo t2j_wave_kernel;; esac; }
for c in ${CONFIGS:-c2}; do
  if [ $c = c5 ]; then
    # the 1M-message batch is generated once, outside the profiler (a fork
    # pool under rocprofv3 did not finish in 120 s, r6z), and mapped by the
    # profiled runs from /dev/shm (bench.py DG_C5_CACHE)
    timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; bench.c5_shared_arena(1 << 20, 45, 1.0, bench.gen_workers())" || exit 1
    export DG_C5_CACHE=1
  fi
  i=0
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/$O/tr_${c}_$i -o run -- python3 -u $ROOT/bench.py --config $c --steps ${TR_STEPS:-2} --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $ROOT/$O/tr_${c}_$i.log 2>&1 || { tail -20 $ROOT/$O/tr_${c}_$i.log; exit 1; }
  done
  python3 $ROOT/tools/traffic.py $ROOT/$O/tr_${c}_1/run_counter_collection.csv $ROOT/$O/tr_${c}_2/run_counter_collection.csv $(kern $c) $ROOT/$O/traffic_$c.json $ROOT/$O/tr_${c}_3/run_counter_collection.csv > /dev/null || exit 1
  python3 -c 'import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d["hbm_bytes_per_launch"],d.get("hbm_bytes_per_launch_by_request_size"))' $ROOT/$O/traffic_$c.json $c
  if [ $c = c5 ]; then
    python3 -c "import sys; sys.path.insert(0, '$ROOT'); import bench; bench.release_c5_cache()"
    unset DG_C5_CACHE
  fi
done
