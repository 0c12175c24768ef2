# instruction-cache counters per kernel (one PMC pass per config)
set -o pipefail
O=${O:-gpurun_out/r5c}
CONFIGS=${CONFIGS:-"c2 c3"}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in $CONFIGS; do
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH --kernel-trace --output-format csv -d $O/ic_$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/ic_$c.log 2>&1 || { tail -20 $O/ic_$c.log; exit 1; }
done
find $O -name "*counter_collection.csv"
