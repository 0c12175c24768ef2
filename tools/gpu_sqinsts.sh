# instructions per message of the wave kernels (SQ_INSTS_*; one PMC pass each config)
set -o pipefail
O=gpurun_out/r4u
PMC=${PMC:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"}
TAG=${TAG:-sq_}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in c3 t2j-c3; do
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $O/$TAG$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/$TAG$c.log 2>&1 || { tail -20 $O/$TAG$c.log; exit 1; }
done
find $O -name "*counter_collection.csv"
