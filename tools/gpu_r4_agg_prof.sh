# r4: where the aggregator's time goes: kernel trace + HIP API trace of the agg bench
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --config agg --steps 5 --warmup 2 --no-cpu-baseline > $O/agg.json 2> $O/agg.err || { tail -20 $O/agg.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o agg -- python3 bench.py --config agg --steps 3 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --runtime-trace --stats -d $O/rt -o agg -- python3 bench.py --config agg --steps 3 --warmup 1 --no-cpu-baseline > $O/rt.log 2>&1 || { tail -20 $O/rt.log; exit 1; }
find $O -name "*stats.csv" | head -20
