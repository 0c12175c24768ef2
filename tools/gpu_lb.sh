set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5s; mkdir -p $O
for lb in 1 16; do
  DG_LIST_BLOCKS=$lb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lb$lb -o run -- python3 -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/lb$lb.log 2>&1 || { tail -20 $O/lb$lb.log; exit 1; }
  tail -1 $O/lb$lb.log | cut -c1-200
done
