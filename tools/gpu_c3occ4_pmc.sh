# C3 HBM traffic of the 4-wave instance of the wave kernel (DG_WAVE_OCC=4), FETCH and WRITE in separate passes
set -o pipefail
ROOT=$(pwd); O=gpurun_out/occ4; mkdir -p $O
export DG_WAVE_OCC=4
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --no-e2e > $O/c3_bench.json 2> $O/c3_bench.err || { tail -5 $O/c3_bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/$O/pmcf_c3 -o run -- python3 $ROOT/bench.py --config c3 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/pmcf_c3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/$O/pmcw_c3 -o run -- python3 $ROOT/bench.py --config c3 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $ROOT/$O/pmcw_c3.log 2>&1 || exit 1
echo done
