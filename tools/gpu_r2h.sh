set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_t2j.py -v --timeout 120 --timeout-method thread > gpurun_out/r2h_t2j.log 2>&1
rc=$?
tail -5 gpurun_out/r2h_t2j.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config t2j-c2 --steps 20 --warmup 3 > gpurun_out/r2h_bench_t2j_c2.json 2> gpurun_out/r2h_bench_t2j_c2.err || exit $?
cat gpurun_out/r2h_bench_t2j_c2.json
timeout -k 10 300 python -u bench.py --config t2j-c3 --steps 20 --warmup 3 > gpurun_out/r2h_bench_t2j_c3.json 2> gpurun_out/r2h_bench_t2j_c3.err || exit $?
cat gpurun_out/r2h_bench_t2j_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2h_prof_t2j_c2 -o prof -- python3 bench.py --config t2j-c2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r2h_prof.log 2>&1 || exit $?
find gpurun_out/r2h_prof_t2j_c2 -name "*stats*" | head
