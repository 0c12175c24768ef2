set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_flat.py -v --timeout 120 --timeout-method thread > gpurun_out/r2i_flat.log 2>&1
rc=$?
tail -15 gpurun_out/r2i_flat.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r2i_c2_flat.json 2> gpurun_out/r2i_c2_flat.err || exit $?
cat gpurun_out/r2i_c2_flat.json
DG_NO_FLAT=1 timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r2i_c2_noflat.json 2> gpurun_out/r2i_c2_noflat.err || exit $?
cat gpurun_out/r2i_c2_noflat.json
