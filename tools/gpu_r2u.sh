set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2u_flat.log 2>&1 || { tail -30 gpurun_out/r2u_flat.log; exit 1; }
tail -2 gpurun_out/r2u_flat.log
for c in c2 c2s c2x; do
timeout -k 10 200 env DG_FLAT=1 python -u bench.py --config $c --no-e2e --no-cpu-baseline > gpurun_out/r2u_flat_$c.json 2>&1 || exit 1
python -c "import json,sys;d=json.loads(open('gpurun_out/r2u_flat_$c.json').read().strip().splitlines()[-1]);print('$c',d['value'],d['config']['per_rank_kernel_ms'],d['config']['exact_path_msgs_per_step'])"
done
timeout -k 10 120 env DG_FLAT=1 DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so python -u tools/flprof.py c2 > gpurun_out/r2u_flprof.log 2>&1 || exit 1
cat gpurun_out/r2u_flprof.log
