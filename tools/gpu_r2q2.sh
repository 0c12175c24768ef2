set -o pipefail
export DG_ALLOW_STALE=1
for v in "" _sp2 _sp4 _sp8; do
timeout -k 10 300 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u bench.py --config t2j-c3 --no-cpu-baseline --steps 5 > gpurun_out/r2q2$v.json 2> gpurun_out/r2q2$v.err || { tail -20 gpurun_out/r2q2$v.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2q2$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['config'].get('ok_msgs_rank0'))"
timeout -k 10 300 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u bench.py --config t2j-c2 --no-cpu-baseline --steps 10 > gpurun_out/r2q2c2$v.json 2> gpurun_out/r2q2c2$v.err || { tail -20 gpurun_out/r2q2c2$v.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r2q2c2$v.json').read().strip().splitlines()[-1]);print('c2 $v',d['value'],d['ms_per_step'])"
done
