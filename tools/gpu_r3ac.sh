# t2j copy-task size: 16/24 (HEAD) vs 32/48 vs 8/12
set -o pipefail
O=gpurun_out/r3ad
mkdir -p $O
for v in ch8 ch4 ch32 ch8; do
  if [ -n "$v" ]; then export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1; else unset DG_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --config t2j-c3 --no-cpu-baseline --no-e2e > $O/c3_$v.json 2> $O/c3_$v.err || { tail -20 $O/c3_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/c3_$v.json')); print('${v:-base}', d['value'], d['ms_per_step'])"
done
for v in ch4; do
  export DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t_$v.so DG_ALLOW_STALE=1
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_t2j.py > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; exit 1; }
  tail -1 $O/t_$v.log
done
