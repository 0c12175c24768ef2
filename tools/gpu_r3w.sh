# t2j: word-wise f64toa digits + walker token ring -- tests, phase profile, bench
set -o pipefail
O=gpurun_out/r3ag
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_t2j.py > $O/t2j_tests.log 2>&1 || { tail -30 $O/t2j_tests.log; exit 1; }
tail -2 $O/t2j_tests.log
DG_ALLOW_STALE=1 DG_LIB_PATH=$(pwd)/dynamicgo_amd/libdgj2t_t2wprof.so timeout -k 10 200 python -u tools/t2wprof.py > $O/t2wprof.log 2>&1 || { tail -20 $O/t2wprof.log; exit 1; }
cat $O/t2wprof.log
for c in t2j-c3 t2j-c2; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/$c.json 2> $O/$c.err || { tail -20 $O/$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'])"
done
echo done
