set -o pipefail
O=gpurun_out/${TAG:-r3k}
mkdir -p $O
DG_ALLOW_STALE=1 DG_LIB_PATH=$(pwd)/dynamicgo_amd/libdgj2t_t2wprof.so timeout -k 10 200 python -u tools/t2wprof.py > $O/t2wprof.log 2>&1 || { tail -20 $O/t2wprof.log; exit 1; }
cat $O/t2wprof.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_t2j.py -x -q --timeout 120 --timeout-method thread > $O/t2j_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/t2j_tests.log | tail -30; exit 1; }
tail -1 $O/t2j_tests.log
timeout -k 10 300 python -u bench.py --config t2j-c3 --no-cpu-baseline > $O/t2j-c3_bench.json 2> $O/t2j-c3_bench.err || { tail -20 $O/t2j-c3_bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/t2j-c3_bench.json').read().strip().splitlines()[-1]);print('t2j-c3',d['value'],d['ms_per_step'],d['roofline']['frac'])"
