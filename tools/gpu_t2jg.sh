# t2j JOut variants: the default pair stores vs 64-byte groups (libdgj2t_t2jg.so, -DDG_T2J_GROUPS=1)
set -o pipefail
O=${O:-gpurun_out/t2jg}; mkdir -p $O
DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/libdgj2t_t2jg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_t2j.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in libdgj2t libdgj2t_t2jg; do
  for c in t2j-c2 t2j-c3; do
    DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/$lib.so timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/${lib}_$c.json 2> $O/${lib}_$c.err || { tail -20 $O/${lib}_$c.err; exit 1; }
    python -c 'import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d["value"],d["ms_per_step"],d["roofline"]["kernel_ms"])' $O/${lib}_$c.json
  done
done
