# A/B of library variants on one box: kernel time of the flat-kernel configs, interleaved, 3 rounds
# usage: VARIANTS="libdgj2t libdgj2t_norm" CONFIGS="c2 c2s" bash tools/gpu_ab.sh
O=${O:-gpurun_out/ab}; mkdir -p $O
for rep in 1 2 3; do
for v in ${VARIANTS:-libdgj2t}; do
for c in ${CONFIGS:-c2}; do
  DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/$v.so timeout -k 10 120 python -u bench.py --config $c --no-cpu-baseline --no-e2e > $O/${v}_${c}_$rep.json 2> $O/${v}_${c}_$rep.err || { tail -5 $O/${v}_${c}_$rep.err; exit 1; }
  python -c 'import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],sys.argv[3],d["value"],d["roofline"]["kernel_ms"])' $O/${v}_${c}_$rep.json $v $c
done; done; done
