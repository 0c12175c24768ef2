# time wave-kernel variant libraries on C3 (tools/build_variants.py output), then C4/C5 through bench
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _licm5 _w5r256; do
    echo "run $r variant '$v'"
    DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t$v.so timeout -k 10 150 python -u tools/wvtime.py 2>&1 | grep us/step || exit 1
  done
done
for c in c4 c5; do
  for v in "" _w5r256; do
    echo "bench $c variant '$v'"
    DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t$v.so timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/wv_$c$v.json 2> gpurun_out/wv_$c$v.err || { tail -5 gpurun_out/wv_$c$v.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'],d['ms_per_step'])" gpurun_out/wv_$c$v.json
  done
done
