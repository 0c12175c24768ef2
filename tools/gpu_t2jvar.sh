# t2j variant libraries (LICM off, message spread) on t2j-c3 / t2j-c2
set -o pipefail
mkdir -p gpurun_out
for c in t2j-c3 t2j-c2; do
  for v in "" _t2jlicm _t2jlicm1 _t2jlicm4; do
    DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t$v.so timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/tv_$c$v.json 2> gpurun_out/tv_$c$v.err || { tail -5 gpurun_out/tv_$c$v.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'])" gpurun_out/tv_$c$v.json "$c$v"
  done
done
