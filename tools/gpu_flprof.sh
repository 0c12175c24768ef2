# flat kernel phase / field / stage profiles (instrumented variant libraries from tools/build_variants.py)
set -o pipefail
O=${O:-gpurun_out/flprof}
mkdir -p $O
for c in ${CONFIGS:-c2}; do
  DG_LIB_PATH=dynamicgo_amd/libdgj2t_flprof.so DG_ALLOW_STALE=1 timeout -k 10 120 python tools/flprof.py $c > $O/phases_$c.txt 2>&1 || exit 1
  DG_LIB_PATH=dynamicgo_amd/libdgj2t_flpf.so DG_ALLOW_STALE=1 timeout -k 10 120 python tools/flprof.py $c --fields > $O/fields_$c.txt 2>&1 || exit 1
  DG_LIB_PATH=dynamicgo_amd/libdgj2t_flpg.so DG_ALLOW_STALE=1 timeout -k 10 120 python tools/flprof.py $c --stages > $O/stages_$c.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/*.txt
