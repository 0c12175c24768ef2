# time wave-kernel variant libraries on C3 (tools/build_variants.py output)
set -o pipefail
for r in 1 2; do
  for v in "" _r128m3584 _r128m2048 _f80 _f120; do
    DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t$v.so timeout -k 10 150 python -u tools/wvtime.py 2>&1 | grep us/step || exit 1
  done
done
