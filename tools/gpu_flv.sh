# time flat-kernel variant libraries on C2 (tools/build_variants.py output): VARIANTS="_a _b"
set -o pipefail
for r in 1 2; do
  for v in "" $VARIANTS; do
    echo -n "variant '$v' "
    DG_ALLOW_STALE=1 DG_LIB_PATH=$PWD/dynamicgo_amd/libdgj2t$v.so timeout -k 10 150 python -u tools/fltime_n.py ${SIZES:-65536} 2>&1 | grep us/step || exit 1
  done
done
