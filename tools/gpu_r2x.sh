set -o pipefail
export DG_FLAT=1 DG_ALLOW_STALE=1
for v in "" _stop1 _stop2 _nolicm _stop1n _stop2n; do
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u tools/fltime.py c2 2>&1 | grep us/step || exit 1
done
