set -o pipefail
export DG_ALLOW_STALE=1
for v in "" _w5 _w5b; do
timeout -k 10 120 env DG_LIB_PATH=dynamicgo_amd/libdgj2t$v.so python -u tools/wvtime.py 2>&1 | grep us/step || exit 1
done
