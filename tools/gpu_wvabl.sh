# wave-kernel ablations on C3 (timing only: outputs are wrong by design)
set -o pipefail
for L in dynamicgo_amd/libdgj2t.so dynamicgo_amd/libdgj2t_wvabl4.so dynamicgo_amd/libdgj2t_wvabl8.so dynamicgo_amd/libdgj2t_wvabl16.so; do
  echo "== $L"; DG_LIB_PATH=$L DG_ALLOW_STALE=1 timeout -k 10 180 python tools/ablate.py c3 || exit 1
done
