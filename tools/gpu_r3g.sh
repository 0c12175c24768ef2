# GPU tests (all), smoke, then the C3 wave-kernel profile
set -o pipefail
T=${TAG:-r3g}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -60 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=$T bash tools/gpu_c3prof.sh
