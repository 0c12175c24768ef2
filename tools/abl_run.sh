#!/bin/bash
# GPU-box script: C2/C3 ablate timings of the default build and abl/lib*.so variants.
set -o pipefail
for L in dynamicgo_amd/libdgj2t.so abl/lib*.so; do
  for C in c2 c3; do DG_LIB_PATH=$L timeout -k 10 180 python tools/ablate.py $C || exit 1; done
done
