set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_exp.sh r2c "DG_WAVE_MIN=1000000 DG_SMALL_MPW=65|c3|3" "DG_WAVE_MIN=4096 DG_SMALL_MPW=65|c3|3" || exit 1
OUT=$PWD/gpurun_out/r2c; ROOT=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-e2e --steps 20 > $OUT/prof_c2.log 2>&1 || { tail $OUT/prof_c2.log; exit 1; }
find $OUT/prof_c2 -name "*kernel_stats.csv" -exec cat {} \;
