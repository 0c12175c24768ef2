# flat kernel ablations under SQ counters: the full kernel, stop after the
# structure phase (stop1), no writes (stop2), no global stores (nostore)
# usage: O=gpurun_out/r5r bash tools/gpu_flabl.sh
set -o pipefail
O=${O:-gpurun_out/flabl}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
for v in ${VARIANTS:-full stop1 stop2 nostore}; do
  lib=dynamicgo_amd/libdgj2t_$v.so
  [ $v = full ] && lib=dynamicgo_amd/libdgj2t.so
  DG_ALLOW_STALE=1 DG_LIB_PATH=$lib timeout -k 10 60 python3 tools/flprof.py ${CFG:-c2} --plain > $O/t_$v.log 2>&1 || { tail -5 $O/t_$v.log; exit 1; }
  cat $O/t_$v.log | tail -1
  DG_ALLOW_STALE=1 DG_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $O/pmc_$v -o run -- python3 tools/flprof.py ${CFG:-c2} --plain > $O/pmc_$v.log 2>&1 || { tail -20 $O/pmc_$v.log; exit 1; }
done
