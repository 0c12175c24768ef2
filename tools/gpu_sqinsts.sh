# instructions per message and wave-cycle breakdown (SQ counters; one PMC pass each)
# usage: O=gpurun_out/r5a CONFIGS="c2 c2s" [PASSES="insts cycles lds vmem"] bash tools/gpu_sqinsts.sh
set -o pipefail
O=${O:-gpurun_out/r5a}
CONFIGS=${CONFIGS:-"c3 t2j-c3"}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in $CONFIGS; do
  for pass in ${PASSES:-insts cycles}; do
    case $pass in
      insts) PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" ;;
      cycles) PMC="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY" ;;
      lds) PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES" ;;
      vmem) PMC="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES" ;;
    esac
    timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d $O/sq_${pass}_$c -o run -- python3 -u bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --inflight 1 > $O/sq_${pass}_$c.log 2>&1 || { tail -20 $O/sq_${pass}_$c.log; exit 1; }
  done
done
find $O -name "*counter_collection.csv"
