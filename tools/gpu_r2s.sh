set -o pipefail
export DG_FLAT=1
bash tools/gpu_pmc.sh r2s_flat "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" -- --no-e2e --steps 5 --warmup 1 > gpurun_out/r2s_flat.txt 2>&1 || { cat gpurun_out/r2s_flat.txt; exit 1; }
cat gpurun_out/r2s_flat.txt
