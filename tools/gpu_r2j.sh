set -o pipefail
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_ANY,SQ_INSTS_SMEM,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT"
bash tools/gpu_pmc.sh r2j_flat "$P1" "$P2" -- --config c2 --steps 3 --warmup 1 --no-e2e || exit $?
DG_NO_FLAT=1 bash tools/gpu_pmc.sh r2j_small "$P1" "$P2" -- --config c2 --steps 3 --warmup 1 --no-e2e || exit $?
