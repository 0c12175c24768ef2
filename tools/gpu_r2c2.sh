set -o pipefail
timeout -k 10 200 env DG_ALLOW_STALE=1 DG_LIB_PATH=dynamicgo_amd/libdgj2t_wprof.so python -u tools/wprof.py c3 > gpurun_out/r2c2_wprof.log 2>&1 || { cat gpurun_out/r2c2_wprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r2c2_wprof.log
bash tools/gpu_pmc.sh r2c2_pmc "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT" "FETCH_SIZE WRITE_SIZE" -- --config c3 --no-e2e --steps 3 --warmup 1 > gpurun_out/r2c2_pmc.txt 2>&1 || { tail -20 gpurun_out/r2c2_pmc.txt; exit 1; }
grep -A10 "wave_kernel" gpurun_out/r2c2_pmc.txt
