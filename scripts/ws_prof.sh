# layer-2 limiter: XPG_WIDE_DBG ablation, then two SQ counter passes on the wide kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ws_ab.py --variants "B3=1;B3=1,DBG=16;B3=1,DBG=32;B3=1,DBG=48" > gpurun_out/ws_dbg.log 2>&1 || exit $?
cat gpurun_out/ws_dbg.log
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
bash scripts/pmc_pass.sh sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" "k_wide_l1s|k_wide_last_ws" python3 tools/ws_ab.py --variants B3=1 --reps 1 || exit $?
bash scripts/pmc_pass.sh sq2 "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" "k_wide_l1s|k_wide_last_ws" python3 tools/ws_ab.py --variants B3=1 --reps 1 || exit $?
