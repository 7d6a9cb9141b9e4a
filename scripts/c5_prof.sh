#!/bin/bash
# c5 forward-kernel counters (k_agg_l1_rows / k_agg / k_dense), one PMC pass each, on the c5 bench
# section (3 jobs)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P="python3 bench.py --sections c5 --no-cpu-baseline"
R="k_agg|k_dense"
bash scripts/pmc_pass.sh ${C5TAG:-c5}sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM" "$R" $P || exit $?
bash scripts/pmc_pass.sh ${C5TAG:-c5}sq2 "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS" "$R" $P || exit $?
bash scripts/pmc_pass.sh ${C5TAG:-c5}fetch "FETCH_SIZE" "$R" $P || exit $?
bash scripts/pmc_pass.sh ${C5TAG:-c5}write "WRITE_SIZE" "$R" $P || exit $?
bash scripts/pmc_pass.sh ${C5TAG:-c5}l2 "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "$R" $P || exit $?
bash scripts/pmc_pass.sh ${C5TAG:-c5}lat "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "$R" $P || exit $?
