#!/bin/bash
# layer-2 memory-path counters (TLB, L1->L2 read latency, TA stalls, L2 hits), one pass each,
# on one 32-row c3 pass (tools/ws_ab.py --variants B3=1 --reps 1)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P="python3 tools/ws_ab.py --variants B3=1 --reps 1"
R="k_wide_l1s|k_wide_last_ws"
bash scripts/pmc_pass.sh tlb "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" "$R" $P || exit $?
bash scripts/pmc_pass.sh lat "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "$R" $P || exit $?
bash scripts/pmc_pass.sh l2 "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "$R" $P || exit $?
