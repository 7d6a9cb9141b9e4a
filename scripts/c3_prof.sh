# c3 wide-path breakdown: kernel trace, HBM counters, SQ counters (ws_ab.py, B3 default)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3kt -o run -- python3 tools/ws_ab.py --variants B3=1 --reps 3 > gpurun_out/c3kt.log 2>&1 || exit $?
bash scripts/pmc_pass.sh c3fetch "FETCH_SIZE" "k_wide" python3 tools/ws_ab.py --variants B3=1 --reps 1 || exit $?
bash scripts/pmc_pass.sh c3write "WRITE_SIZE" "k_wide" python3 tools/ws_ab.py --variants B3=1 --reps 1 || exit $?
bash scripts/pmc_pass.sh c3sq1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" "k_wide_l1s|k_wide_last_ws" python3 tools/ws_ab.py --variants B3=1 --reps 1 || exit $?
echo done
