# fit stamp probe: old vs new binary A/B, then the new one's phase stamps
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/probe_ab.sh ./tools/wlm_probe_old ./tools/wlm_probe 1193 12800 256 3 > gpurun_out/probe_cmp.log 2>&1 || exit $?
timeout -k 5 60 ./tools/wlm_probe 1193 12800 256 | tail -9 >> gpurun_out/probe_cmp.log || exit $?
cat gpurun_out/probe_cmp.log
