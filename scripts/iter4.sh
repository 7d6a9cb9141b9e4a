cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/wlm_check.sh || exit $?
bash scripts/probe_ab.sh ./tools/wlm_probe_old ./tools/wlm_probe 1193 12800 256 2 > gpurun_out/iter_probe_ab.log 2>&1 || exit $?
cat gpurun_out/iter_probe_ab.log
timeout -k 5 60 ./tools/wlm_probe 1193 12800 256 | tail -9
