# full GPU suite, c3 A/B (layer-1 kernels), fit-chain A/B with per-kernel times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1; rc=$?
tail -4 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ws_ab.py --variants "B3=1;B3=1,L1=gather;B3=1,DBG=16" > gpurun_out/iter_ab.log 2>&1; rc=$?
cat gpurun_out/iter_ab.log
[ $rc -eq 0 ] || exit $rc
bash scripts/probe_ab.sh ./tools/wlm_probe_old ./tools/wlm_probe 1193 12800 256 2 > gpurun_out/iter_probe_ab.log 2>&1 || exit $?
cat gpurun_out/iter_probe_ab.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wlm_probe -o run -- ./tools/wlm_probe 1193 12800 256 > gpurun_out/prof_wlm_probe.log 2>&1 || exit $?
echo probe profiled
