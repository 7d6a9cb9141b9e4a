cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coverage.py -x -q --timeout 200 --timeout-method thread -k "wide or full_graph or hub or c3" > gpurun_out/iter_tests.log 2>&1; rc=$?
tail -3 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ws_ab.py --variants "B3=1;B3=1,DBG=48;B3=1,L1=gather" > gpurun_out/iter_ab.log 2>&1; rc=$?
cat gpurun_out/iter_ab.log
exit $rc
