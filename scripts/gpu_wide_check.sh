# wide-path parity + full-graph timing (one GPU call)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "wide or full_graph or c2_scale or synthetic" > gpurun_out/wide_tests.log 2>&1 || { tail -30 gpurun_out/wide_tests.log; exit 1; }
tail -2 gpurun_out/wide_tests.log
timeout -k 10 200 python -u tools/c3_probe.py --skip-a --rows-b 32 --dbg ${DBG:-0} 2>&1 | grep "full forward"
