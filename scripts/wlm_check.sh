# surrogate-fit changes: fit parity tests + the c2 headline bench (one GPU call)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "wlm or fit or explainer or run or golden or c5 or queries or sharded" > gpurun_out/wlm_tests.log 2>&1; rc=$?
tail -5 gpurun_out/wlm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --sections headline --no-cpu-baseline > gpurun_out/wlm_bench.log 2>&1; rc=$?
tail -2 gpurun_out/wlm_bench.log | cut -c1-1500
exit $rc
