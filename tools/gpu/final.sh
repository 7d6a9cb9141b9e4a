#!/bin/bash
# Round-end evidence on one box: full GPU suite, smoke, full bench line, rocprofv3 kernel stats of
# the bench (each step under its own limit; stop at the first fault / abort / time-out)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/final_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/final_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/final_bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/final_prof.log 2>&1 || exit $?
echo done
