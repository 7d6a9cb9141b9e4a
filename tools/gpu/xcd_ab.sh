set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "forward or rows or parity or explainer or golden" > gpurun_out/xcd_tests.log 2>&1 || exit $?
for r in 1 2; do
  XPG_BENCH_FIT_DEPTH=1 timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline > gpurun_out/x_d1_$r.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline > gpurun_out/x_d2_$r.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --sections node_c3 --no-cpu-baseline > gpurun_out/x_nodec3.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/xtrace -o run -- python3 bench.py --sections headline --no-cpu-baseline --steps 20 > gpurun_out/xtrace.log 2>&1
