cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "shapley or sampler or communit or wlm or fit or explainer or run or golden or c5 or queries or sharded or smoke or counts" > gpurun_out/graph_tests.log 2>&1; rc=$?
tail -3 gpurun_out/graph_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for v in "" "--no-graph"; do
  timeout -k 10 300 python -u bench.py --sections headline --no-cpu-baseline --steps 50 $v > gpurun_out/gb.log 2>&1 || { tail -20 gpurun_out/gb.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/gb.log').read().strip().split('\n')[-1]); print('$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['phases_ms'].items()})"
done
done
