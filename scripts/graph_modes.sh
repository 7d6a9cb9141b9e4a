cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for mode in ${MODES:-pipe graph split eager}; do
  extra=""
  [ $mode = split ] && export XPG_BENCH_SPLIT_GRAPH=1 || unset XPG_BENCH_SPLIT_GRAPH
  [ $mode = pipe ] && export XPG_BENCH_PIPE=1 || export XPG_BENCH_PIPE=0
  [ $mode = eager ] && extra="--no-graph"
  timeout -k 10 300 python -u bench.py --sections headline --no-cpu-baseline --steps ${STEPS:-50} $extra > gpurun_out/gm_$mode.log 2>&1 || { tail -20 gpurun_out/gm_$mode.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/gm_$mode.log').read().strip().split('\n')[-1]); print('$mode', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'check', d['graph_check_max_abs_diff'], d['config']['launch'][:40])"
done
