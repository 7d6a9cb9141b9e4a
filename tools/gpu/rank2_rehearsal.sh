# N=2 rehearsal of bench.py's headline on ONE GPU (gloo, both ranks on cuda:0): pipelined and
# split graph modes, each checked against an eager step (graph_check_max_abs_diff)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for pipe in 1 0; do
  XPG_BENCH_PIPE=$pipe XPG_BENCH_BACKEND=gloo XPG_BENCH_ONE_GPU=1 timeout -k 10 300 \
    python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --sections headline --no-cpu-baseline --steps 20 > gpurun_out/r2_pipe$pipe.log 2>&1 || { tail -30 gpurun_out/r2_pipe$pipe.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r2_pipe$pipe.log') if l.startswith('{')][-1]); print('pipe=$pipe', d['n_gpus'], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'check', d['graph_check_max_abs_diff'], d['config']['launch'][:50])"
done
