cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
for v in 1 0; do
  XPG_SIDE_STREAM=$v timeout -k 10 300 python -u bench.py --sections headline --no-cpu-baseline --steps 50 > gpurun_out/side_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/side_$v.log').read().strip().split('\n')[-1]); print('side=$v', round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['phases_ms'].items()})"
done
done
