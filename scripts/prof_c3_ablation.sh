cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in 0 1 2 8; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/c3dbg$d -o run -- python3 tools/c3_probe.py --skip-a --rows-b 32 --dbg $d > gpurun_out/c3dbg$d.log 2>&1 || exit 1
  echo "dbg $d done"; grep "full forward" gpurun_out/c3dbg$d.log
done
