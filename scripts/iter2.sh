# layer-2 A/B + surrogate-fit chain A/B (old vs new probe binaries) with per-kernel times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ws_ab.py --variants "B3=0;B3=1;B3=1,DBG=16;B3=1,DBG=32" > gpurun_out/iter_ab.log 2>&1; rc=$?
cat gpurun_out/iter_ab.log
[ $rc -eq 0 ] || exit $rc
bash scripts/probe_ab.sh ./tools/wlm_probe_old ./tools/wlm_probe 1193 12800 256 3 > gpurun_out/iter_probe_ab.log 2>&1 || exit $?
cat gpurun_out/iter_probe_ab.log
for b in wlm_probe wlm_probe_old; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$b -o run -- ./tools/$b 1193 12800 256 > gpurun_out/prof_$b.log 2>&1 || exit $?
done
echo probes profiled
