set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline > gpurun_out/hb_base_$r.log 2>&1 || exit $?
XPG_BENCH_FIT_DEPTH=1 timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline --repeats 2 --steps 10 > gpurun_out/hb_r2l1_$r.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline --repeats 2 --steps 10 > gpurun_out/hb_r2l2_$r.log 2>&1 || exit $?
XPG_BENCH_FIT_DEPTH=1 timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline --repeats 4 --steps 8 > gpurun_out/hb_r4l1_$r.log 2>&1 || exit $?
done
