# A/B of two library builds on the headline section, alternating on one box:
# tools/libxpgnn_base.so (the build to compare against) and the in-tree library
set -e
for r in 1 2 3; do
  XPG_LIB=tools/libxpgnn_base.so timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline > gpurun_out/hab_base_$r.log 2>&1
  timeout -k 10 200 python bench.py --sections headline --no-cpu-baseline > gpurun_out/hab_new_$r.log 2>&1
done
