# A/B of two library builds on the c3 wide pass (tools/ws_ab.py, B3 layer 2), alternating:
# tools/libxpgnn_base.so (the build to compare against) and the in-tree library; then the wide /
# c3 GPU tests on the in-tree library
set -e
for r in 1 2; do
  XPG_LIB=tools/libxpgnn_base.so timeout -k 10 200 python -u tools/ws_ab.py --variants "B3=1" --reps 5 > gpurun_out/wsab_base_$r.log 2>&1
  timeout -k 10 200 python -u tools/ws_ab.py --variants "B3=1" --reps 5 > gpurun_out/wsab_new_$r.log 2>&1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_coverage.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "wide or c3 or hub" > gpurun_out/wide_pk_tests.log 2>&1
