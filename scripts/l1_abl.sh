# c5 layer-1 ablation (timing only; XPG_L1_DBG changes the results): 0 full, 1 no keep loads,
# 2 self row for every source (scalar-cache hits), 3 both
for d in 0 1 2 3 0; do XPG_L1_DBG=$d bash scripts/gpu_check.sh prof_c5 > /dev/null && python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_c5/run_kernel_stats.csv')))
print('XPG_L1_DBG=$d', [(r['Name'][:40], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'l1_rows' in r['Name']])
" || exit 1; done
