# c5: k_rows_no_edge rows per wave sweep + k_degree time (kernel stats of bench.py --sections c5)
for n in 1 2 4 8; do XPG_RNE_RPW=$n bash scripts/gpu_check.sh prof_c5 > /dev/null && python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_c5/run_kernel_stats.csv')))
print('XPG_RNE_RPW=$n', [(r['Name'][:40], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'no_edge' in r['Name'] or 'k_degree' in r['Name']])
" || exit 1; done
