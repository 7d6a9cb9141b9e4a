for nb in 1024 2048 4096 8192 16384; do XPG_COMM_BLOCKS=$nb bash scripts/gpu_check.sh prof_c5 > /dev/null && python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_c5/run_kernel_stats.csv')))
print($nb, [ (r['Name'][:40], round(float(r['AverageNs'])/1e3,1)) for r in rows if 'k_communities' in r['Name']])
" || exit 1; done
