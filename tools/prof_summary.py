"""Print a compact per-kernel table from a rocprofv3 *_kernel_stats.csv (diagnostic helper)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:top]:
    n = r["Name"]
    m = re.search(r"(k_\w+(<[^>]*>)?)", n)
    n = m.group(1) if m else n.split("(")[0][-48:]
    print(f"{n:48s} calls={r['Calls']:>6} avg_us={float(r['AverageNs']) / 1e3:10.2f} "
          f"total_ms={float(r['TotalDurationNs']) / 1e6:9.3f} {float(r['Percentage']):6.2f}%")
