"""Diagnostic: per-kernel averages of every counter in one or more rocprofv3 PMC pass dirs
(sum over a dispatch's rows, mean over dispatches).

    python tools/pmc_table.py gpurun_out/c5usq1 gpurun_out/c5usq2 ... [--match k_agg]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "")
    table = defaultdict(lambda: defaultdict(list))
    for d in args:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            names = {}
            for row in csv.DictReader(open(fn, newline="")):
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = row["Kernel_Name"]
            for (disp, cn), v in per.items():
                table[names[disp]][cn].append(v)
    for kn, cs in table.items():
        if match not in kn:
            continue
        print(kn[:90])
        for cn in sorted(cs):
            vals = cs[cn]
            print(f"    {cn:36s} {sum(vals) / len(vals):16.4g}  (n={len(vals)})")


if __name__ == "__main__":
    main()
