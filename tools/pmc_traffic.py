"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write [OPS] > profiles/pmc_<section>.json

Reads the `*counter_collection.csv` of each pass, sums the counter over the rows of one dispatch
and averages over the dispatches of each kernel.  FETCH_SIZE / WRITE_SIZE are in KB
(rocprofv3 derived counters: TCC_EA0_RDREQ/WRREQ x 64 B / 1024).  Per MI355X_MICROARCH.md
(HBM section) FETCH_SIZE counts 128-B read requests at 64 B on gfx950, so the corrected read
bytes are 2 x FETCH_SIZE; WRITE_SIZE is taken as is.  Output: JSON {kernel: {dispatches,
fetch_kb_raw, write_kb, read_bytes, write_bytes, traffic_bytes}} per launch, plus
`"_ops": OPS` = the number of section operations (bench repeats / steps) the profiled run made,
so bench.py can turn dispatch totals into bytes per operation whatever its own step count.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pass_dir, counter):
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    per_dispatch = defaultdict(float)
    names = {}
    for fn in files:
        with open(fn, newline="") as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                key = (fn, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per_dispatch[key] += float(row["Counter_Value"])
                names[key] = row.get("Kernel_Name", "?")
    out = defaultdict(list)
    for key, v in per_dispatch.items():
        out[names[key]].append(v)
    return out


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    res = {}
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        rb = 2 * fk * 1024 if fk is not None else None
        wb = wk * 1024 if wk is not None else None
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()
        res[short] = {"kernel": name, "dispatches": max(len(f), len(w)), "fetch_kb_raw": fk,
                      "write_kb": wk, "read_bytes": rb, "write_bytes": wb,
                      "traffic_bytes": (rb or 0) + (wb or 0) if (rb is not None or wb is not None)
                      else None}
    if len(sys.argv) > 3:
        res["_ops"] = int(sys.argv[3])
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
