"""SQ / GRBM counters per kernel from one rocprofv3 PMC pass, as JSON (profiles/sq_<section>.json).

    python tools/sq_json.py gpurun_out/sq_c3 > profiles/sq_c3.json

Reads the pass's `*counter_collection.csv`, sums each counter over the rows of one dispatch,
averages over the dispatches of each exact kernel instantiation, and derives (per
MI355X_MICROARCH.md, "DVFS give-back" and the s_memtime / PMC units row):
  clock_ghz  = GRBM_GUI_ACTIVE / 8 / dispatch duration   (GRBM is summed over the 8 XCDs)
  cycles     = GRBM_GUI_ACTIVE / 8                        (the kernel's shader-clock cycles)
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x cycles) (MFMA-pipe busy fraction of the chip:
               SQ_VALU_MFMA_BUSY_CYCLES counts MFMA cycles summed over the SIMDs, 32 per
               32x32x16 bf16 MFMA, 64 per 32x32x2 f32)
  wait_frac  = SQ_WAIT_ANY / SQ_WAVE_CYCLES               (waves parked on s_waitcnt / barriers)
SIMDs = 4 per CU x the agent's CU count (256 on MI355X; --cus overrides).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cus = next((int(a.split("=", 1)[1]) for a in sys.argv[1:] if a.startswith("--cus=")), 256)
    per = defaultdict(lambda: defaultdict(float))
    dur = {}
    names = {}
    for d in args:
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(fn, newline="")):
                key = (fn, row["Dispatch_Id"])
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
                dur[key] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
                names[key] = row["Kernel_Name"]
    by = defaultdict(list)
    for key, cs in per.items():
        by[names[key]].append((cs, dur[key]))
    out = {"_simds": 4 * cus, "_source": args}
    for name, recs in sorted(by.items()):
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].strip()
        counters = sorted({c for cs, _ in recs for c in cs})
        mean = {c: sum(cs.get(c, 0.0) for cs, _ in recs) / len(recs) for c in counters}
        sec = sum(t for _, t in recs) / len(recs)
        rec = {"kernel": name, "dispatches": len(recs), "duration_ms": sec * 1e3, "counters": mean}
        g = mean.get("GRBM_GUI_ACTIVE")
        if g:
            cycles = g / 8.0
            rec["cycles"] = cycles
            rec["clock_ghz"] = cycles / sec / 1e9 if sec > 0 else None
            if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
                rec["mfma_busy"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * cus * cycles)
        if mean.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in mean:
            rec["wait_frac"] = mean["SQ_WAIT_ANY"] / mean["SQ_WAVE_CYCLES"]
        out[short] = rec
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
