"""Diagnostic (not part of the product): the rows forward on the c2 headline plan and the c3
node_prediction plan — mean time per call over 20 calls and a hash of the outputs (an A/B of two
library builds gives the same hash when the outputs are bitwise equal).

    XPG_LIB=<lib> python tools/rows_ab.py
"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bikg_graph_explainability_public_amd import engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    sys.argv = sys.argv[:1]
    args = bench.parse()
    for name, build, rows in (("c2", bench.build_c2, 12800), ("c3node", bench.WORKLOADS["c3node"]["build"], 25600)):
        arch, sub_feat, sub_ei, q, plan = build(args, dev)
        bits = engine.sample_shapley(7, rows, plan.cols, dev)
        for _ in range(3):
            y = plan.forward(bits)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            y = plan.forward(bits)
        b.record()
        torch.cuda.synchronize()
        h = hashlib.sha1(y.cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"{name:7s} rows {rows}: {a.elapsed_time(b) / 20 * 1e3:8.1f} us per forward, y hash {h}", flush=True)


if __name__ == "__main__":
    main()
