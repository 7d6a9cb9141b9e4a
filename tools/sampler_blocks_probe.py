"""Shapley sampler (k_shapley) time at the c3 graph_prediction shape (25,600 rows x 1M columns)
for several grid sizes (XPG_SHAPLEY_BLOCKS, diagnostics switch; -1 = one row per block, the
pre-round-6 launch) and a bitwise check that the rows do not depend on it.  Diagnostics only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bikg_graph_explainability_public_amd import engine  # noqa: E402

os.environ["XPG_DIAGNOSTICS"] = "1"
dev = torch.device("cuda", 0)
R, S = 25_600, 1_000_000
W = (S + 31) // 32
ref = None
for nb in ("-1", "0", "4096", "8192", "32768", "-1", "0"):
    os.environ["XPG_SHAPLEY_BLOCKS"] = nb
    b0, c0 = engine.sample_shapley(1, R, S, dev, with_counts=True)
    if ref is None:
        ref = (b0.clone(), c0.clone())
    same = torch.equal(b0, ref[0]) and torch.equal(c0, ref[1])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(5):
        engine.sample_shapley(2 + i, R, S, dev, with_counts=True)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    print(f"blocks={nb}: {ms:.3f} ms, {R * W * 4 / ms / 1e6:.0f} GB/s, same bits {same}", flush=True)
