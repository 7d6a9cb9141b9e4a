"""Shapley sampler (k_shapley) bandwidth by row alignment: S = 1M columns (31,250 words per row:
rows 8-B aligned, two dwordx2 stores per lane) against S = 1,000,064 (31,252 words: 16-B aligned,
one dwordx4 store) at 25,600 rows, the c3 graph_prediction shape.  Diagnostics only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bikg_graph_explainability_public_amd import engine

dev = torch.device("cuda", 0)
R = 25_600
for S in (1_000_000, 1_000_064, 1_000_000, 1_000_064):
    W = (S + 31) // 32
    engine.sample_shapley(1, R, S, dev, with_counts=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(5):
        engine.sample_shapley(2 + i, R, S, dev, with_counts=True)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    print(f"S={S} words={W} words%4={W % 4}: {ms:.3f} ms, {R * W * 4 / ms / 1e6:.0f} GB/s", flush=True)
