"""Diagnostic: k-hop extraction time on the c3 graph (1M nodes, 10M edges, L+1 = 3 hops),
HIP (`engine.khop_subgraph`) vs the numpy restatement (oracle, host cores)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from bikg_graph_explainability_public_amd import engine  # noqa: E402

N, E, hops, seed = 1_000_000, 10_000_000, 3, 7
dev = torch.device("cuda", 0)
ei = torch.randint(0, N, (2, E), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
for _ in range(3):
    out = engine.khop_subgraph(seed, hops, ei, N)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
a.record()
for _ in range(20):
    out = engine.khop_subgraph(seed, hops, ei, N)
b.record()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 20
print(f"hip khop: {a.elapsed_time(b) / 20:.3f} ms/call (events)  {wall * 1e3:.3f} ms wall  "
      f"|subset|={out[0].numel()} kept={out[1].shape[1]}")
h = ei.cpu().numpy()
t0 = time.perf_counter()
o = oracle.k_hop_subgraph(seed, hops, h, N)
print(f"numpy khop: {(time.perf_counter() - t0) * 1e3:.1f} ms  |subset|={o[0].size}")
