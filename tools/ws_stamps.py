"""Diagnostic (not part of the product): where the warp-specialised layer 2 (k_wide_last_ws)
spends its cycles, per wave role, on the c3 full-graph pass.  Needs the stamps build:

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -fPIC -shared -DXPG_WIDE_STAMPS \\
        -o tools/libxpgnn_stamps.so bikg_graph_explainability_public_amd/csrc/xpgnn.hip
    XPG_LIB=$PWD/tools/libxpgnn_stamps.so python tools/ws_stamps.py [--variants "B3=1;B3=1,SORT=0"]

Prints, per wave of the workgroup, the average s_memtime cycles per target interval in each
phase (the stamps' own cost included), averaged over all workgroups.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bikg_graph_explainability_public_amd import _lib, engine, pipeline  # noqa: E402
from bikg_graph_explainability_public_amd.nn import ConvStack  # noqa: E402
from ws_ab import set_env  # noqa: E402

GATHER = ("barrier", "rows wait+sum", "in-place rest", "own row", "pf loads", "mean+split+store",
          "pf list hdr", "pf slots")
MFMA = ("barrier", "index chain", "logit out", "products", "epilogue")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--nodes", type=int, default=1_000_000)
    p.add_argument("--edges", type=int, default=10_000_000)
    p.add_argument("--feat", type=int, default=128)
    p.add_argument("--variants", default="B3=1")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    lib.xpg_debug_wide_stamps.argtypes = [ctypes.c_void_p]
    lib.xpg_debug_wide_stamps.restype = ctypes.c_int
    g = torch.Generator().manual_seed(0)
    N, E, F = args.nodes, args.edges, args.feat
    feat = torch.randn((N, F), generator=g).to(dev)
    ei = torch.randint(0, N, (2, E), generator=g).to(dev)
    torch.manual_seed(0)
    arch = ConvStack("sage", [F, F, F], [F, 1]).eval().to(dev)
    plan = pipeline.build_plan(arch, feat, ei, list(range(N)))
    bits = engine.sample_shapley(13, 32, N, dev)
    for spec in args.variants.split(";"):
        set_env(spec)
        plan.forward(bits)
        torch.cuda.synchronize()
        plan.forward(bits)
        torch.cuda.synchronize()
        buf = np.zeros((512, 16, 8), dtype=np.uint64)
        _lib.check(lib.xpg_debug_wide_stamps(buf.ctypes.data))
        wg = buf.sum(axis=2) > 0
        nwg = int(wg[:, 0].sum())
        ntgt = N / max(1, nwg)  # targets per workgroup (persistent grid)
        print(f"[{spec}] {nwg} workgroups, {ntgt:.0f} targets each; cycles per target interval:")
        for w in range(12):
            v = buf[:nwg, w, :].astype(np.float64).mean(axis=0) / ntgt
            names = GATHER if w < 8 else MFMA
            role = f"gather w{w}" if w < 8 else ("logit+mfma w8" if w == 8 else ("index+mfma w11" if w == 11 else f"mfma w{w}"))
            cells = "  ".join(f"{n} {v[k]:7.0f}" for k, n in enumerate(names))
            print(f"  {role:14s} total {v.sum():7.0f} | {cells}", flush=True)
    set_env("")


if __name__ == "__main__":
    main()
