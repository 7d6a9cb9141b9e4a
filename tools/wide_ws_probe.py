"""Diagnostics: does the wide forward (k_wide_bits -> k_wide_l1s -> k_wide_last_ws, pass overlap)
depend on the contents of a fresh caller workspace?  One thread, one stream: the same forward
into workspaces pre-filled with zeros / 0x7F bytes / 0xFF bytes (NaN) / random bytes, with the
pass overlap on and off, each compared bitwise with a first forward.  Prints one line per case."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_gpu_coverage import _wide_plan  # noqa: E402
from bikg_graph_explainability_public_amd import engine  # noqa: E402

DEV = torch.device("cuda:0")


def main():
    plan = _wide_plan()
    N = plan.cols
    e = engine
    bits = e.sample_shapley(41, 96, N, DEV)
    ref = plan.forward(bits).clone()
    torch.cuda.synchronize()
    nb = plan.workspace_bytes(96)
    fills = {"zero": lambda t: t.zero_(), "x7f": lambda t: t.fill_(0x7F), "xff": lambda t: t.fill_(0xFF),
             "rand": lambda t: t.random_(0, 256)}
    for ov in ("1", "0"):
        os.environ["XPG_WIDE_OVERLAP"] = ov
        for name, fn in fills.items():
            ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
            fn(ws)
            torch.cuda.synchronize()
            out = torch.empty_like(ref)
            plan.forward(bits, out=out, workspace=ws)
            torch.cuda.synchronize()
            same = torch.equal(out, ref)
            d = (out - ref).abs()
            nbad = int((d > 0).sum()) if not same else 0
            print(f"overlap={ov} fill={name}: equal={same} mismatches={nbad} "
                  f"max|d|={float(torch.nan_to_num(d, nan=1e30).max()):.3g}", flush=True)
    os.environ.pop("XPG_WIDE_OVERLAP", None)


if __name__ == "__main__":
    main()
