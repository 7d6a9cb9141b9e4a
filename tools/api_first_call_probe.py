"""Diagnostic (not part of the product): which host call of Explainer.run's fit phase takes the
time on a query's first call (c2 workload, device sampler, times = 10).  Every native call
(`_lib.call`), the fit workspace allocation and the status read are timed on the host; the run's
phase clock gives host / device ms per phase.

    python tools/api_first_call_probe.py [--times 10]
"""
import argparse
import collections
import gc
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bikg_graph_explainability_public_amd import _lib, engine  # noqa: E402
from bikg_graph_explainability_public_amd.explainer import Explainer  # noqa: E402
from bikg_graph_explainability_public_amd.nn import ConvStack  # noqa: E402

LOG = []


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        r = fn(*a, **k)
        LOG.append((name, (time.perf_counter() - t0) * 1e3))
        return r
    return w


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--times", type=int, default=10)
    p.add_argument("--queries", default="8,9,10,11,12,13,10,14")
    args = p.parse_args()
    dev = torch.device("cuda", 0)
    gc_t = {}

    def gc_cb(phase, info):  # Python's cyclic collections, timed
        if phase == "start":
            gc_t["t"] = time.perf_counter()
        else:
            LOG.append((f"gc gen{info['generation']}", (time.perf_counter() - gc_t["t"]) * 1e3))
    gc.callbacks.append(gc_cb)
    orig_call = _lib.call

    def call(name, *a):
        t0 = time.perf_counter()
        orig_call(name, *a)
        LOG.append((name, (time.perf_counter() - t0) * 1e3))
    _lib.call = call
    engine.call = call
    engine._workspace = timed("_workspace", engine._workspace)
    engine.check_fit_status = timed("check_fit_status", engine.check_fit_status)
    g = torch.Generator().manual_seed(0)
    n, e, f = 100_000, 1_000_000, 64
    feat = torch.randn((n, f), generator=g)
    ei = torch.randint(0, n, (2, e), generator=g)
    torch.manual_seed(0)
    arch = ConvStack("gcn", [f, 64, 64], [64, 1]).eval()
    params = {"seed": 1, "interpret_samples": 256, "epochs": 50, "optimizer": "adam", "lr": 0.01,
              "lr_patience": 10, "l1_lambda": 1e-4, "mask_sampler": "device"}
    exp = Explainer(feat.to(dev), ei.to(dev), arch, params, [str(i) for i in range(n)])
    if os.environ.get("PROBE_GC_FREEZE") == "1":  # the inputs (100k names ...) out of the collector's way
        gc.freeze()
    for q in args.queries.split(","):
        LOG.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        exp.run(q, args.times)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        ph = exp.last_run["phases"].times()
        print(f"run({q}): {wall:.2f} ms S={exp.last_run['S']} phases host/device "
              f"{ {k: (round(v['host_ms'], 2), round(v['device_ms'], 2)) for k, v in ph.items() if isinstance(v, dict)} }",
              flush=True)
        agg = collections.defaultdict(lambda: [0, 0.0])
        for name, ms in LOG:
            agg[name][0] += 1
            agg[name][1] += ms
        top = sorted(agg.items(), key=lambda kv: -kv[1][1])[:8]
        print("   calls (n, host ms): " + ", ".join(f"{k} {v[0]} {v[1]:.2f}" for k, v in top), flush=True)


if __name__ == "__main__":
    main()
