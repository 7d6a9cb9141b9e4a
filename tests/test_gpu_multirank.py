"""The sharded bench paths at world size 2, run by the driver's `pytest -m gpu` every round (the
8-GPU RCCL runs are the driver's SCALE job; a 1-GPU box rehearses the same code with gloo and
both ranks on cuda:0: XPG_BENCH_BACKEND=gloo XPG_BENCH_ONE_GPU=1).

`bench.py --gpus 2` starts its two ranks itself (torch.distributed.run child process); this test
starts bench.py as a child process of its own, so nothing here execs from a process that touched
the GPU.  Checked, per DESIGN.md §7:
* rank_layout.world == 2 on every section;
* the pipelined captured headline: replayed fits equal an eager step (graph_check) and every
  rank's all-gathered slot equals its own rows (exchange_check), bitwise;
* c3 full graph: the 512 north-star rows sharded in 32-row passes, the query columns gathered;
* c4 / c5: the rows of the forward sharded, logits + kernel weights all-gathered, fits split by
  repeat -> the mean / std result checksum equals a 1-rank run's bit for bit.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(gpus, sections, extra_env=None, timeout=110):
    env = dict(os.environ)
    env.update(extra_env or {})
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--sections",
           sections, "--steps", "4", "--warmup", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_rank_rehearsal_matches_one_rank():
    two = _bench(2, "headline,c3,c4,c5", {"XPG_BENCH_BACKEND": "gloo", "XPG_BENCH_ONE_GPU": "1"})
    assert two["n_gpus"] == 2 and two["rank_layout"]["world"] == 2
    assert two["rank_layout"]["backend"] == "gloo"
    assert two["graph_check_max_abs_diff"] == 0.0
    assert two["exchange_check_max_abs_diff"] == 0.0
    assert two["value"] > 0
    reg = two["regimes"]
    assert reg["c3_full_graph"]["samples_per_s"] > 0
    one = _bench(1, "c4,c5")
    for sec in ("hetero_c4", "c5_hetero"):
        assert reg[sec]["result_checksum"] == one["regimes"][sec]["result_checksum"], sec
