"""The sharded bench paths at world size 2, run by the driver's `pytest -m gpu` every round (the
8-GPU RCCL runs are the driver's SCALE job; a 1-GPU box rehearses the same code with gloo and
both ranks on cuda:0: XPG_BENCH_BACKEND=gloo XPG_BENCH_ONE_GPU=1).

`bench.py --gpus 2` starts its two ranks itself (torch.distributed.run child process); this test
starts bench.py as a child process of its own, so nothing here execs from a process that touched
the GPU.  Checked, per DESIGN.md §7:
* rank_layout.world == 2 on every section;
* the pipelined captured headline: replayed fits equal an eager step (graph_check) and every
  rank's all-gathered slot equals its own rows (exchange_check), bitwise;
* c3 full graph: 80 rows sharded in 32-row passes (2 + a partial 1), the query-column logits
  gathered unevenly -> their checksum equals a 1-rank run's bit for bit;
* c4 / c5: the rows of the forward sharded, logits + kernel weights all-gathered, fits split by
  repeat -> the mean / std result checksum equals a 1-rank run's bit for bit.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(gpus, sections, extra_env=None, timeout=110, extra_args=()):
    env = dict(os.environ)
    env.update(extra_env or {})
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--sections",
           sections, "--steps", "4", "--warmup", "1", "--no-cpu-baseline"] + list(extra_args)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


REHEARSAL = {"XPG_BENCH_BACKEND": "gloo", "XPG_BENCH_ONE_GPU": "1"}


@pytest.mark.gpu
def test_bench_two_rank_rehearsal_matches_one_rank():
    two = _bench(2, "headline,c4,c5", REHEARSAL)
    assert two["n_gpus"] == 2 and two["rank_layout"]["world"] == 2
    assert two["rank_layout"]["backend"] == "gloo"
    assert two["graph_check_max_abs_diff"] == 0.0
    assert two["exchange_check_max_abs_diff"] == 0.0
    assert two["value"] > 0
    reg = two["regimes"]
    one = _bench(1, "c4,c5")
    for sec in ("hetero_c4", "c5_hetero"):
        assert reg[sec]["result_checksum"] == one["regimes"][sec]["result_checksum"], sec


@pytest.mark.gpu
def test_bench_two_rank_c3_uneven_shard_matches_one_rank():
    """The north-star c3 full-graph section at world 2 with 80 mask rows = three 32-row passes,
    the last one partial: rank 0 forwards two passes (64 rows), rank 1 one partial pass (16
    rows), then the uneven all-gather of the query-column logits — bitwise equal to one rank
    forwarding all 80 rows (explainer.py:490-519: the rows are independent)."""
    rows = ["--c3-rows", "80"]
    two = _bench(2, "c3", REHEARSAL, timeout=170, extra_args=rows)
    one = _bench(1, "c3", timeout=120, extra_args=rows)
    c2, c1 = two["regimes"]["c3_full_graph"], one["regimes"]["c3_full_graph"]
    assert two["rank_layout"]["world"] == 2 and c2["rows"] == 80
    assert c2["rows_per_rank"] == 64  # rank 0's shard (rank 1: 16)
    assert c1["rows_per_rank"] == 80
    assert c2["logits_checksum"] == c1["logits_checksum"]


@pytest.mark.gpu
def test_bench_rccl_one_rank_rehearsal():
    """The RCCL code path on real hardware: a process group of ONE rank over RCCL
    (XPG_BENCH_RCCL1=1) takes every N-rank branch of the bench -- the headline's exchange
    staging and async all-gathers (all_gather_into_tensor on the "nccl" backend, a work handle
    whose wait() orders the current stream), the c3 uneven all-gather, the max over ranks -- so
    the collectives the driver's 8-GPU run uses are executed here, and give the 1-rank answers
    bit for bit (graph / exchange checks 0, c3 logits checksum equal to a plain 1-rank run's)."""
    rows = ["--c3-rows", "80"]
    r = _bench(1, "headline,c3", {"XPG_BENCH_RCCL1": "1"}, timeout=170, extra_args=rows)
    assert r.get("rccl1_rehearsal") is True
    assert r["rank_layout"]["backend"] == "nccl (RCCL)" and r["rank_layout"]["world"] == 1
    assert r["graph_check_max_abs_diff"] == 0.0
    assert r["exchange_check_max_abs_diff"] == 0.0
    assert r["value"] > 0
    one = _bench(1, "c3", timeout=120, extra_args=rows)
    assert r["regimes"]["c3_full_graph"]["logits_checksum"] == one["regimes"]["c3_full_graph"]["logits_checksum"]
