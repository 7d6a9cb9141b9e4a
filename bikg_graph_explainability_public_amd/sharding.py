"""Multi-GPU sharding of the perturbation-scoring path.

One process per GPU (`torchrun`, RCCL through torch.distributed "nccl"; "gloo" for the CPU
tests).  The reference runs `times` independent repeats of R mask rows one after another
(explainer.py:490-532).  Here:

* the masked forward and KernelSHAP are row-independent, so the `times * R` rows are split in
  contiguous balanced shards (`shard_range`) and the per-row outputs (fp32 logits, fp64 kernel
  weights) are exchanged with one all-gather each (`gather_rows`);
* the surrogate fits are repeat-independent, so repeats are split the same way and the fitted
  weight vectors are exchanged with one all-gather (`gather_rows` on [times, S]).

Every rank ends with the same full tensors, so `weight_stacking` (mean / population std over
repeats) and the DataFrames are identical on every rank and identical to a single-GPU run.
torch.distributed's all_gather needs equal shard shapes: shards are padded to the largest one.
"""

import torch


def world_info(group=None):
    """(world_size, rank) of `group`, or (1, 0) when torch.distributed is not initialised."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _backend_device(t, group=None):
    """Collectives run on the device the backend supports: RCCL ("nccl") on the GPU, gloo on the
    host (gloo is the CPU test backend; its GPU-tensor support is partial)."""
    import torch.distributed as dist
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return t.device if t.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())


def sync_rng(group=None, src=0):
    """Make every rank's torch CPU generator equal to rank `src`'s (one broadcast of the state).

    Explainer.run draws the compat masks, the device samplers' seeds and the surrogates' initial
    weights from torch's CPU generator (the reference's RNG order).  Each rank draws the SAME
    values only if the generators agree, so a rank seeded differently (or `times > 1` without
    set_seed) would otherwise fit against another rank's masks.  After this call they agree."""
    import torch.distributed as dist
    world, _ = world_info(group)
    if world == 1:
        return
    state = torch.get_rng_state()
    buf = state.to(_backend_device(state, group))
    dist.broadcast(buf, src=dist.get_global_rank(group, src) if group is not None else src,
                   group=group)
    torch.set_rng_state(buf.cpu())


def checksum(t):
    """Order-sensitive int64 checksum of a tensor's bytes (position-weighted word sum)."""
    b = t.detach().contiguous().view(torch.uint8).reshape(-1)
    pad = (-b.numel()) % 4
    if pad:
        b = torch.cat([b, b.new_zeros(pad)])
    w = b.view(torch.int32).to(torch.int64)
    pos = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 1000003 + 1
    return int((w * pos).sum().item())


def assert_replicated(t, what, group=None):
    """Raise if `t` differs between ranks (compares checksums with one small all-gather)."""
    import torch.distributed as dist
    world, _ = world_info(group)
    if world == 1:
        return
    c = torch.tensor([checksum(t)], dtype=torch.int64)
    c = c.to(_backend_device(c, group))
    outs = [torch.empty_like(c) for _ in range(world)]
    dist.all_gather(outs, c, group=group)
    vals = [int(o.item()) for o in outs]
    if len(set(vals)) != 1:
        raise RuntimeError(f"{what} differ between ranks (checksums {vals}): every rank must draw "
                           "the same masks and initial weights")


def shard_range(n, world, rank):
    """Contiguous balanced split of n units: the first n % world ranks get one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    base, extra = divmod(int(n), world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local, n, group=None):
    """All-gather the row shards of an [n, ...] tensor split by `shard_range`.

    `local` holds this rank's rows (possibly zero of them); returns the full [n, ...] tensor on
    every rank, in global row order.  One collective, padded to the largest shard.
    """
    import torch.distributed as dist
    world, rank = world_info(group)
    if world == 1 or n == 0:
        if local.shape[0] != n:
            raise ValueError(f"expected {n} rows, got {local.shape[0]}")
        return local
    s, e = shard_range(n, world, rank)
    if local.shape[0] != e - s:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, its shard is {e - s}")
    cap = shard_range(n, world, 0)[1]
    dev = _backend_device(local, group)
    buf = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    buf[:e - s] = local.to(dev)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    parts = []
    for r in range(world):
        rs, re_ = shard_range(n, world, r)
        parts.append(outs[r][:re_ - rs])
    return torch.cat(parts, 0).to(local.device)


class _Done:
    """Handle of an exchange that already completed (gloo rehearsal)."""

    def wait(self):
        return True


def all_gather_async(out, inp, group=None):
    """out [world * n, ...] <- every rank's inp [n, ...] (equal shard sizes), rank-major, without
    a host sync: RCCL returns a work handle whose wait() makes the CURRENT stream wait for the
    exchange (the host never blocks), so a caller can overlap it with the next step and wait
    only before it overwrites `inp` or reads `out`.  gloo (CPU test backend; GPU tensors go
    through host copies): synchronous, returns a finished handle."""
    import torch.distributed as dist
    world, _ = world_info(group)
    if out.numel() != world * inp.numel():
        raise ValueError(f"all_gather_async: out holds {out.numel()} elements, expected "
                         f"{world} x {inp.numel()}")
    if dist.get_backend(group) == "gloo" and inp.device.type != "cpu":
        ob = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(ob, inp.cpu().contiguous(), group=group)
        out.copy_(ob)
        return _Done()
    return dist.all_gather_into_tensor(out, inp.contiguous(), group=group, async_op=True)


def gather_map(n, fn, group=None):
    """Run `fn(start, stop)` on this rank's shard of n units and all-gather the results.

    `fn` returns a tensor whose leading dimension is stop - start (it is called with an empty
    range on ranks that own no unit and must still return a correctly shaped empty tensor)."""
    world, rank = world_info(group)
    s, e = shard_range(n, world, rank)
    return gather_rows(fn(s, e), n, group)


_SIDE = {}


def _side_stream(device):
    """One side stream per device, reused by every call: torch.cuda.Stream() hands out the next
    stream of torch's pool, and the first work on each new HIP stream pays its hardware-queue
    setup (~6 ms per call on the first new streams: profiles/r4_api_first_calls.log)."""
    key = (device.type, device.index)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


def gather_map_beside(n, fn, side_fn, group=None):
    """`gather_map(n, fn)` with a second row-sharded job run beside it on a side stream.

    `side_fn(start, stop)` (e.g. the KernelSHAP weights of the shard, which need only the mask
    bits) is launched right after `fn` (the masked forward) on its own HIP stream, so its small
    kernels fill the CUs the forward leaves free instead of queueing behind it; both outputs
    are then all-gathered.  Returns (gathered fn output, gathered side_fn output).  CPU
    tensors / no GPU: sequential."""
    world, rank = world_info(group)
    s, e = shard_range(n, world, rank)
    if not torch.cuda.is_available():
        return gather_rows(fn(s, e), n, group), gather_rows(side_fn(s, e), n, group)
    cur = torch.cuda.current_stream()
    side = _side_stream(cur.device)
    side.wait_stream(cur)  # the inputs (mask bits) are produced on the current stream
    main = fn(s, e)
    with torch.cuda.stream(side):
        other = side_fn(s, e)
    cur.wait_stream(side)
    other.record_stream(cur)  # allocated on the side stream, consumed on this one
    return gather_rows(main, n, group), gather_rows(other, n, group)
