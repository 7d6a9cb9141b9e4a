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
    buf = local.new_zeros((cap,) + tuple(local.shape[1:]))
    buf[:e - s] = local
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    parts = []
    for r in range(world):
        rs, re_ = shard_range(n, world, r)
        parts.append(outs[r][:re_ - rs])
    return torch.cat(parts, 0)


def gather_map(n, fn, group=None):
    """Run `fn(start, stop)` on this rank's shard of n units and all-gather the results.

    `fn` returns a tensor whose leading dimension is stop - start (it is called with an empty
    range on ranks that own no unit and must still return a correctly shaped empty tensor)."""
    world, rank = world_info(group)
    s, e = shard_range(n, world, rank)
    return gather_rows(fn(s, e), n, group)
