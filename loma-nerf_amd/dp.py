"""Data-parallel step glue: one process per GPU, rays sharded, one RCCL all-reduce per step.

The loss is a sum over rays (scripts/nerf.py:297-302) and the reference seeds its gradient with
that loss (train_nerf.py:477). Each rank therefore computes *unit-seeded* gradients of its own rays
into a packed buffer [dW (L*w_k*w_n) | db (L*w_n) | loss (1)]; one SUM all-reduce (RCCL over xGMI
with the "nccl" backend, gloo on CPU) yields the global unit-seeded gradients and the global
loss; multiplying the gradient part by the reduced loss gives exactly the loss-seeded gradient of
the whole batch. The optimizer update is then replicated, so weights stay identical on all ranks.
"""
from __future__ import annotations


def shard_rays(n_rays: int, world: int, rank: int):
    """Contiguous ray range of `rank` (SURVEY.md §8e partitioning)."""
    lo = n_rays * rank // world
    hi = n_rays * (rank + 1) // world
    return lo, hi


def allreduce_loss_seeded(packed, dist, scale_fn=None, group=None):
    """SUM-all-reduce the packed [grads | loss] buffer, then scale grads by the global loss.

    `scale_fn(buf, scalar)` does buf *= scalar on the buffer's device (the engine's
    lnerf_scale_by_device_scalar on GPU); defaults to an in-place tensor multiply."""
    dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=group)
    grads, loss = packed[:-1], packed[-1:]
    if scale_fn is None:
        grads.mul_(loss)
    else:
        scale_fn(grads, loss)
    return packed


def gather_rows(local, n_total, dist, group=None):
    """Config 5's final gather ("replicas only, then a final gather of 640 000 x 3
    colours"): every rank holds the rows [lo, hi) of its dp.shard_rays range; returns the whole
    (n_total, ...) array on every rank. Shards differ by at most one row, so each is padded to
    ceil(n_total / world) rows for one all_gather and the padding is dropped in rank order."""
    import torch
    world = dist.get_world_size(group)
    chunk = -(-n_total // world)
    pad = torch.zeros((chunk,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    rows = []
    for r in range(world):
        lo, hi = shard_rays(n_total, world, r)
        rows.append(parts[r][: hi - lo])
    return torch.cat(rows, 0)
