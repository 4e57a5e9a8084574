"""Multi-process (world_size 2, gloo, CPU) test of the data-parallel protocol in
loma-nerf_amd/dp.py: each rank computes unit-seeded gradients of its ray shard (here with the C
oracle standing in for the device kernels), one SUM all-reduce of the packed [dW | db | loss]
buffer, then scaling by the reduced loss must equal the loss-seeded gradient of the full batch
(train_nerf.py:477 seeds the gradient with the loss; the loss is a sum over rays). Every rank then
applies the reference's Adam step (train_nerf.py:133-161) to its own replica of the parameters,
and the replicas must stay bit-identical (no broadcast in the protocol)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _adam1(p, g, lr=5e-4, b1=0.9, b2=0.999, eps=1e-8):
    """First AdamOptimizer.update of train_nerf.py:143-161 (float32 arrays, t = 1)."""
    t = 1
    lr_t = lr * (np.sqrt(1 - b2 ** t) / (1 - b1 ** t))
    m = (1 - b1) * g
    v = (1 - b2) * (g ** 2)
    return p - lr_t * (m / (1 - b1 ** t)) / (np.sqrt(v / (1 - b2 ** t)) + eps)


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (os.path.join(repo, "oracle"), os.path.join(repo, "loma-nerf_amd")):
        sys.path.insert(0, p)
    import dp
    import nerf_np
    import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = nerf_np.make_workload("cfg2", rays=20, samples=8)
    shapes = [x.shape for x in w.ws]
    lo, hi = dp.shard_rays(w.N, world, rank)
    X = w.X.reshape(w.N, w.S, -1)[lo:hi].reshape(-1, w.X.shape[1])
    r = oracle.standard_forward_backward(X, w.wp, w.bp, shapes, w.dists[lo:hi], w.target[lo:hi],
                                         w.S, seed=1.0)
    packed = torch.from_numpy(np.concatenate([r["dW"].ravel(), r["dB"].ravel(),
                                              [np.float32(r["loss"])]]).astype(np.float32))
    dp.allreduce_loss_seeded(packed, dist)
    params = np.concatenate([w.wp.ravel(), w.bp.ravel()]).astype(np.float32)
    out.put((rank, packed.numpy().copy(), _adam1(params, packed.numpy()[:-1])))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_allreduce_matches_full_batch(oracle_lib):
    import nerf_np
    import oracle
    from loma_calls import assert_close
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, pn)) for r, g, pn in (q.get(timeout=120), q.get(timeout=120)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = res[0][0]
    # the all-reduced buffer and the replicated Adam step are bit-identical on both ranks
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])
    w = nerf_np.make_workload("cfg2", rays=20, samples=8)
    shapes = [x.shape for x in w.ws]
    full = oracle.standard_forward_backward(w.X, w.wp, w.bp, shapes, w.dists, w.target, w.S,
                                            seed=None)
    nW = full["dW"].size
    nB = full["dB"].size
    assert abs(got[-1] - full["loss"]) <= 1e-5 * full["loss"]
    assert_close("dW", got[:nW].reshape(full["dW"].shape), full["dW"], rtol=1e-4, atol_scale=1e-5)
    assert_close("dB", got[nW:nW + nB].reshape(full["dB"].shape), full["dB"], rtol=1e-4,
                 atol_scale=1e-5)
    # the replicated update equals Adam on the full-batch gradient, except where a gradient is
    # so small that fp32 summation order decides its sign (Adam's first step is +-lr there)
    p0 = np.concatenate([w.wp.ravel(), w.bp.ravel()]).astype(np.float32)
    gfull = np.concatenate([full["dW"].ravel(), full["dB"].ravel()]).astype(np.float32)
    want = _adam1(p0, gfull)
    big = np.abs(gfull) > 1e-3 * np.abs(gfull).max()
    assert big.sum() > 0.5 * (gfull != 0).sum()
    assert np.allclose(res[0][1][big], want[big], rtol=1e-6, atol=1e-6)


def test_shard_rays_partitions():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "loma-nerf_amd"))
    import dp
    for n in (1, 7, 4096):
        for world in (1, 2, 3, 8):
            spans = [dp.shard_rays(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c


def test_strong_scaling_shards_cover_one_batch():
    """bench.py --strong (config 4): the ranks' shards of one batch concatenate to that batch."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "loma-nerf_amd"))
    import dp
    import scene
    b = scene.make_batch("cfg2", rays=37)
    for world in (1, 2, 8):
        parts = [scene.shard_batch(b, *dp.shard_rays(b["N"], world, r)) for r in range(world)]
        assert sum(p["N"] for p in parts) == b["N"] and all(p["N_total"] == b["N"] for p in parts)
        for k in ("pts", "dists", "rays", "target"):
            assert np.array_equal(np.concatenate([p[k] for p in parts]), b[k]), k


def _gather_worker(rank, world, port, n, out):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "loma-nerf_amd"))
    import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frame = torch.arange(n * 3, dtype=torch.float32).reshape(n, 3)
    lo, hi = dp.shard_rays(n, world, rank)
    got = dp.gather_rows(frame[lo:hi].clone(), n, dist)
    out.put((rank, bool(torch.equal(got, frame))))
    dist.barrier()
    dist.destroy_process_group()


def test_render_frame_gather_uneven_shards():
    """bench.py --render at N > 1 (config 5): each rank renders its dp.shard_rays share of the frame
    and dp.gather_rows reassembles the whole frame in ray order on every rank (train_nerf.py:659-681
    assembles the eval image), shards of unequal length included (7 rows over 3 ranks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world, n = 3, 7
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(res[r] for r in range(world)), res
