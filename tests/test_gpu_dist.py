"""The data-parallel training step on the device over RCCL, in one
process: a world-size-1 "nccl" process group (FileStore rendezvous) on cuda:0.

The protocol of loma-nerf_amd/dp.py -- unit-seeded gradients, one SUM all-reduce of the packed
[dW | db | loss] buffer, then the gradient part scaled by the reduced loss on the device
(lnerf_scale_by_device_scalar), then the replicated Adam update (train_nerf.py:133-161) -- must
give bit-for-bit the single-GPU loss-seeded step (train_nerf.py:477) followed by the same Adam
update, iteration after iteration. At world size 1 the all-reduce is the identity, so any
difference would come from the seeding arithmetic: the fused path seeds with the loss as one
multiply of the reduced gradient (grad_reduce_kernel), the same operation the DP path applies
after the exchange. The N > 1 arithmetic (the SUM over ranks) is covered by tests/test_dist.py
(gloo, 2 ranks) and test_gpu_native.py's ray-shard additivity test at full size."""
import numpy as np
import pytest

import nerf_np

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nccl(tmp_path_factory):
    import torch
    import torch.distributed as dist
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    store = dist.FileStore(str(tmp_path_factory.mktemp("pg") / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


def _params(w, dev):
    import torch
    p = torch.from_numpy(np.concatenate([w.wp.ravel(), w.bp.ravel()])).to(dev)
    nW = w.wp.size
    return p, p[:nW].view(w.wp.shape), p[nW:].view(w.bp.shape)


@pytest.mark.parametrize("rays", [256, 1024])
def test_rccl_step_equals_single_gpu_loss_seeded(engine, nccl, rays):
    import dp
    import lnerf
    import torch
    dev = "cuda:0"
    w = nerf_np.make_workload("cfg3", rays=rays)   # 33 -> 256 x 7 -> 4: the k16 + dw16 path
    shapes = [x.shape for x in w.ws]
    mlp = lnerf.make_mlp(shapes, w.wp.shape[1], w.wp.shape[2])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    x, dists, target = t(w.pts32.reshape(-1, 3)), t(w.dists), t(w.target)
    pa, wa, ba = _params(w, dev)
    pb, wb, bb = _params(w, dev)
    ma, va = torch.zeros_like(pa), torch.zeros_like(pa)
    mb, vb = torch.zeros_like(pb), torch.zeros_like(pb)
    ga = engine.alloc_grads(len(shapes), w.wp.shape[1], w.wp.shape[2])
    gb = engine.alloc_grads(len(shapes), w.wp.shape[1], w.wp.shape[2])
    for it in range(1, 4):
        # single GPU: the gradient seeded with the batch loss (train_nerf.py:477), then Adam
        engine.train_step(mlp, wa, ba, x, dists, target, samples=w.S, num_freqs=w.F, seed=None,
                          flags=lnerf.FAST, grads=ga)
        engine.adam_update(pa, ga[0][:-1], ma, va, it, 5e-4)
        # data-parallel: unit seed, RCCL SUM of [dW | db | loss], scale by the reduced loss, Adam
        engine.train_step(mlp, wb, bb, x, dists, target, samples=w.S, num_freqs=w.F, seed=1.0,
                          flags=lnerf.FAST, grads=gb)
        dp.allreduce_loss_seeded(gb[0], nccl, engine.scale_by_device_scalar)
        engine.adam_update(pb, gb[0][:-1], mb, vb, it, 5e-4)
        torch.cuda.synchronize()
        assert engine.last_path()["k16"]
        assert torch.isfinite(ga[0]).all()
        assert float(ga[0][-1]) == float(gb[0][-1]), it           # the loss slot
        assert torch.equal(ga[0], gb[0]), (it, (ga[0] - gb[0]).abs().max().item())
        assert torch.equal(pa, pb), it
        assert torch.equal(ma, mb) and torch.equal(va, vb), it
    assert not torch.equal(pa, _params(w, dev)[0])                  # the parameters moved


def test_rccl_allreduce_sums_two_shards_like_the_full_batch(engine, nccl):
    """The exchange's arithmetic with a real SUM: the two halves of a ray batch run as two
    'ranks' on one GPU; their packed unit-seeded buffers are added (what a two-rank SUM
    delivers), passed through the RCCL step (all-reduce at world size 1, then the scale by the
    reduced loss). The result equals the full batch's loss-seeded gradient within fp32
    summation-order noise (the loss is a sum over rays, nerf.py:297-302)."""
    import dp
    import lnerf
    import torch
    dev = "cuda:0"
    w = nerf_np.make_workload("cfg3", rays=512)
    shapes = [x.shape for x in w.ws]
    mlp = lnerf.make_mlp(shapes, w.wp.shape[1], w.wp.shape[2])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    _, ws, bs = _params(w, dev)
    full = engine.alloc_grads(len(shapes), w.wp.shape[1], w.wp.shape[2])
    engine.train_step(mlp, ws, bs, t(w.pts32.reshape(-1, 3)), t(w.dists), t(w.target), samples=w.S,
                      num_freqs=w.F, seed=None, flags=lnerf.FAST, grads=full)
    packed = []
    for lo, hi in (dp.shard_rays(w.N, 2, 0), dp.shard_rays(w.N, 2, 1)):
        g = engine.alloc_grads(len(shapes), w.wp.shape[1], w.wp.shape[2])
        pts = w.pts32.reshape(w.N, w.S, 3)[lo:hi].reshape(-1, 3)
        engine.train_step(mlp, ws, bs, t(pts), t(w.dists[lo:hi]), t(w.target[lo:hi]), samples=w.S,
                          num_freqs=w.F, seed=1.0, flags=lnerf.FAST, grads=g)
        packed.append(g[0])
    summed = packed[0] + packed[1]            # what the SUM over two ranks delivers
    dp.allreduce_loss_seeded(summed, nccl, engine.scale_by_device_scalar)
    torch.cuda.synchronize()
    got, want = summed.cpu().numpy(), full[0].cpu().numpy()
    assert abs(got[-1] - want[-1]) <= 1e-6 * abs(want[-1])
    scale = np.abs(want[:-1]).max()
    assert np.abs(got[:-1] - want[:-1]).max() <= 1e-5 * scale
