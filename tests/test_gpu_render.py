"""The config-5 render kernel kr (lnerf_render.hip: plain bf16, two 16-sample groups per wave)
against k16's forward in the same precision and against the fp32-class render.

kr and k16's bf16 forward read the same one-plane packed weights, round every layer input to
bf16 the same way and accumulate in fp32, but in different MFMA orders (kr: each fragment feeds two
sample groups; the sums over k are the same k16 k-steps): colours agree to fp32 summation-order
level (not bitwise), and both stay within the bf16 bound of the fp32-class render.
Reference: train_nerf.py:558-712 (eval render), scripts/nerf.py:67-302.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")


@pytest.mark.parametrize("side,S", [(64, 128), (37, 100), (20, 7), (16, 1)])
def test_kr_matches_k16_bf16_forward(engine, side, S):
    """Full frames of device get_rays at several sample counts (256 % S != 0 leaves partial
    tiles; S = 1 packs 256 rays per workgroup): kr vs k16's bf16 forward (LNERF_RENDER_K16),
    colour and loss."""
    import lnerf
    import scene
    import torch
    shapes, wp, bp = scene.init_mlp(33, 4, 8, 256)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    ws, bs = _dev(wp), _dev(bp)
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    rays = engine.get_rays(side, K, scene.look_at_pose())
    tgt = _dev(np.random.RandomState(2).uniform(0, 1, (side * side, 3)).astype(np.float32))
    fl = lnerf.FAST | lnerf.MFMA_BF16
    la, a = engine.render(mlp, ws, bs, rays, None, tgt, samples=S, input_mode=lnerf.INPUT_RAYS, flags=fl)
    pa = engine.last_path()
    assert pa["kr"] and pa["planes"] == 1, pa
    a = a.clone()
    lb, b = engine.render(mlp, ws, bs, rays, None, tgt, samples=S, input_mode=lnerf.INPUT_RAYS,
                          flags=fl | lnerf.RENDER_K16)
    assert not engine.last_path()["kr"]
    torch.cuda.synchronize()
    a, b = a.cpu().numpy(), b.cpu().numpy()
    assert np.isfinite(a).all()
    np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
    assert abs(float(la) - float(lb)) <= 1e-4 * abs(float(lb))


def test_kr_psnr_against_fp32_class_render(engine):
    """The 64x64 frame at 128 samples: kr (bf16) vs the fp16x3 render, PSNR > 35 dB."""
    import lnerf
    import scene
    import torch
    shapes, wp, bp = scene.init_mlp(33, 4, 8, 256)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    ws, bs = _dev(wp), _dev(bp)
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    c2w = scene.look_at_pose()
    ref = scene.render_image(engine, mlp, ws, bs, 64, K, c2w, 128, 5, flags=lnerf.FAST)
    got = scene.render_image(engine, mlp, ws, bs, 64, K, c2w, 128, 5, flags=lnerf.FAST | lnerf.MFMA_BF16)
    assert engine.last_path()["kr"]
    torch.cuda.synchronize()
    assert scene.compute_psnr(got.cpu().numpy(), ref.cpu().numpy()) > 35.0


def test_kr_points_and_encoded_inputs(engine):
    """kr's other input modes (POINTS: device encoding from host points; ENCODED: the loma
    layer_input) give k16's bf16 forward colours on a cfg2-shaped MLP (30 wide: HT = 2)."""
    import lnerf
    import nerf_np
    import torch
    w = nerf_np.make_workload("cfg2", rays=300)
    shapes = [x.shape for x in w.ws]
    mlp = lnerf.make_mlp(shapes, w.wp.shape[1], w.wp.shape[2])
    ws, bs = _dev(w.wp), _dev(w.bp)
    for x, mode in ((w.pts32.reshape(-1, 3), lnerf.INPUT_POINTS), (w.X, lnerf.INPUT_ENCODED)):
        out = []
        for extra in (0, lnerf.RENDER_K16):
            l, c = engine.render(mlp, ws, bs, _dev(x), _dev(w.dists), _dev(w.target), samples=w.S,
                                 input_mode=mode, flags=lnerf.FAST | lnerf.MFMA_BF16 | extra)
            assert engine.last_path()["kr"] == (extra == 0)
            torch.cuda.synchronize()
            out.append((float(l), c.cpu().numpy().copy()))
        np.testing.assert_allclose(out[0][1], out[1][1], rtol=2e-5, atol=2e-6)


# ---- kr against the float64 restatement directly --------------------------

def bf16_round(a):
    """Round-to-nearest-even to bf16 (8 significant bits), as kr's operand conversion (__bf16)x
    and the one-plane weight packing (pack16_kernel) do; returned as float64."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def render_np(X, ws, bs, dists, S, operands=None):
    """The eval-render forward of scripts/nerf.py:67-288 (MLP, sigmoid rgb, ReLU sigma, inclusive
    transmittance) in float64. operands="bf16": every layer input and weight rounded to bf16 first,
    the bias added after the sum -- exactly the arithmetic kr performs, with exact float64 sums in
    place of its fp32 MFMA accumulation. Returns colours (N, 3) and the per-layer float64 inputs
    and weights the bound below needs."""
    a = np.asarray(X, np.float64)
    acts = []
    for l, (W, b) in enumerate(zip(ws, bs)):
        x = bf16_round(a) if operands == "bf16" else a
        Wl = bf16_round(W) if operands == "bf16" else np.asarray(W, np.float64)
        acts.append(np.abs(a))
        z = x @ Wl + np.asarray(b, np.float64)
        a = np.maximum(z, 0.0) if l < len(ws) - 1 else z
    rgb = 1.0 / (1.0 + np.exp(-a[:, :3]))
    sigma = np.maximum(a[:, 3], 0.0)
    N = a.shape[0] // S
    d = np.asarray(dists, np.float64).reshape(N, S)
    alpha = 1.0 - np.exp(-sigma.reshape(N, S) * d)
    T = np.cumprod(1.0 - alpha + 1e-10, axis=1)
    T[:, 0] = 1.0
    w = alpha * T
    return (w[:, :, None] * rgb.reshape(N, S, 3)).sum(1), dict(acts=acts, T=T, w=w, dists=d)


def bf16_render_bound(X, ws, bs, dists, S, colour, K_acc=256, sigmas=6.0, floor=1e-4):
    """Per-element error model of kr's colours against float64, derived like
    the fp16x3 split bounds of earlier rounds from the operand format: bf16 keeps 8 significant bits
    (u = 2^-8 relative per rounded operand), products of two bf16 are exact in fp32 and summed in
    fp32 (gamma = K_acc 2^-24 of the sum of |terms|). Layer l's pre-activation z_l[s, n] carries a
    local error
        |e_l[s, n]| <= (2u + u^2 + gamma) sum_k |x_l[s, k]| |W_l[k, n]| + gamma |b_l[n]|,
    which reaches colour channel c through the exact Jacobian dC_c / dz_l[s, n] -- the reverse pass
    of nerf_np seeded so that dL/dC = e_c (target = C - e_c / 2, seed 1). The roundings are
    independent, each uniform within its bound (variance e^2 / 3), so to first order
        |dC_c| <= sigmas * sqrt(sum_{s in ray, l, n} (dC_c / dz_l[s, n])^2 e_l[s, n]^2 / 3) + floor.
    Worst-case signs (sum of |J| |e|) would allow ~1 on colours in [0, 1] over 8 layers x 256
    units x 128 samples, which says nothing; the floor covers what first order misses: a ReLU'd
    sigma whose pre-activation sits within its error of 0 (the Jacobian there is 0 on one side) and
    the fp32 sigmoid / exp / compositing rounding (~1e-6)."""
    import nerf_np
    u, gamma = 2.0 ** -8, K_acc * 2.0 ** -24
    a = np.asarray(X, np.float64)
    eps = []
    for l, (W, b) in enumerate(zip(ws, bs)):
        Wa = np.abs(np.asarray(W, np.float64))
        eps.append((2 * u + u * u + gamma) * (np.abs(a) @ Wa) + gamma * np.abs(np.asarray(b, np.float64)))
        z = a @ np.asarray(W, np.float64) + np.asarray(b, np.float64)
        a = np.maximum(z, 0.0)
    N = a.shape[0] // S
    out = np.zeros((N, 3))
    for c in range(3):
        t = np.array(colour, np.float64)
        t[:, c] -= 0.5
        r = nerf_np.nerf_forward_backward(X, ws, bs, dists, t, S, seed=1.0)
        acc = np.zeros(N * S)
        for l in range(len(ws)):
            acc += ((r["G"][l] * eps[l]) ** 2).sum(1)
        out[:, c] = acc.reshape(N, S).sum(1)
    return sigmas * np.sqrt(out / 3.0) + floor


def _kr_frame(engine, side, S, mlp_seed=215):
    import lnerf
    import nerf_np
    import scene
    shapes, wp, bp = scene.init_mlp(33, 4, 8, 256, seed=mlp_seed)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    rays = engine.get_rays(side, K, scene.look_at_pose())
    r = rays.cpu().numpy().astype(np.float64)
    pts, dists = nerf_np.sample_rays(r[:, :3], r[:, 3:], S)
    X = nerf_np.positional_encoding_3d(pts, 5).reshape(-1, 33)
    ws = [wp[l, :k, :n] for l, (k, n) in enumerate(shapes)]
    bs = [bp[l, :n] for l, (_, n) in enumerate(shapes)]
    return mlp, wp, bp, rays, X, dists.astype(np.float32), ws, bs


def test_kr_vs_float64_per_element(engine):
    """kr (plain bf16, config 5's precision) on a 16x16 frame at S = 128 with the config-5 MLP
    (33->256x7->4), every ray and channel against the float64 restatement:
      * with the operands rounded to bf16 as kr rounds them (its arithmetic, exact sums): within
        3e-4 absolute, 1/6 of the bf16 effect itself (1.7e-3 here; measured 1.1e-4) -- the fp32
        accumulation order and the layer inputs whose fp32 value sits on the other side of a bf16
        rounding boundary (~2^-12 of the 262 144 roundings of a ray) are all that differ;
      * unrounded float64: within bf16_render_bound, the per-element error model of 8-bit operands
        with fp32 accumulation (not a PSNR; CPU-checked on three weight seeds at <= 0.78 of it)."""
    import lnerf
    import torch
    S = 128
    mlp, wp, bp, rays, X, dists, ws, bs = _kr_frame(engine, 16, S)
    tgt = torch.zeros(rays.shape[0], 3, dtype=torch.float32, device="cuda:0")
    _, acc = engine.render(mlp, _dev(wp), _dev(bp), rays, None, tgt, samples=S, input_mode=lnerf.INPUT_RAYS,
                           flags=lnerf.FAST | lnerf.MFMA_BF16)
    assert engine.last_path()["kr"]
    torch.cuda.synchronize()
    got = acc.cpu().numpy().astype(np.float64)
    emu, _ = render_np(X, ws, bs, dists, S, operands="bf16")
    err_emu = np.abs(got - emu)
    ref, _ = render_np(X, ws, bs, dists, S)
    bound = bf16_render_bound(X, ws, bs, dists, S, ref)
    err = np.abs(got - ref)
    print(f"kr vs bf16-operand float64: max err {err_emu.max():.3g}; vs float64: max err {err.max():.3g}, "
          f"max err / bound {(err / bound).max():.3g}, median bound {np.median(bound):.3g}")
    assert np.isfinite(got).all()
    assert err_emu.max() <= 3e-4, err_emu.max()
    assert (err <= bound).all(), float((err / bound).max())


def test_kr_config5_frame_subset_vs_float64(engine):
    """the config-5 workload itself -- the 800x800 frame at 128 samples through
    kr (what bench.py --render times) -- checked on a seeded subset of 512 of its rays, every
    channel, against the float64 restatement: within 3e-4 of the bf16-operand emulation (kr's own
    arithmetic with exact sums) and within bf16_render_bound of plain float64 (train_nerf.py:616-662,
    scripts/nerf.py:67-288)."""
    import lnerf
    import nerf_np
    import scene
    import torch
    S = 128
    shapes, wp, bp = scene.init_mlp(33, 4, 8, 256)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    rays = engine.get_rays(800, K, scene.look_at_pose())
    tgt = torch.zeros(rays.shape[0], 3, dtype=torch.float32, device="cuda:0")
    _, acc = engine.render(mlp, _dev(wp), _dev(bp), rays, None, tgt, samples=S, input_mode=lnerf.INPUT_RAYS,
                           flags=lnerf.FAST | lnerf.MFMA_BF16)
    assert engine.last_path()["kr"]
    torch.cuda.synchronize()
    sel = np.sort(np.random.RandomState(5).choice(rays.shape[0], 512, replace=False))
    got = acc.cpu().numpy().astype(np.float64)[sel]
    r = rays.cpu().numpy().astype(np.float64)[sel]
    pts, dists = nerf_np.sample_rays(r[:, :3], r[:, 3:], S)
    X = nerf_np.positional_encoding_3d(pts, 5).reshape(-1, 33)
    dists = dists.astype(np.float32)
    ws = [wp[l, :k, :n] for l, (k, n) in enumerate(shapes)]
    bs = [bp[l, :n] for l, (_, n) in enumerate(shapes)]
    emu, _ = render_np(X, ws, bs, dists, S, operands="bf16")
    ref, _ = render_np(X, ws, bs, dists, S)
    bound = bf16_render_bound(X, ws, bs, dists, S, ref)
    err_emu, err = np.abs(got - emu), np.abs(got - ref)
    print(f"config-5 frame, 512-ray subset: kr vs bf16-operand float64 max err {err_emu.max():.3g}; vs float64 "
          f"max err {err.max():.3g}, max err / bound {(err / bound).max():.3g}")
    assert np.isfinite(got).all()
    assert err_emu.max() <= 3e-4, err_emu.max()
    assert (err <= bound).all(), float((err / bound).max())


def test_kr_full_frame_is_its_row_shards(engine):
    """The config-5 frame itself (800x800 rays x 128 samples, what bench.py --render times):
    every colour finite and in [0, 1], and the frame equals, bit for bit, kr run on four
    contiguous shards of its rays (what each rank renders at N = 4 before the gather,
    dp.shard_rays; train_nerf.py:659-681 assembles the image): a ray's colour depends on its own
    samples only."""
    import dp
    import lnerf
    import scene
    import torch
    shapes, wp, bp = scene.init_mlp(33, 4, 8, 256)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    ws, bs = _dev(wp), _dev(bp)
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    rays = engine.get_rays(800, K, scene.look_at_pose())
    n = rays.shape[0]
    fl = lnerf.FAST | lnerf.MFMA_BF16
    tgt = torch.zeros(n, 3, dtype=torch.float32, device="cuda:0")
    lw, whole = engine.render(mlp, ws, bs, rays, None, tgt, samples=128, input_mode=lnerf.INPUT_RAYS, flags=fl)
    assert engine.last_path()["kr"]
    whole = whole.clone()
    parts, lsum = [], 0.0
    for r in range(4):
        lo, hi = dp.shard_rays(n, 4, r)
        l, c = engine.render(mlp, ws, bs, rays[lo:hi].contiguous(), None, tgt[lo:hi].contiguous(), samples=128,
                             input_mode=lnerf.INPUT_RAYS, flags=fl)
        parts.append(c.clone())
        lsum += float(l)
    torch.cuda.synchronize()
    a = whole.cpu().numpy()
    assert np.isfinite(a).all() and a.min() >= 0.0 and a.max() <= 1.0
    assert np.array_equal(a, torch.cat(parts).cpu().numpy())
    assert abs(float(lw) - lsum) <= 1e-5 * abs(lsum)


def _render_pair(engine, shapes_dims, seed, S=64, rays=96):
    import lnerf
    import nerf_np
    import torch
    rng = np.random.RandomState(seed)
    dims = shapes_dims
    ws = [(rng.randn(k, n) * np.sqrt(2.0 / k)).astype(np.float32) for k, n in zip(dims, dims[1:])]
    bs = [(rng.randn(n) * 0.5).astype(np.float32) for n in dims[1:]]
    wp, bp = nerf_np.pad_weights(ws, bs)
    w = nerf_np.make_workload("cfg2", rays=rays, samples=S)
    mlp = lnerf.make_mlp([x.shape for x in ws], wp.shape[1], wp.shape[2])
    out = []
    for extra in (0, lnerf.RENDER_K16):
        l, c = engine.render(mlp, _dev(wp), _dev(bp), _dev(w.pts32.reshape(-1, 3)), _dev(w.dists), _dev(w.target),
                             samples=S, input_mode=lnerf.INPUT_POINTS, flags=lnerf.FAST | lnerf.MFMA_BF16 | extra)
        assert engine.last_path()["kr"] == (extra == 0), engine.last_path()
        torch.cuda.synchronize()
        out.append((float(l), c.cpu().numpy().copy()))
    X = nerf_np.positional_encoding_3d(w.pts32.astype(np.float64), 5).reshape(-1, 33)
    emu, _ = render_np(X, ws, bs, w.dists, S, operands="bf16")
    return out, emu


@pytest.mark.parametrize("dims", [[33, 128, 256, 64, 100, 4], [33, 4]], ids=["nonuniform", "head_only"])
def test_kr_nonuniform_and_head_only(engine, dims):
    """kr runs every hidden pass at the widest layer's tile count over zero-padded
    packed weights; a non-uniform MLP (33->128->256->64->100->4) and a head-only one (L = 1) give
    k16's bf16 forward colours and the bf16-operand float64 colours."""
    ((la, a), (lb, b)), emu = _render_pair(engine, dims, seed=3)
    np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-6)
    assert abs(la - lb) <= 1e-4 * abs(lb)
    assert np.abs(a - emu).max() <= 3e-4, np.abs(a - emu).max()
