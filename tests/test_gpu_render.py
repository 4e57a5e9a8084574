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
