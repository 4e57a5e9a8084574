"""config 1 on the device: fit_img.py's 2-D image-fitting MLP (scripts/mlp_fit.py) through the
fused k16 path with the mlp_fit head (lnerf.HEAD_FIT), against the C oracle's restatement of
mlp_fit / grad_mlp_fit (oracle/nerf_oracle.c, scripts/mlp_fit.py:1-147).

Workload: a 256x256 image (fit_img.py's img_size; data/warren.jpeg is absent, so a smooth
synthetic RGB image stands in), input = positional_encoding_2d of the pixel grid
(pos_encoding.py:4-37, F = 5: 22 features), MLP 22 -> 16 -> 16 -> 3 (fit_img.py:180-206,
get_sample_mlp with filter 16), gradient seeded with the previous loss and plain SGD at step 1e-4
(fit_img.py:468-532). One test runs all 65 536 rows as one batch, one runs fit_img's 256-row
chunk loop; the oracle runs the same rows with standard semantics (zero-initialised
intermediates, ios rows = rows)."""
import numpy as np
import pytest

from loma_calls import assert_close

pytestmark = pytest.mark.gpu

TOL = dict(rtol=1e-5, atol_scale=1e-5)


def positional_encoding_2d(x, F=5):
    """pos_encoding.py:4-37: [x, sin(2^0 x), cos(2^0 x), ...] per input feature (feature-major)."""
    parts = [x]
    for i in range(F):
        parts.append(np.sin((2.0 ** i) * x))
        parts.append(np.cos((2.0 ** i) * x))
    c = np.transpose(np.array(parts), (1, 0, 2))
    return np.reshape(c, (c.shape[0], -1)).astype(np.float32)


def image_workload(side=256, seed=215):
    import scene
    g = np.linspace(0, 1, side)
    coords = np.stack(np.meshgrid(g, g), axis=-1).reshape(-1, 2)        # fit_img.py:391-394
    X = positional_encoding_2d(coords)
    u, v = coords[:, 0], coords[:, 1]
    img = np.stack([0.5 + 0.4 * np.sin(6 * u) * np.cos(4 * v), 0.5 + 0.3 * np.cos(5 * u + 2 * v),
                    u * v], -1).astype(np.float32)
    shapes, wp, bp = scene.init_mlp(X.shape[1], 3, 3, 16, seed=seed)
    return X, img, shapes, wp, bp


def oracle_fit(X, T, wp, bp, shapes, seed):
    """mlp_fit + grad_mlp_fit (standard semantics) through the C oracle: (loss, outputs, dW, dB)."""
    import oracle
    rows, L = X.shape[0], len(shapes)
    io_cols = max(4, max(n for _, n in shapes))
    d = oracle.make_dims(L, rows, X.shape[1], rows, T.shape[1], 0, shapes, [[rows, n] for _, n in shapes],
                         X.shape[1], wp.shape[1], wp.shape[2], wp.shape[2], rows, io_cols, T.shape[1], 3,
                         bias_shapes=[[n, 1] for _, n in shapes])
    IO = np.zeros((L, rows, io_cols), np.float32)
    loss = oracle.mlp_fit_forward(d, X, wp, bp, T, IO)
    prim = dict(X=X, W=wp, B=bp, T=T, IO=np.zeros_like(IO))
    adj = dict(W=np.zeros_like(wp), B=np.zeros_like(bp), T=np.zeros_like(T), IO=np.zeros_like(IO))
    oracle.mlp_fit_grad(d, prim, adj, seed)
    return loss, IO[L - 1, :, :T.shape[1]].copy(), adj["W"], adj["B"]


def f64_fit(X, T, wp, bp, shapes, seed):
    """The same step in float64 numpy (exact ReLU / sigmoid derivatives): (loss, outputs, dW, dB)."""
    L = len(shapes)
    A = X.astype(np.float64)
    acts, zs = [A], []
    for l, (k, n) in enumerate(shapes):
        Z = A @ wp[l, :k, :n].astype(np.float64) + bp[l, :n].astype(np.float64)
        zs.append(Z)
        A = np.maximum(Z, 0.0) if l < L - 1 else 1.0 / (1.0 + np.exp(-Z))
        acts.append(A)
    O = A
    loss = float(((O - T) ** 2).sum())
    G = 2.0 * seed * (O - T) * O * (1.0 - O)
    dW, dB = np.zeros(wp.shape), np.zeros(bp.shape)
    for l in range(L - 1, -1, -1):
        k, n = shapes[l]
        dW[l, :k, :n] = acts[l].T @ G
        dB[l, :n] = G.sum(0)
        if l:
            G = (G @ wp[l, :k, :n].T.astype(np.float64)) * (zs[l - 1] > 0)
    return loss, O, dW, dB


@pytest.fixture(scope="module")
def fit():
    return image_workload()


def test_mlp_fit_step_matches_oracle_256x256(engine, fit):
    import lnerf
    import torch
    X, T, shapes, wp, bp = fit
    dev = "cuda:0"
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    seed = 1.7   # fit_img.py:515 seeds grad_mlp_fit with the previous chunk's loss
    loss, out, g = engine.mlp_fit_step(mlp, t(wp), t(bp), t(X), t(T), seed=seed, flags=lnerf.FAST)
    torch.cuda.synchronize()
    path = engine.last_path()
    assert path["k16"] and path["dw16"] and path["planes"] == 2, path
    nW = wp.size
    gd = g.cpu().numpy()
    got = dict(loss=float(loss), out=out.cpu().numpy(), dW=gd[:nW].reshape(wp.shape), dB=gd[nW:-1].reshape(bp.shape))
    # float64 at 1e-5 (the fp16x3 products are fp32-class); the loma-order fp32 oracle at
    # north_star's 1e-4 (its sequential fp32 sums over 65 536 rows carry ~1e-5 of their own)
    for ref, tol in ((f64_fit(X, T, wp, bp, shapes, seed), TOL), (oracle_fit(X, T, wp, bp, shapes, seed),
                                                                   dict(rtol=1e-4, atol_scale=1e-4))):
        want_loss, want_out, want_dW, want_dB = ref
        assert abs(got["loss"] - want_loss) <= tol["rtol"] * abs(want_loss), (got["loss"], want_loss)
        assert_close("outputs", got["out"], want_out, **tol)
        assert_close("dW", got["dW"], want_dW, **tol)
        assert_close("dB", got["dB"], want_dB, **tol)
    # forward only (the loss fit_img.py:515-532 reads after the update) equals the train forward
    loss2, out2, _ = engine.mlp_fit_step(mlp, t(wp), t(bp), t(X), t(T), want_grad=False, flags=lnerf.FAST)
    torch.cuda.synchronize()
    assert float(loss2) == float(loss)
    assert torch.equal(out2, out)


def test_mlp_fit_sgd_loop_matches_oracle(engine, fit):
    """fit_img.py:423-532's inner loop on the device over 8 chunks of 256 rows (chunk_size^2): the
    gradient of chunk c seeded with the previous step's loss (c_float(0) before the first),
    ws -= 1e-4 d_ws, then the forward loss of chunk c, which seeds the next gradient. The C oracle
    runs the same loop in float32; losses and weights must agree at every step."""
    import lnerf
    import torch
    X, T, shapes, wp, bp = fit
    dev = "cuda:0"
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    Xd, Td = t(X), t(T)
    params = torch.cat([t(wp).reshape(-1), t(bp).reshape(-1)])
    ws, bs = params[:wp.size].view(wp.shape), params[wp.size:].view(bp.shape)
    grads = engine.alloc_grads(len(shapes), wp.shape[1], wp.shape[2])
    wq, bq = wp.copy(), bp.copy()
    prev_d, prev_o = 0.0, 0.0
    step = np.float32(1e-4)
    losses = []
    for c in range(8):
        r = slice(256 * c, 256 * (c + 1))
        engine.mlp_fit_step(mlp, ws, bs, Xd[r], Td[r], seed=prev_d, flags=lnerf.FAST, grads=grads)
        params -= 1e-4 * grads[0][:-1]
        loss_d, _, _ = engine.mlp_fit_step(mlp, ws, bs, Xd[r], Td[r], want_grad=False, flags=lnerf.FAST)
        torch.cuda.synchronize()
        _, _, dW, dB = oracle_fit(X[r], T[r], wq, bq, shapes, prev_o)
        wq = wq - step * dW
        bq = bq - step * dB
        loss_o = oracle_fit(X[r], T[r], wq, bq, shapes, 0.0)[0]
        prev_d, prev_o = float(loss_d), loss_o
        losses.append(prev_d)
        assert abs(prev_d - prev_o) <= 1e-5 * abs(prev_o), (c, prev_d, prev_o)
        p = params.cpu().numpy()
        assert_close(f"ws chunk {c}", p[:wp.size].reshape(wp.shape), wq, rtol=1e-5, atol_scale=1e-6)
        assert_close(f"bs chunk {c}", p[wp.size:].reshape(bp.shape), bq, rtol=1e-5, atol_scale=1e-6)
    assert not np.array_equal(wq, wp) and np.isfinite(losses).all()   # the loop moved the weights


def test_mlp_fit_head_rejects_unsupported_calls(engine, fit):
    import lnerf
    import torch
    X, T, shapes, wp, bp = fit
    dev = "cuda:0"
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a[:64])).to(dev)
    for bad in (lnerf.GENERIC, lnerf.ONE_WAVE, lnerf.K32, lnerf.MFMA_F32, lnerf.MFMA_BF16X6):
        with pytest.raises(RuntimeError):
            engine.mlp_fit_step(mlp, t(wp), t(bp), t(X), t(T), seed=1.0, flags=bad)
