"""CPU tests of the oracle (test infrastructure) -- pins it before anything is checked against it.

  * C oracle (nerf_oracle.c, loma-order fp32) vs the committed golden fixtures, which come from the
    independent float64 numpy restatement (tests/golden/make_golden.py)
  * the numpy restatement's hand-derived backward vs float64 central differences
  * the C oracle's loma reverse-mode semantics (incoming buffers accumulated into, incoming
    adjoints as cotangents of the final state, the intermediate_output_shapes row quirk) vs torch
    autograd of a float64 torch restatement
  * the reference's own known answer (mult_a_b, fit_img.py:363-374)
"""
import os

import numpy as np
import pytest

import nerf_np
import oracle
from loma_calls import NerfCall, assert_close

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLD, name), allow_pickle=False))


@pytest.mark.parametrize("name", ["chunk_4x30.npz", "deep8_w64_2x64.npz", "trained_weights_8x16.npz"])
def test_c_oracle_matches_golden(name, oracle_lib):
    if not os.path.exists(os.path.join(GOLD, name)):
        pytest.skip("fixture not generated")
    g = load(name)
    shapes = [tuple(s) for s in g["shapes"]]
    S = int(g["S"])
    r = oracle.standard_forward_backward(g["X"], g["wp"], g["bp"], shapes, g["dists"], g["target"],
                                         S, seed=1.0, dX=True)
    assert abs(r["loss"] - g["loss"]) <= 1e-5 * abs(g["loss"])
    tol = dict(rtol=1e-4, atol_scale=2e-5)
    assert_close("acc", r["acc"], g["acc"], **tol)
    assert_close("dW", r["dW"], g["dW"], **tol)
    assert_close("dB", r["dB"], g["dB"], **tol)
    assert_close("dX", r["dX"], g["dX"], **tol)
    assert_close("d_dists", r["d_dists"], g["d_dists"], **tol)
    assert_close("d_target", r["d_target"], g["d_target"], **tol)


def test_mult_a_b_known_answer(oracle_lib):
    g = load("mult_a_b.npz")
    c = np.zeros((3, 1), np.float32)
    oracle.mult_a_b(g["a"], g["b"], c)
    assert np.array_equal(c, g["c"])


def test_positional_encoding_matches_reference_layout(oracle_lib):
    w = nerf_np.make_workload("chunk")
    pe = oracle.positional_encoding_3d(w.pts, w.F)
    assert np.array_equal(pe, w.X)
    # block-major layout: [x, sin(2^0 x), cos(2^0 x), sin(2^1 x), ...] (pos_encoding.py:54-66)
    p = w.pts.reshape(-1, 3)
    assert np.array_equal(pe[:, 0:3], p.astype(np.float32))
    assert np.array_equal(pe[:, 3:6], np.sin(p).astype(np.float32))
    assert np.array_equal(pe[:, 6:9], np.cos(p).astype(np.float32))
    assert np.array_equal(pe[:, 9:12], np.sin(2.0 * p).astype(np.float32))


def test_numpy_backward_vs_finite_differences():
    """The hand-derived backward against float64 central differences."""
    w = nerf_np.make_workload("chunk", rays=2, samples=6)
    base = nerf_np.nerf_forward_backward(w.X, w.ws, w.bs, w.dists, w.target, w.S)
    rng = np.random.RandomState(0)
    eps = 1e-6
    for l in range(len(w.ws)):
        for _ in range(6):
            k = rng.randint(w.ws[l].shape[0])
            n = rng.randint(w.ws[l].shape[1])
            wp = [x.astype(np.float64).copy() for x in w.ws]
            wm = [x.astype(np.float64).copy() for x in w.ws]
            wp[l][k, n] += eps
            wm[l][k, n] -= eps
            fp = nerf_np.nerf_forward_backward(w.X, wp, w.bs, w.dists, w.target, w.S)["loss"]
            fm = nerf_np.nerf_forward_backward(w.X, wm, w.bs, w.dists, w.target, w.S)["loss"]
            fd = (fp - fm) / (2 * eps)
            an = base["dW"][l][k, n]
            assert abs(fd - an) <= 1e-6 + 1e-5 * abs(an), (l, k, n, fd, an)
    # dists (the last one is 1e8: its derivative is exactly 0 at fp64 too)
    for j in range(w.S - 1):
        dp = w.dists.astype(np.float64).copy()
        dm = dp.copy()
        dp[0, j] += eps
        dm[0, j] -= eps
        fp = nerf_np.nerf_forward_backward(w.X, w.ws, w.bs, dp, w.target, w.S)["loss"]
        fm = nerf_np.nerf_forward_backward(w.X, w.ws, w.bs, dm, w.target, w.S)["loss"]
        assert abs((fp - fm) / (2 * eps) - base["d_dists"][0, j]) <= 1e-6 + 1e-5 * abs(base["d_dists"][0, j])


# ---- torch autograd restatement of the loma call semantics ------------------------------------

def torch_loma_call(c: NerfCall):
    """float64 torch restatement of one nerf_evaluate_and_march call with the reference's exact
    loop bounds (nerf.py:67-302), returning the loss and every array's final state."""
    import torch
    t = lambda a: torch.tensor(np.asarray(a, np.float64), requires_grad=True)
    X, W, B, T = t(c.X), t(c.wp), t(c.bp), t(c.target)
    IO0, D, ACC0 = t(c.io), t(c.dists), t(c.acc)
    L, S, N = c.L, c.S, c.N
    ios = c.ios
    wsh = c.ws_shape
    io = [IO0[l] for l in range(L)]
    for l in range(L):
        cur = io[l].clone()
        if l == 0:
            rows, K = X.shape[0], X.shape[1]
            A = X[:rows, :K]
        else:
            rows, K = int(ios[l - 1][0]), int(ios[l - 1][1])
            A = io[l - 1][:rows, :K]
        cols = int(wsh[l][1])
        upd = cur.clone()
        upd[:rows, :cols] = cur[:rows, :cols] + A @ W[l][:K, :cols]
        r0, c0 = int(ios[l][0]), int(ios[l][1])
        z = upd.clone()
        z[:r0, :c0] = upd[:r0, :c0] + B[l][:c0][None, :]
        a = z.clone()
        if l < L - 1:
            a[:r0, :c0] = torch.relu(z[:r0, :c0])
        else:
            sig = 1.0 / (1.0 + torch.exp(-z[:r0, :c0]))
            rel = torch.relu(z[:r0, :c0])
            colmask = torch.zeros(c0, dtype=torch.bool)
            if c0 > 3:
                colmask[3] = True
            a[:r0, :c0] = torch.where(colmask[None, :], rel, sig)
        io[l] = a
    rgba = io[L - 1][: N * S, :4].reshape(N, S, 4)
    alpha = 1.0 - torch.exp(-rgba[..., 3] * D)
    cc = (1.0 - alpha) + 1e-10
    P = torch.cumprod(cc, dim=1)
    cp = torch.cat([torch.ones(N, 1, dtype=P.dtype), P[:, 1:]], dim=1)
    wsamp = alpha * cp
    acc = ACC0.clone()
    acc[:, :3] = ACC0[:, :3] + (wsamp[..., None] * rgba[..., :3]).sum(1)
    loss = ((acc[:, :3] - T) ** 2).sum()
    inputs = dict(X=X, W=W, B=B, T=T, IO=IO0, dists=D, acc=ACC0)
    finals = dict(IO=torch.stack(io), rgba=rgba, alpha=alpha, cp=cp, wsamp=wsamp, acc=acc,
                  X=X, W=W, B=B, T=T, dists=D)
    return loss, inputs, finals


@pytest.mark.parametrize("quirk", ["fake_trace_256", "real_rows"])
def test_oracle_reverse_semantics_vs_torch_autograd(quirk, oracle_lib):
    import torch
    w = nerf_np.make_workload("chunk", rays=3, samples=5)
    shapes = [x.shape for x in w.ws]
    R = w.X.shape[0]
    ios = [[24, s[1]] for s in shapes] if quirk == "fake_trace_256" else [[R, s[1]] for s in shapes]
    c = NerfCall(w.X, w.wp, w.bp, shapes, w.target, w.dists, w.S, ios=ios, io_alloc=(24, 32),
                 rng=np.random.RandomState(7), init_scale=0.1, adj_scale=0.1)
    seed = 0.7
    fwd = c.oracle_forward()
    loss, inputs, finals = torch_loma_call(c)
    assert abs(float(loss.detach()) - fwd["loss"]) <= 1e-5 * abs(fwd["loss"])
    assert_close("io", finals["IO"].detach().numpy(), fwd["io"], rtol=1e-5, atol_scale=1e-6)
    # VJP: seed on the loss + incoming adjoints as cotangents of every final state
    obj = seed * loss
    for k, v in finals.items():
        obj = obj + (v * torch.tensor(c.d[k].astype(np.float64))).sum()
    names = list(inputs)
    grads = torch.autograd.grad(obj, [inputs[k] for k in names])
    got = c.oracle_grad(seed)
    for k, gk in zip(names, grads):
        assert_close("d" + k, got[k], gk.numpy(), rtol=1e-4, atol_scale=1e-5)
    for k in ("rgba", "alpha", "cp", "wsamp"):
        assert not got[k].any(), k   # overwritten before read: adjoint ends at 0


def test_oracle_sigmoid_adjoint_nan_below_minus_88(oracle_lib):
    """loma's reverse of 1/(1+exp(-x)) is NaN once exp(-x) overflows fp32 (x < -88.7): the
    reference's train_nerf.py:486-489 NaN guard exists for this; the oracle keeps it."""
    w = nerf_np.make_workload("chunk", rays=1, samples=4)
    shapes = [x.shape for x in w.ws]
    bp = w.bp.copy()
    bp[2, 0] = -200.0
    r = oracle.standard_forward_backward(w.X, w.wp, bp, shapes, w.dists, w.target, w.S, seed=1.0)
    assert np.isnan(r["dW"]).any()
    bp[2, 0] = -60.0            # exp(60) finite, (1+e)^2 overflows -> adjoint exactly 0, no NaN
    r = oracle.standard_forward_backward(w.X, w.wp, bp, shapes, w.dists, w.target, w.S, seed=1.0)
    assert np.isfinite(r["dW"]).all()
