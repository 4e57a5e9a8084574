"""GPU parity of the loma-compat C ABI (the drop-in boundary) against the C oracle.

Calls go through libloma_nerf.so exactly as train_nerf.py / fit_img.py make them (nested ctypes
pointer tables, compiler.compile-set argtypes), and are compared with oracle/nerf_oracle.c on the
same inputs. The compat path runs the loma-order HIP kernels, so results agree to a few ulp (the
remaining differences are expf implementations: device ocml vs glibc).
"""
import ctypes

import numpy as np
import pytest

import nerf_np
from loma_calls import NerfCall, assert_close
from loma_marshal import from_ctypes, to_ctypes

pytestmark = pytest.mark.gpu

TOL = dict(rtol=2e-6, atol_scale=2e-6)


@pytest.fixture(scope="module")
def lib():
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip("no GPU")
    import lnerf
    # the same CDLL + argtypes compiler.compile hands to train_nerf.py (tested in test_abi.py)
    return lnerf.load_library(lnerf.LIB_PATH)


def chunk_call(**kw):
    w = nerf_np.make_workload("chunk")
    shapes = [x.shape for x in w.ws]
    return NerfCall(w.X, w.wp, w.bp, shapes, w.target, w.dists, w.S, **kw)


def test_chunk_forward_matches_oracle(lib):
    c = chunk_call()
    got, want = c.lib_forward(lib), c.oracle_forward()
    assert np.isfinite(got["loss"])
    assert abs(got["loss"] - want["loss"]) <= 2e-6 * abs(want["loss"])
    for k in ("io", "rgba", "alpha", "cp", "wsamp", "acc"):
        assert_close(k, got[k], want[k], **TOL)
    # the 256-row fake trace (train_nerf.py:229-234) makes rows 120..255 of every layer live
    assert np.abs(got["io"][0, 120:256, :30]).sum() > 0


def test_chunk_grad_matches_oracle(lib):
    c = chunk_call()
    loss = c.oracle_forward()["loss"]
    got, want = c.lib_grad(lib, loss), c.oracle_grad(loss)
    for k in ("W", "B", "X", "T", "IO", "dists", "acc", "rgba", "alpha", "cp", "wsamp"):
        assert_close("d" + k, got[k], want[k], **TOL)
    assert np.abs(got["W"]).sum() > 0
    # loma restores primal buffers and never writes int adjoints
    assert np.array_equal(got["_io_after"], c.io)
    assert got["_ints"] == [0] * 5
    # adjoints of overwritten buffers end at zero
    for k in ("rgba", "alpha", "cp", "wsamp"):
        assert not got[k].any()


def test_nonzero_buffers_follow_loma_semantics(lib):
    """Incoming intermediate_outputs / accumulated_color are accumulated into, and incoming
    adjoints act as cotangents of the buffers' final state (reverse_diff.py:576-616)."""
    c = chunk_call(init_scale=0.1, adj_scale=0.1)
    got, want = c.lib_forward(lib), c.oracle_forward()
    for k in ("io", "acc"):
        assert_close(k, got[k], want[k], **TOL)
    assert abs(got["loss"] - want["loss"]) <= 2e-6 * abs(want["loss"])
    g, w = c.lib_grad(lib, 0.37), c.oracle_grad(0.37)
    for k in ("W", "B", "X", "T", "IO", "dists", "acc", "rgba", "alpha", "cp", "wsamp"):
        assert_close("d" + k, g[k], w[k], **TOL)


def test_real_row_trace_variant(lib):
    """intermediate_output_shapes traced on the real rows (fit_img.py:434-437 style)."""
    w = nerf_np.make_workload("chunk")
    shapes = [x.shape for x in w.ws]
    R = w.X.shape[0]
    c = NerfCall(w.X, w.wp, w.bp, shapes, w.target, w.dists, w.S,
                 ios=[[R, s[1]] for s in shapes], io_alloc=(R, 32))
    got, want = c.lib_forward(lib), c.oracle_forward()
    assert_close("acc", got["acc"], want["acc"], **TOL)
    g, o = c.lib_grad(lib, got["loss"]), c.oracle_grad(got["loss"])
    assert_close("dW", g["W"], o["W"], **TOL)
    assert_close("dB", g["B"], o["B"], **TOL)


def test_edge_numerics(lib):
    """sigma exactly 0 (ReLU-masked), tiny sigma with delta = 1e8, alpha -> 1 underflow into fp32
    denormals, and a bias driving the RGB pre-activation below -88 (loma's sigmoid adjoint is NaN
    there: exp overflows)."""
    w = nerf_np.make_workload("chunk")
    shapes = [x.shape for x in w.ws]
    bp = w.bp.copy()
    bp[2, 3] = -50.0          # sigma = ReLU(very negative) = 0 for every sample
    c0 = NerfCall(w.X, w.wp, bp, shapes, w.target, w.dists, w.S)
    for c in (c0,):
        got, want = c.lib_forward(lib), c.oracle_forward()
        assert_close("acc", got["acc"], want["acc"], **TOL)
        g, o = c.lib_grad(lib, got["loss"]), c.oracle_grad(got["loss"])
        assert_close("dW", g["W"], o["W"], **TOL)
    bp = w.bp.copy()
    bp[2, 3] = 40.0           # dense: alpha ~ 1, transmittance underflows to denormals / 0
    c1 = NerfCall(w.X, w.wp, bp, shapes, w.target, w.dists, w.S)
    got, want = c1.lib_forward(lib), c1.oracle_forward()
    assert_close("cp", got["cp"], want["cp"], **TOL)
    g, o = c1.lib_grad(lib, got["loss"]), c1.oracle_grad(got["loss"])
    assert_close("dW", g["W"], o["W"], **TOL)
    bp = w.bp.copy()
    bp[2, 0] = -200.0         # rgb pre-activation < -88: NaN adjoint like the loma C target
    c2 = NerfCall(w.X, w.wp, bp, shapes, w.target, w.dists, w.S)
    got = c2.lib_forward(lib)
    g, o = c2.lib_grad(lib, got["loss"]), c2.oracle_grad(got["loss"])
    assert np.isnan(o["W"]).any()
    assert np.array_equal(np.isnan(g["W"]), np.isnan(o["W"]))


@pytest.fixture(scope="module")
def fitlib(lib):
    return lib


def test_mult_a_b_known_answer(fitlib):
    """fit_img.py:363-374, the reference's only executed known-answer test near the path."""
    a = np.array([[1, 2], [3, 4], [5, 6]], np.float32)
    b = np.array([[100], [200]], np.float32)
    c = np.array([[0], [0], [0]], np.float32)
    cc = to_ctypes(c)
    fitlib.mult_a_b(to_ctypes(a), 3, 2, to_ctypes(b), 2, 1, cc)
    out = from_ctypes(cc, c.shape)
    assert np.allclose(out, np.array([[500], [1100], [1700]], np.float32))


def test_mlp_fit_matches_oracle(fitlib):
    import oracle
    rng = np.random.RandomState(3)
    # fit_img.py:387-441: 2D PE input, 3-layer MLP (filter 16), one 16x16 chunk
    coords = np.stack(np.meshgrid(np.linspace(0, 1, 16), np.linspace(0, 1, 16)), -1).reshape(-1, 2)
    parts = [coords]
    for f in range(5):
        parts += [np.sin(2.0 ** f * coords), np.cos(2.0 ** f * coords)]
    X = np.transpose(np.array(parts), (1, 0, 2)).reshape(256, -1).astype(np.float32)
    np.random.seed(215)
    ws, bs = nerf_np.get_sample_mlp(X.shape[1], 3, 3, 16)
    wp, bp = nerf_np.pad_weights(ws, bs)
    shapes = [w.shape for w in ws]
    T = rng.uniform(0, 1, (256, 3)).astype(np.float32)
    ios = np.array([[256, s[1]] for s in shapes], np.int32)
    io = np.zeros((3, 256, 22), np.float32)
    d = oracle.make_dims(3, 256, X.shape[1], 256, 3, 0, shapes, ios, X.shape[1], wp.shape[1],
                         wp.shape[2], bp.shape[1], io.shape[1], io.shape[2], 3, 3)
    io_o = io.copy()
    loss_o = oracle.mlp_fit_forward(d, X, wp, bp, T, io_o)
    io_c = to_ctypes(io)
    loss = fitlib.mlp_fit(to_ctypes(X), 256, X.shape[1], to_ctypes(np.zeros((256, 3), np.float32)),
                          to_ctypes(wp), to_ctypes(bp), to_ctypes(T), 256, 3, 3,
                          to_ctypes(np.array(shapes, np.int32)),
                          to_ctypes(np.array([[s[1], 1] for s in shapes], np.int32)),
                          to_ctypes(ios), io_c)
    assert abs(loss - loss_o) <= 2e-6 * abs(loss_o)
    assert_close("io", from_ctypes(io_c, io.shape), io_o, **TOL)
    adj = {k: np.zeros_like(v) for k, v in dict(X=X, W=wp, B=bp, T=T, IO=io).items()}
    oracle.mlp_fit_grad(d, dict(X=X, W=wp, B=bp, T=T, IO=io), adj, loss_o)
    dws, dbs, dio, dx, dt = (to_ctypes(np.zeros_like(wp)), to_ctypes(np.zeros_like(bp)),
                             to_ctypes(np.zeros_like(io)), to_ctypes(np.zeros_like(X)),
                             to_ctypes(np.zeros_like(T)))
    zi = lambda a: to_ctypes(np.zeros_like(a))
    b = lambda: ctypes.byref(ctypes.c_int(0))
    fitlib.grad_mlp_fit(to_ctypes(X), dx, 256, b(), X.shape[1], b(),
                        to_ctypes(np.zeros((256, 3), np.float32)), zi(np.zeros((256, 3), np.float32)),
                        to_ctypes(wp), dws, to_ctypes(bp), dbs, to_ctypes(T), dt, 256, b(), 3, b(), 3,
                        b(), to_ctypes(np.array(shapes, np.int32)), zi(np.array(shapes, np.int32)),
                        to_ctypes(np.array([[s[1], 1] for s in shapes], np.int32)),
                        zi(np.array(shapes, np.int32)), to_ctypes(ios), zi(ios), to_ctypes(io), dio,
                        loss_o)
    assert_close("dW", from_ctypes(dws, wp.shape), adj["W"], **TOL)
    assert_close("dB", from_ctypes(dbs, bp.shape), adj["B"], **TOL)
    assert_close("dX", from_ctypes(dx, X.shape), adj["X"], **TOL)
