"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the C oracle (nerf_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
Parity status: see nerf_oracle.h ("parity unpinned" against the loma .so; independently
cross-validated).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liblnerf_oracle.so")
MAXL = 16

_f32p = ctypes.POINTER(ctypes.c_float)


class Dims(ctypes.Structure):
    _fields_ = [
        ("num_weights", ctypes.c_int),
        ("layer_input_h", ctypes.c_int),
        ("layer_input_w", ctypes.c_int),
        ("target_image_h", ctypes.c_int),
        ("target_image_w", ctypes.c_int),
        ("num_samples", ctypes.c_int),
        ("weight_shapes", (ctypes.c_int * 2) * MAXL),
        ("bias_shapes", (ctypes.c_int * 2) * MAXL),
        ("intermediate_output_shapes", (ctypes.c_int * 2) * MAXL),
        ("x_cols", ctypes.c_int),
        ("w_k", ctypes.c_int),
        ("w_n", ctypes.c_int),
        ("b_n", ctypes.c_int),
        ("io_rows", ctypes.c_int),
        ("io_cols", ctypes.c_int),
        ("t_cols", ctypes.c_int),
        ("acc_cols", ctypes.c_int),
    ]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _lib.oracle_nerf_forward.restype = ctypes.c_float
        _lib.oracle_mlp_fit_forward.restype = ctypes.c_float
        _lib.oracle_train_step.restype = ctypes.c_float
        _lib.oracle_nerf_grad.restype = None
        _lib.oracle_nerf_grad.argtypes = [ctypes.POINTER(Dims)] + [_f32p] * 22 + [ctypes.c_float]
        _lib.oracle_mlp_fit_grad.argtypes = [ctypes.POINTER(Dims)] + [_f32p] * 10 + [ctypes.c_float]
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"], (a.dtype, a.flags)
    return a.ctypes.data_as(_f32p)


def make_dims(L, layer_input_h, layer_input_w, target_h, target_w, S, weight_shapes, ios,
              x_cols, w_k, w_n, b_n, io_rows, io_cols, t_cols, acc_cols, bias_shapes=None):
    d = Dims()
    d.num_weights, d.layer_input_h, d.layer_input_w = L, layer_input_h, layer_input_w
    d.target_image_h, d.target_image_w, d.num_samples = target_h, target_w, S
    for l in range(L):
        d.weight_shapes[l][0], d.weight_shapes[l][1] = int(weight_shapes[l][0]), int(weight_shapes[l][1])
        d.intermediate_output_shapes[l][0], d.intermediate_output_shapes[l][1] = int(ios[l][0]), int(ios[l][1])
        if bias_shapes is not None:
            d.bias_shapes[l][0], d.bias_shapes[l][1] = int(bias_shapes[l][0]), int(bias_shapes[l][1])
    d.x_cols, d.w_k, d.w_n, d.b_n = x_cols, w_k, w_n, b_n
    d.io_rows, d.io_cols, d.t_cols, d.acc_cols = io_rows, io_cols, t_cols, acc_cols
    return d


def standard_dims(wp: np.ndarray, shapes, R: int, rays: int, S: int, io_rows=None, io_cols=None):
    """Dims for a standard-semantics call: rows = R, ios = [[io_rows or R, N_l]]."""
    L = len(shapes)
    io_rows = io_rows or R
    io_cols = io_cols or max(4, max(s[1] for s in shapes))
    ios = [[io_rows, s[1]] for s in shapes]
    return make_dims(L, R, shapes[0][0], rays, 3, S, shapes, ios, shapes[0][0], wp.shape[1],
                     wp.shape[2], wp.shape[2], io_rows, io_cols, 3, 3,
                     bias_shapes=[[s[1], 1] for s in shapes])


def nerf_forward(d: Dims, X, W, B, T, IO, rgba, dists, alpha, cp, wsamp, acc) -> float:
    return float(lib().oracle_nerf_forward(ctypes.byref(d), _p(X), _p(W), _p(B), _p(T), _p(IO),
                                           _p(rgba), _p(dists), _p(alpha), _p(cp), _p(wsamp),
                                           _p(acc)))


def nerf_grad(d: Dims, prim: dict, adj: dict, dreturn: float) -> None:
    """prim/adj keys: X W B T IO rgba dists alpha cp wsamp acc (adj may lack X -> no dX)."""
    keys = ["X", "W", "B", "T", "IO", "rgba", "dists", "alpha", "cp", "wsamp", "acc"]
    args = []
    for k in keys:
        args += [_p(prim[k]), _p(adj.get(k))]
    lib().oracle_nerf_grad(ctypes.byref(d), *args, ctypes.c_float(dreturn))


def mlp_fit_forward(d: Dims, X, W, B, T, IO) -> float:
    return float(lib().oracle_mlp_fit_forward(ctypes.byref(d), _p(X), _p(W), _p(B), _p(T), _p(IO)))


def mlp_fit_grad(d: Dims, prim: dict, adj: dict, dreturn: float) -> None:
    keys = ["X", "W", "B", "T", "IO"]
    args = []
    for k in keys:
        args += [_p(prim[k]), _p(adj.get(k))]
    lib().oracle_mlp_fit_grad(ctypes.byref(d), *args, ctypes.c_float(dreturn))


def mult_a_b(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> None:
    lib().oracle_mult_a_b(_p(a), a.shape[0], a.shape[1], a.shape[1], _p(b), b.shape[0], b.shape[1],
                          b.shape[1], _p(c), c.shape[1])


def positional_encoding_3d(pts: np.ndarray, F: int) -> np.ndarray:
    pts = np.ascontiguousarray(pts, np.float64).reshape(-1, 3)
    out = np.zeros((pts.shape[0], 3 + 6 * F), np.float32)
    lib().oracle_positional_encoding_3d(pts.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        ctypes.c_long(pts.shape[0]), F, _p(out))
    return out


def standard_forward_backward(X, wp, bp, shapes, dists, target, S, seed=None, dX=False):
    """Standard-semantics fwd+grad through the oracle (zero init buffers, io rows = R).
    seed=None -> seed with the loss itself (train_nerf.py:477). Returns dict."""
    X = np.ascontiguousarray(X, np.float32)
    R = X.shape[0]
    rays = R // S
    d = standard_dims(wp, shapes, R, rays, S)
    L = len(shapes)
    z = lambda *s: np.zeros(s, np.float32)
    IO = z(L, d.io_rows, d.io_cols)
    rgba, alpha, cp, ws_, acc = z(rays, S, 4), z(rays, S), z(rays, S), z(rays, S), z(rays, 3)
    dists = np.ascontiguousarray(dists, np.float32).reshape(rays, S)
    T = np.ascontiguousarray(target, np.float32).reshape(rays, 3)
    W = np.ascontiguousarray(wp, np.float32)
    B = np.ascontiguousarray(bp, np.float32)
    loss = nerf_forward(d, X, W, B, T, IO, rgba, dists, alpha, cp, ws_, acc)
    prim = dict(X=X, W=W, B=B, T=T, IO=z(L, d.io_rows, d.io_cols), rgba=z(rays, S, 4), dists=dists,
                alpha=z(rays, S), cp=z(rays, S), wsamp=z(rays, S), acc=z(rays, 3))
    adj = {k: np.zeros_like(v) for k, v in prim.items()}
    if not dX:
        adj.pop("X")
    nerf_grad(d, prim, adj, loss if seed is None else seed)
    return dict(loss=loss, acc=acc, dW=adj["W"], dB=adj["B"], dX=adj.get("X"),
                d_dists=adj["dists"], d_target=adj["T"], d_io=adj["IO"], rgba=rgba, io=IO)


def train_step(X, wp, bp, shapes, dists, target, S, threads=1):
    """CPU baseline (oracle_train_step): returns (loss, dW, dB)."""
    X = np.ascontiguousarray(X, np.float32)
    rays = X.shape[0] // S
    L = len(shapes)
    kd = (ctypes.c_int * L)(*[int(s[0]) for s in shapes])
    nd = (ctypes.c_int * L)(*[int(s[1]) for s in shapes])
    dW = np.zeros_like(wp, dtype=np.float32)
    dB = np.zeros_like(bp, dtype=np.float32)
    dists = np.ascontiguousarray(dists, np.float32)
    target = np.ascontiguousarray(target, np.float32)
    loss = lib().oracle_train_step(L, kd, nd, wp.shape[1], wp.shape[2], _p(X), rays, S, _p(dists),
                                   _p(target), _p(np.ascontiguousarray(wp, np.float32)),
                                   _p(np.ascontiguousarray(bp, np.float32)), _p(dW), _p(dB), threads)
    return float(loss), dW, dB
