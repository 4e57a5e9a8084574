"""Test helper: build the exact argument sets train_nerf.py / fit_img.py pass to the loma ABI,
run them through libloma_nerf.so (GPU) and through the C oracle, and return both results.

train_nerf.py:216-241 (shapes, the 256-row fake trace for intermediate_output_shapes, padded
weights), :296-317 (per-chunk buffers), :325-366 (forward call), :370-478 (grad call).
"""
from __future__ import annotations

import ctypes

import numpy as np

import oracle
from loma_marshal import from_ctypes, to_ctypes


class NerfCall:
    """All numpy buffers of one nerf_evaluate_and_march / grad call (float32 unless int)."""

    def __init__(self, X, wp, bp, wshapes, target, dists, S, ios=None, io_alloc=(256, 256),
                 rng=None, init_scale=0.0, adj_scale=0.0):
        rng = rng or np.random.RandomState(5)
        L = wp.shape[0]
        self.L, self.S = L, S
        self.X = np.ascontiguousarray(X, np.float32)
        self.wp = np.ascontiguousarray(wp, np.float32)
        self.bp = np.ascontiguousarray(bp, np.float32)
        self.ws_shape = np.array(wshapes, np.int32)
        self.bs_shape = np.array([[s[1], 1] for s in wshapes], np.int32)
        if ios is None:
            ios = [[256, s[1]] for s in wshapes]   # the train_nerf.py:230-234 fake trace
        self.ios = np.array(ios, np.int32)
        self.target = np.ascontiguousarray(target, np.float32)
        self.dists = np.ascontiguousarray(dists, np.float32)
        N = self.target.shape[0]
        self.N = N
        rows, cols = io_alloc
        z = lambda *s: np.zeros(s, np.float32)
        g = lambda *s: (rng.standard_normal(s) * init_scale).astype(np.float32)
        self.io = g(L, rows, cols)            # intermediate_outputs (loma accumulates into it)
        self.rgba = z(N, S, 4)
        self.alpha = z(N, S)
        self.cp = z(N, S)
        self.wsamp = z(N, S)
        self.acc = g(N, 3)
        a = lambda *s: (rng.standard_normal(s) * adj_scale).astype(np.float32)
        self.d = dict(X=a(*self.X.shape), W=a(*self.wp.shape), B=a(*self.bp.shape),
                      T=a(*self.target.shape), IO=a(L, rows, cols), rgba=a(N, S, 4),
                      dists=a(N, S), alpha=a(N, S), cp=a(N, S), wsamp=a(N, S), acc=a(N, 3))

    # ---- oracle ---------------------------------------------------------------------------
    def dims(self):
        L = self.L
        return oracle.make_dims(L, self.X.shape[0], self.X.shape[1], self.N, 3, self.S,
                                self.ws_shape, self.ios, self.X.shape[1], self.wp.shape[1],
                                self.wp.shape[2], self.bp.shape[1], self.io.shape[1],
                                self.io.shape[2], 3, 3, bias_shapes=self.bs_shape)

    def oracle_forward(self):
        io, rgba, al, cp, ws, acc = (self.io.copy(), self.rgba.copy(), self.alpha.copy(),
                                     self.cp.copy(), self.wsamp.copy(), self.acc.copy())
        loss = oracle.nerf_forward(self.dims(), self.X, self.wp, self.bp, self.target, io, rgba,
                                   self.dists, al, cp, ws, acc)
        return dict(loss=loss, io=io, rgba=rgba, alpha=al, cp=cp, wsamp=ws, acc=acc)

    def oracle_grad(self, seed):
        prim = dict(X=self.X, W=self.wp, B=self.bp, T=self.target, IO=self.io, rgba=self.rgba,
                    dists=self.dists, alpha=self.alpha, cp=self.cp, wsamp=self.wsamp, acc=self.acc)
        adj = {k: v.copy() for k, v in self.d.items()}
        oracle.nerf_grad(self.dims(), prim, adj, seed)
        return adj

    # ---- library (loma ABI) -----------------------------------------------------------------
    def lib_forward(self, lib):
        io_c = to_ctypes(self.io)
        rgba_c, al_c, cp_c, ws_c = (to_ctypes(self.rgba), to_ctypes(self.alpha),
                                    to_ctypes(self.cp), to_ctypes(self.wsamp))
        acc_c = to_ctypes(self.acc)
        loss = lib.nerf_evaluate_and_march(
            to_ctypes(self.X), self.X.shape[0], self.X.shape[1], to_ctypes(self.wp),
            to_ctypes(self.bp), to_ctypes(self.target), self.N, 3, self.L,
            to_ctypes(self.ws_shape), to_ctypes(self.bs_shape), to_ctypes(self.ios), io_c, rgba_c,
            self.S, to_ctypes(self.dists), al_c, cp_c, ws_c, acc_c)
        return dict(loss=loss, io=from_ctypes(io_c, self.io.shape),
                    rgba=from_ctypes(rgba_c, self.rgba.shape),
                    alpha=from_ctypes(al_c, self.alpha.shape), cp=from_ctypes(cp_c, self.cp.shape),
                    wsamp=from_ctypes(ws_c, self.wsamp.shape), acc=from_ctypes(acc_c, self.acc.shape))

    def lib_grad(self, lib, seed):
        dc = {k: to_ctypes(v) for k, v in self.d.items()}
        ints = [ctypes.c_int(0) for _ in range(5)]
        zi = lambda a: to_ctypes(np.zeros_like(a))
        io_c = to_ctypes(self.io)
        lib.grad_nerf_evaluate_and_march(
            to_ctypes(self.X), dc["X"], self.X.shape[0], ctypes.byref(ints[0]), self.X.shape[1],
            ctypes.byref(ints[1]), to_ctypes(self.wp), dc["W"], to_ctypes(self.bp), dc["B"],
            to_ctypes(self.target), dc["T"], self.N, ctypes.byref(ints[2]), 3,
            ctypes.byref(ints[3]), self.L, ctypes.byref(ints[4]), to_ctypes(self.ws_shape),
            zi(self.ws_shape), to_ctypes(self.bs_shape), zi(self.bs_shape), to_ctypes(self.ios),
            zi(self.ios), io_c, dc["IO"], to_ctypes(self.rgba), dc["rgba"], self.S,
            ctypes.byref(ctypes.c_int(0)), to_ctypes(self.dists), dc["dists"],
            to_ctypes(self.alpha), dc["alpha"], to_ctypes(self.cp), dc["cp"],
            to_ctypes(self.wsamp), dc["wsamp"], to_ctypes(self.acc), dc["acc"], seed)
        out = {k: from_ctypes(v, self.d[k].shape) for k, v in dc.items()}
        out["_io_after"] = from_ctypes(io_c, self.io.shape)   # primal must be unchanged
        out["_ints"] = [i.value for i in ints]
        return out


def assert_close(name, got, want, rtol=1e-5, atol_scale=1e-5):
    """|got - want| <= rtol*|want| + atol_scale*max|want| (fp32 parity)."""
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (name, got.shape, want.shape)
    scale = max(np.abs(want).max(initial=0.0), 1e-30)
    err = np.abs(got - want)
    bad = err > rtol * np.abs(want) + atol_scale * scale
    bad &= ~(np.isnan(got) & np.isnan(want))
    if bad.any():
        i = np.unravel_index(np.argmax(np.where(bad, err, -1)), err.shape)
        raise AssertionError(f"{name}: {bad.sum()} / {bad.size} mismatches; worst at {i}: got "
                             f"{got[i]!r} want {want[i]!r} (max|want|={scale:.3g})")
