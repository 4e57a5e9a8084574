#!/usr/bin/env python3
"""Compat-boundary benchmark (measurement script, not the headline bench): the reference's own
per-chunk call pattern through the loma C-ABI, as an unchanged train_nerf.py drives it.

One training chunk = nerf_evaluate_and_march + grad_nerf_evaluate_and_march on the reference
chunk (train_nerf.py:190-200, 296-478: 4 rays x 30 samples, PE F=5, MLP 33->30->30->4, the
256-row fake trace, loss-seeded gradient), with the nested host pointer tables loma's C backend
emits. Both legs run on the SAME tables:
  * GPU: libloma_nerf.so (host gather, H2D, the loma-order kernels, D2H, scatter; synchronous
    like loma);
  * CPU: the loma-order C restatement behind the same ABI (oracle/nerf_oracle_abi.c: its own
    gather + the oracle + scatter), one host core.
Before every call pair the buffers train_nerf.py allocates fresh per chunk are zeroed in place
through the tables (train_nerf.py:313-317: sample_rgba, alpha, cumprod_alpha, weights_samples,
accumulated_color; :370-392: every adjoint; intermediate_outputs is allocated once and zeroed
here too, so every iteration computes the same chunk from the same state). The zeroing and the
pointer-table construction (the drivers' own Python cost, mlp_utils.py:67-110, common to both
libraries) are outside the timed calls; both legs must report the same loss.

    python scripts/bench_compat.py [--iters 200]

Prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in ("oracle", "loma-nerf_amd", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))


def zero_table(t):
    """memset every float row of a to_ctypes() table in place (the caller's buffer stays)."""
    for obj in t._keep[1] if isinstance(t._keep, tuple) else ():
        if isinstance(obj, ctypes.Array) and obj._type_ is ctypes.c_float:
            ctypes.memset(obj, 0, ctypes.sizeof(obj))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--cpu-only", action="store_true", help="the oracle leg alone (no GPU)")
    args = ap.parse_args()
    import numpy as np
    import lnerf
    import nerf_np
    import oracle
    from loma_calls import NerfCall
    from loma_marshal import to_ctypes

    lib = None if args.cpu_only else lnerf.load_library(lnerf.LIB_PATH)
    olib = oracle.lib()
    olib.oracle_abi_nerf_evaluate_and_march.argtypes = lnerf.NERF_ARGTYPES
    olib.oracle_abi_nerf_evaluate_and_march.restype = ctypes.c_float
    olib.oracle_abi_grad_nerf_evaluate_and_march.argtypes = lnerf.rev_argtypes(lnerf.NERF_ARGTYPES)
    olib.oracle_abi_grad_nerf_evaluate_and_march.restype = None

    w = nerf_np.make_workload("chunk")
    c = NerfCall(w.X, w.wp, w.bp, [x.shape for x in w.ws], w.target, w.dists, w.S)
    samples = c.N * c.S
    T = to_ctypes
    io, rgba, alpha, cp, wsamp, acc = T(c.io), T(c.rgba), T(c.alpha), T(c.cp), T(c.wsamp), T(c.acc)
    fwd_args = (T(c.X), c.X.shape[0], c.X.shape[1], T(c.wp), T(c.bp), T(c.target), c.N, 3, c.L,
                T(c.ws_shape), T(c.bs_shape), T(c.ios), io, rgba, c.S, T(c.dists), alpha, cp, wsamp,
                acc)
    dc = {k: T(np.zeros_like(v)) for k, v in c.d.items()}
    ints = [ctypes.c_int(0) for _ in range(6)]
    z = lambda a: T(np.zeros_like(a))
    grad_head = (T(c.X), dc["X"], c.X.shape[0], ctypes.byref(ints[0]), c.X.shape[1],
                 ctypes.byref(ints[1]), T(c.wp), dc["W"], T(c.bp), dc["B"], T(c.target), dc["T"],
                 c.N, ctypes.byref(ints[2]), 3, ctypes.byref(ints[3]), c.L, ctypes.byref(ints[4]),
                 T(c.ws_shape), z(c.ws_shape), T(c.bs_shape), z(c.bs_shape), T(c.ios), z(c.ios),
                 io, dc["IO"], rgba, dc["rgba"], c.S, ctypes.byref(ints[5]), T(c.dists),
                 dc["dists"], alpha, dc["alpha"], cp, dc["cp"], wsamp, dc["wsamp"], acc, dc["acc"])
    fresh = [io, rgba, alpha, cp, wsamp, acc] + list(dc.values())

    def chunk(fwd, grad):
        """one call pair on freshly zeroed buffers; returns (seconds in the two calls, loss)"""
        for t in fresh:
            zero_table(t)
        t0 = time.perf_counter()
        loss = fwd(*fwd_args)
        grad(*grad_head, loss)
        dt = time.perf_counter() - t0
        return dt, loss

    legs = {} if lib is None else {"gpu_compat": (lib.nerf_evaluate_and_march,
                                                  lib.grad_nerf_evaluate_and_march)}
    legs |= {"cpu_oracle_1core": (olib.oracle_abi_nerf_evaluate_and_march,
                                 olib.oracle_abi_grad_nerf_evaluate_and_march)}
    out = {"metric": "compat-ABI training chunk (fwd + grad call pair), reference chunk",
           "workload": f"{c.N} rays x {c.S} samples, MLP 33->30->30->4, 256-row fake trace, "
                       f"buffers zeroed per chunk as train_nerf.py does",
           "iters": args.iters}
    dws = {}
    for name, (fwd, grad) in legs.items():
        for _ in range(10):
            chunk(fwd, grad)
        tot, losses = 0.0, []
        for _ in range(args.iters):
            dt, loss = chunk(fwd, grad)
            tot += dt
            losses.append(loss)
        dt = tot / args.iters
        from loma_marshal import from_ctypes
        dws[name] = from_ctypes(dc["W"], c.wp.shape)
        out[name] = {"ms_per_chunk": dt * 1e3, "ray_samples_per_s": samples / dt,
                     "loss": float(losses[-1]), "loss_spread": float(max(losses) - min(losses))}
    if lib is None:
        print(json.dumps(out), flush=True)
        return
    g, cpu = out["gpu_compat"], out["cpu_oracle_1core"]
    out["same_loss"] = abs(g["loss"] - cpu["loss"]) <= 1e-5 * abs(cpu["loss"])
    scale = float(np.abs(dws["cpu_oracle_1core"]).max())
    out["max_dw_err_rel"] = float(np.abs(dws["gpu_compat"] - dws["cpu_oracle_1core"]).max()) / scale
    out["gpu_speedup"] = cpu["ms_per_chunk"] / g["ms_per_chunk"]
    out["note"] = ("per-call latency path: the loma ABI is synchronous and per-chunk (<= 256 rows), so "
                   "these calls are launch/transfer-bound; throughput goes through the batched native "
                   "API (bench.py)")
    print(json.dumps(out), flush=True)
    assert out["same_loss"], (g["loss"], cpu["loss"])


if __name__ == "__main__":
    main()
