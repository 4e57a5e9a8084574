#!/usr/bin/env python3
"""Compat-boundary benchmark (measurement script, not the headline bench): the reference's own
per-chunk call pattern through the loma C-ABI, as an unchanged train_nerf.py drives it.

One training chunk = nerf_evaluate_and_march + grad_nerf_evaluate_and_march on the reference
chunk (train_nerf.py:190-200, 296-478: 4 rays x 30 samples, PE F=5, MLP 33->30->30->4, the
256-row fake trace, loss-seeded gradient), with the nested host pointer tables loma's C backend
emits. Timed through libloma_nerf.so on the GPU (host gather, H2D, the loma-order kernels, D2H,
synchronous like loma) and through the loma-order C restatement (oracle/, one host core) on the
same buffers. The pointer tables are built once (the reference's drivers build them per chunk in
Python for either library, mlp_utils.py:67-110, so that cost is common and excluded); the GPU
time is the library call itself: gather through the tables, H2D, kernels, D2H, scatter.

    python scripts/bench_compat.py [--iters 200]

Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in ("oracle", "loma-nerf_amd", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    import lnerf
    import nerf_np
    from loma_calls import NerfCall

    lib = lnerf.load_library(lnerf.LIB_PATH)
    w = nerf_np.make_workload("chunk")
    c = NerfCall(w.X, w.wp, w.bp, [x.shape for x in w.ws], w.target, w.dists, w.S)
    samples = c.N * c.S

    import ctypes
    import numpy as np
    from loma_marshal import to_ctypes
    T = to_ctypes
    fwd_args = (T(c.X), c.X.shape[0], c.X.shape[1], T(c.wp), T(c.bp), T(c.target), c.N, 3, c.L,
                T(c.ws_shape), T(c.bs_shape), T(c.ios), T(c.io), T(c.rgba), c.S, T(c.dists),
                T(c.alpha), T(c.cp), T(c.wsamp), T(c.acc))
    dc = {k: T(v) for k, v in c.d.items()}
    ints = [ctypes.c_int(0) for _ in range(6)]
    z = lambda a: T(np.zeros_like(a))
    grad_head = (T(c.X), dc["X"], c.X.shape[0], ctypes.byref(ints[0]), c.X.shape[1],
                 ctypes.byref(ints[1]), T(c.wp), dc["W"], T(c.bp), dc["B"], T(c.target), dc["T"],
                 c.N, ctypes.byref(ints[2]), 3, ctypes.byref(ints[3]), c.L, ctypes.byref(ints[4]),
                 T(c.ws_shape), z(c.ws_shape), T(c.bs_shape), z(c.bs_shape), T(c.ios), z(c.ios),
                 T(c.io), dc["IO"], T(c.rgba), dc["rgba"], c.S, ctypes.byref(ints[5]), T(c.dists),
                 dc["dists"], T(c.alpha), dc["alpha"], T(c.cp), dc["cp"], T(c.wsamp), dc["wsamp"],
                 T(c.acc), dc["acc"])

    def gpu_chunk():
        loss = lib.nerf_evaluate_and_march(*fwd_args)
        lib.grad_nerf_evaluate_and_march(*grad_head, loss)
        return loss

    def gpu_chunk_marshal():   # + building the pointer tables in Python per call, as the tests do
        loss = c.lib_forward(lib)["loss"]
        c.lib_grad(lib, loss)
        return loss

    def cpu_chunk():
        loss = c.oracle_forward()["loss"]
        c.oracle_grad(loss)
        return loss

    out = {"metric": "compat-ABI training chunk (fwd + grad call pair), reference chunk",
           "workload": f"{c.N} rays x {c.S} samples, MLP 33->30->30->4, 256-row fake trace",
           "iters": args.iters}
    for name, fn in (("gpu_compat", gpu_chunk), ("gpu_compat_incl_python_marshalling", gpu_chunk_marshal),
                     ("cpu_oracle_1core", cpu_chunk)):
        for _ in range(10):
            fn()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            loss = fn()
        dt = (time.perf_counter() - t0) / args.iters
        out[name] = {"ms_per_chunk": dt * 1e3, "ray_samples_per_s": samples / dt, "loss": float(loss)}
    out["note"] = ("per-call latency path: the loma ABI is synchronous and per-chunk (<= 256 "
                   "rows), so these calls are launch/marshalling-bound; throughput goes through "
                   "the batched native API (bench.py)")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
