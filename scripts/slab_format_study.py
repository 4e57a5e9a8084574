#!/usr/bin/env python3
"""What a narrower slab format would cost in dW / db accuracy, on the CPU.

k1 writes every post-ReLU activation A_l and every gradient G_l = dL/dZ_l as an fp32 "slab"
(14 720 B/sample at cfg3) and k2 reads them back for dW_l = sum_s A_{l-1}[s]^T G_l[s],
db_l = sum_s G_l[s] (reverse_diff.py:673-696). This script rounds A and G to a candidate storage
format, forms dW / db in float64 from the rounded values, and reports the error against float64
from the unrounded values -- the error the FORMAT adds, before any MFMA arithmetic -- in the
units the parity tests use: max |err| / max |want| per tensor (TOL64's 1e-5) and the worst
per-column error / column max (the full-size test's 1e-4).

Formats (all take the fp32 value k1 holds):
  fp32        the current slabs (reference row: no rounding)
  top24       fp32 with the low mantissa byte rounded off (bits + 0x80, keep 24 bits; 16
              significant bits)
  hi16+e5m2   k1's own fp16 hi of x 2^e (e = the row's fp16x3 shift) + its fp16 lo rounded to
              e5m2 (the top byte of the fp16 bit pattern): 3 bytes, hi usable by k2 as it is
  hi16+q8     fp16 hi + the lo as a signed 8-bit multiple of ulp(hi)/256: 3 bytes, 19 bits
  int24       fixed point of x 2^(e+8) per row (|x 2^e| < 2^14): 3 bytes, 2^-23 of the row max
              (the shipped format, lnerf_internal.h a24_slabs)
  A:<format>  only the activation slabs (X, A_l) in the format, the gradient slabs G_l in fp32

    python scripts/slab_format_study.py [--rays 256]
Test/report infrastructure (imports the oracle restatement); writes profiles/r04_slab_formats.json.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def row_shift(x32):
    """fp16x3_shift of each row's max |x| (lnerf_internal.h): m 2^e in [2^13, 2^14)."""
    m = np.abs(x32).max(axis=1)
    e = np.zeros(len(m), np.int64)
    ok = (m > 0) & np.isfinite(m)
    _, ex = np.frexp(m[ok])
    e[ok] = np.minimum(14 - ex, 127)
    return e


def q_top24(x32):
    b = x32.view(np.uint32).astype(np.uint64)
    b = ((b + 0x80) & 0xFFFFFF00).astype(np.uint32)
    return b.view(np.float32)


def q_hi16_e5m2(x32):
    e = row_shift(x32)[:, None]
    y = np.ldexp(x32.astype(np.float64), e)
    hi = y.astype(np.float16)
    lo = (y - hi.astype(np.float64)).astype(np.float16)
    lb = lo.view(np.uint16).astype(np.uint32)
    lb = (((lb + 0x80) & 0xFF00) & 0xFFFF).astype(np.uint16)
    lo8 = lb.view(np.float16)
    return np.ldexp(hi.astype(np.float64) + lo8.astype(np.float64), -e).astype(np.float32)


def q_hi16_q8(x32):
    e = row_shift(x32)[:, None]
    y = np.ldexp(x32.astype(np.float64), e)
    hi = y.astype(np.float16).astype(np.float64)
    _, eh = np.frexp(np.where(hi == 0, 1.0, hi))
    ulp = np.ldexp(1.0, np.maximum(eh - 11, -24))   # fp16 ulp (subnormal floor 2^-24)
    q = np.clip(np.rint((y - hi) / ulp * 256.0), -127, 127)
    return np.ldexp(hi + q * ulp / 256.0, -e).astype(np.float32)


def q_int24(x32):
    """The shipped format (lnerf_internal.h a24_slabs): q = rint(x 2^(e + 8)), |q| < 2^22, via the
    fp32 add of 1.5 2^23 (round to nearest even)."""
    e = row_shift(x32)[:, None]
    y = np.rint(np.ldexp(x32.astype(np.float64), e + 8))
    y = np.clip(y, -(2 ** 22 - 1), 2 ** 22 - 1)
    return np.ldexp(y, -(e + 8)).astype(np.float32)


FORMATS = {"fp32": lambda x: x, "top24": q_top24, "hi16+e5m2": q_hi16_e5m2, "hi16+q8": q_hi16_q8,
           "int24": q_int24}


def slabs(X, ws, bs, dists, target, S, seed=1.0):
    """A_{l-1} (layer inputs, X for l = 0) and G_l = dL/dZ_l of every layer, float64, from
    nerf_np.nerf_forward_backward (scripts/nerf.py:1-304 and its rev_diff)."""
    import nerf_np
    r = nerf_np.nerf_forward_backward(X, ws, bs, dists, target, S, seed=seed)
    return r["A"], r["G"]


def study(name, X, ws, bs, dists, target, S):
    A, G = slabs(X, ws, bs, dists, target, S)
    out = {}
    exact_dW = [a.T @ g for a, g in zip(A, G)]
    exact_db = [g.sum(0) for g in G]
    variants = [(f, q, True) for f, q in FORMATS.items()] + \
        [("A:" + f, q, False) for f, q in FORMATS.items() if f != "fp32"]
    for fname, q, both in variants:
        worst_t, worst_c, worst_b = 0.0, 0.0, 0.0
        for l, (a, g) in enumerate(zip(A, G)):
            qa = q(a.astype(np.float32)).astype(np.float64)
            qg = (q(g.astype(np.float32)) if both else g.astype(np.float32)).astype(np.float64)
            dW = qa.T @ qg
            want = exact_dW[l]
            err = np.abs(dW - want)
            mx = np.abs(want).max()
            if mx > 0:
                worst_t = max(worst_t, float(err.max() / mx))
            cm = np.abs(want).max(axis=0)
            live = cm > 0
            if live.any():
                worst_c = max(worst_c, float((err.max(axis=0)[live] / cm[live]).max()))
            db = qg.sum(0)
            bm = np.abs(exact_db[l]).max()
            if bm > 0:
                worst_b = max(worst_b, float(np.abs(db - exact_db[l]).max() / bm))
        out[fname] = {"dW_max_rel": worst_t, "dW_worst_column_rel": worst_c, "db_max_rel": worst_b}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=256)
    args = ap.parse_args()
    import nerf_np
    res = {}
    for cfg, rays in (("cfg3", args.rays), ("cfg2", None)):
        w = nerf_np.make_workload(cfg, rays=rays)
        res[f"{cfg}_{w.N}rays"] = study(cfg, w.X, w.ws, w.bs, w.dists, w.target, w.S)
    gdir = os.path.join(REPO, "tests", "golden")
    for fn in sorted(os.listdir(gdir)):
        if not fn.endswith(".npz"):
            continue
        g = dict(np.load(os.path.join(gdir, fn), allow_pickle=False))
        if "shapes" not in g or "X" not in g:
            continue
        shapes = [tuple(int(v) for v in s) for s in g["shapes"]]
        ws = [g["wp"][l, :k, :n] for l, (k, n) in enumerate(shapes)]
        bs = [g["bp"][l, :n] for l, (_, n) in enumerate(shapes)]
        with np.errstate(all="ignore"):
            r = study(fn, g["X"], ws, bs, g["dists"], g["target"], int(g["S"]))
        res[fn] = r
    print(f"{'workload':34s} {'format':10s} {'dW max/max':>11s} {'dW worst col':>13s} {'db max/max':>11s}")
    for k, v in res.items():
        for f, e in v.items():
            print(f"{k:34s} {f:10s} {e['dW_max_rel']:11.3g} {e['dW_worst_column_rel']:13.3g} {e['db_max_rel']:11.3g}")
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r04_slab_formats.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
