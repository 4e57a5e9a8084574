"""CPU study for the fp16x3 column guard (round 6): per layer, the column-independent bound of what
k1's fp16x3 reverse chain can lose in a dW element, E_l = sum_s 2^(14 - xa_s) 2^(14 - xg_s) (the
row scales k1's shifts imply), against each live column's max |dW|. Prints, per layer, the smallest
live column max over E_l -- the guard fires (whole step re-run on the bf16x6 split) when that falls
below 1e-4^-1 x 2^-38 x the guard's safety factor -- for the cfg3 bench batch and the edge fixtures.

  python scripts/xcheck_study.py [--rays 4096]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import nerf_np  # noqa: E402


def scale_of(X):
    m = np.abs(X).max(axis=1).astype(np.float32)
    out = np.zeros(len(m))
    ok = (m > 0) & np.isfinite(m)
    out[ok] = np.ldexp(1.0, np.frexp(m[ok])[1])   # 2^(14 - xa): the power of two above the row max
    return out


def study(X, ws, bs, dists, target, S, chunk=256):
    L = len(ws)
    E = np.zeros(L)
    dW = [0.0] * L
    N = X.shape[0] // S
    for lo in range(0, N, chunk):
        hi = min(N, lo + chunk)
        rows = slice(lo * S, hi * S)
        with np.errstate(all="ignore"):
            r = nerf_np.nerf_forward_backward(X[rows], ws, bs, dists[lo:hi], target[lo:hi], S)
        for l in range(L):
            E[l] += float((scale_of(r["A"][l]) * scale_of(r["G"][l])).sum())
            dW[l] = dW[l] + np.nan_to_num(r["dW"][l])
    out = []
    for l in range(L):
        cm = np.abs(dW[l]).max(axis=0)
        live = cm > 0
        out.append((float(cm[live].min() / E[l]) if live.any() and E[l] > 0 else float("inf"),
                    float(np.median(cm[live]) / E[l]) if live.any() and E[l] > 0 else float("inf")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=4096)
    a = ap.parse_args()
    w = nerf_np.make_workload("cfg3", rays=a.rays)
    print("cfg3 bench batch: per layer log2(min live colmax / E_l), log2(median colmax / E_l)")
    for l, (mn, md) in enumerate(study(w.X, w.ws, w.bs, w.dists, w.target, w.S)):
        print(f"  layer {l}: {np.log2(mn):7.2f} {np.log2(md):7.2f}")
    for name in ("edge_finite_6x8.npz", "deep8_w64_2x64.npz", "trained_weights_8x16.npz", "chunk_4x30.npz"):
        g = dict(np.load(os.path.join(os.path.dirname(HERE), "tests", "golden", name), allow_pickle=False))
        if "shapes" not in g:
            continue
        shapes = [tuple(int(v) for v in s) for s in g["shapes"]]
        ws = [g["wp"][l, :k, :n] for l, (k, n) in enumerate(shapes)]
        bs = [g["bp"][l, :n] for l, (_, n) in enumerate(shapes)]
        res = study(g["X"], ws, bs, g["dists"], g["target"], int(g["S"]))
        print(name, " ".join(f"{np.log2(mn):.1f}" for mn, _ in res))


if __name__ == "__main__":
    main()
