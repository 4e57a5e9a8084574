#!/usr/bin/env python3
"""Diagnostic (test infrastructure): where the fused dW differs from the loma-order C oracle and
from the float64 restatement on a cfg3 subset, per layer, for both fused kernels
(LNERF_K16=1: the wave-pair kernel; LNERF_K16=0: the one-wave-per-SIMD kernel).

    python scripts/diag_dw.py [--rays 24]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in ("oracle", "loma-nerf_amd", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=24)
    ap.add_argument("--seed-one", action="store_true")
    args = ap.parse_args()
    import lnerf
    import nerf_np
    from test_gpu_native import oracle_ref, run_native

    w = nerf_np.make_workload("cfg3", rays=args.rays)
    seed = 1.0 if args.seed_one else None
    want = oracle_ref(w, seed=seed)
    X64 = nerf_np.positional_encoding_3d(w.pts32.astype(np.float64), w.F).reshape(w.X.shape)
    ref = nerf_np.nerf_forward_backward(X64, [x.astype(np.float64) for x in w.ws],
                                        [x.astype(np.float64) for x in w.bs], w.dists, w.target,
                                        w.S, seed=1.0)
    s64 = ref["loss"] if seed is None else 1.0
    d64 = np.zeros(w.wp.shape)
    for l in range(len(w.ws)):
        k, n = w.ws[l].shape
        d64[l, :k, :n] = ref["dW"][l] * s64
    eng = lnerf.Engine(0)
    for k16 in ("1", "0"):
        os.environ["LNERF_K16"] = k16
        got = run_native(eng, w, seed=seed, flags=lnerf.FAST)
        print(f"== LNERF_K16={k16}: loss {got['loss']:.7g} oracle {want['loss']:.7g} f64 {ref['loss']:.7g}")
        scale = np.abs(want["dW"]).max()
        for l in range(len(w.ws)):
            g, o, r = got["dW"][l], want["dW"][l], d64[l]
            err_o = np.abs(g - o)
            bad = err_o > 1e-4 * np.abs(o) + 1e-4 * scale
            rows = np.unique(np.nonzero(bad)[0])
            cols = np.unique(np.nonzero(bad)[1])
            print(f"  l{l}: max|got-oracle|/max {err_o.max() / scale:.2e}  max|got-f64|/max "
                  f"{np.abs(g - r).max() / scale:.2e}  max|oracle-f64|/max {np.abs(o - r).max() / scale:.2e}"
                  f"  bad {bad.sum()} rows {rows[:8].tolist()}{'...' if len(rows) > 8 else ''} "
                  f"cols {cols[:8].tolist()}{'...' if len(cols) > 8 else ''}")
        db = np.abs(got["dB"] - want["dB"]).max() / np.abs(want["dB"]).max()
        print(f"  dB max|got-oracle|/max {db:.2e}; acc {np.abs(got['acc'] - want['acc']).max():.2e}")
    eng.close()


if __name__ == "__main__":
    main()
