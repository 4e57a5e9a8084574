#!/usr/bin/env python3
"""Accuracy of each step implementation against the float64 numpy restatement (oracle/nerf_np.py)
on a cfg3 subset (the bench MLP 33->256x7->4, 64 samples): the C loma-order fp32 oracle, the
generic device path, the fused path with the fp16x3 split (k16 + dw16, the default) and with the
bf16x6 split (k16 + dw16). Reported twice: on all rays, and
without the rays holding a ReLU decision below fp32 resolution (nerf_np.relu_tie_rays: |z| <
5e-7 sum|terms|, where any fp32 summation order may decide either way and the flipped sample's
whole gradient row moves). Test/report infrastructure (imports the oracle); writes
gpurun_out/precision.json.

    python scripts/precision_report.py [--rays 64]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in ("oracle", "loma-nerf_amd", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))


def errors(got, ref):
    out = {}
    for k in ("acc", "dW", "dB", "d_dists", "d_target"):
        g = np.asarray(got[k], np.float64)
        r = np.asarray(ref[k], np.float64)
        scale = np.abs(r).max()
        big = np.abs(r) > 1e-3 * scale
        out[k] = {"max_abs_over_max": float(np.abs(g - r).max() / scale),
                  "median_rel": float(np.median(np.abs(g - r)[big] / np.abs(r)[big])),
                  "p99_rel": float(np.percentile(np.abs(g - r)[big] / np.abs(r)[big], 99))}
    out["loss_rel"] = float(abs(got["loss"] - ref["loss"]) / abs(ref["loss"]))
    return out


def f64_reference(w):
    import nerf_np
    X64 = nerf_np.positional_encoding_3d(w.pts32.astype(np.float64), w.F).reshape(w.X.shape)
    ref = nerf_np.nerf_forward_backward(X64, [x.astype(np.float64) for x in w.ws],
                                        [x.astype(np.float64) for x in w.bs], w.dists, w.target,
                                        w.S, seed=1.0)
    dW = np.zeros(w.wp.shape)
    dB = np.zeros(w.bp.shape)
    for l in range(len(w.ws)):
        k, n = w.ws[l].shape
        dW[l, :k, :n] = ref["dW"][l]
        dB[l, :n] = ref["db"][l]
    return dict(loss=ref["loss"], acc=ref["acc"], dW=dW, dB=dB, d_dists=ref["d_dists"],
                d_target=ref["d_target"])


def report(eng, w):
    import lnerf
    from test_gpu_native import oracle_ref, run_native
    ref = f64_reference(w)
    rep = {"oracle_c_fp32": errors(oracle_ref(w, seed=1.0), ref),
           "generic_device": errors(run_native(eng, w, seed=1.0, flags=lnerf.GENERIC), ref),
           "fused_f16x3_k16_dw16": errors(run_native(eng, w, seed=1.0, flags=lnerf.FAST), ref),
           "fused_bf16x6_k16_dw16": errors(run_native(eng, w, seed=1.0, flags=lnerf.FAST | lnerf.MFMA_BF16X6), ref)}
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=64)
    args = ap.parse_args()
    import lnerf
    import nerf_np

    w = nerf_np.make_workload("cfg3", rays=args.rays)
    ties = nerf_np.relu_tie_rays(w)
    eng = lnerf.Engine(0)
    rep = {"workload": f"cfg3 subset: {args.rays} rays x {w.S} samples, MLP 33->256x7->4, seed 1",
           "reference": "float64 numpy restatement (oracle/nerf_np.py)",
           "all_rays": report(eng, w),
           "tie_rays": [int(r) for r in ties],
           "without_tie_rays": report(eng, nerf_np.without_relu_ties(w))}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "precision.json"), "w") as fh:
        json.dump(rep, fh, indent=1)
    for part in ("all_rays", "without_tie_rays"):
        print(part)
        for k, v in rep[part].items():
            print(" ", k, {kk: (float("%.3g" % vv["max_abs_over_max"]) if isinstance(vv, dict) else vv)
                           for kk, vv in v.items()})
    eng.close()


if __name__ == "__main__":
    main()
