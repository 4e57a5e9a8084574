"""Generates the golden fixtures in tests/golden/ (committed; re-run to regenerate).

Expected outputs come from the float64 numpy restatement (oracle/nerf_np.py), which is
independent of the C oracle and of the HIP kernels; the inputs reproduce the reference's own
producers (train_nerf.py:23-62, :289-311; pos_encoding.py:38-69; mlp_utils.py:166-204, seed 215).
The reference ships no golden vectors for this path, so these pin our two
restatements against each other; the mult_a_b case is the reference's own known answer
(fit_img.py:363-374). The trained-weights case reads the reference's models/weights.npy and
models/biases.npy (plain .npy, allow_pickle=False) when /root/reference is present.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import nerf_np  # noqa: E402


def pack(w, out, **extra):
    d = dict(X=w.X, pts=w.pts, dists=w.dists, target=w.target, wp=w.wp, bp=w.bp,
             shapes=np.array([x.shape for x in w.ws], np.int32), S=np.int32(w.S), F=np.int32(w.F),
             loss=np.float64(out["loss"]), acc=out["acc"], d_dists=out["d_dists"],
             d_target=out["d_target"], dX=out["dX"])
    L = len(w.ws)
    dWp = np.zeros(w.wp.shape, np.float64)
    dBp = np.zeros(w.bp.shape, np.float64)
    for l in range(L):
        k, n = w.ws[l].shape
        dWp[l, :k, :n] = out["dW"][l]
        dBp[l, :n] = out["db"][l]
    d.update(dW=dWp, dB=dBp)
    d.update(extra)
    return d


def main():
    # 1. the train_nerf.py chunk: 4 rays x 30 samples, 33->30->30->4, seed = 1 (unit)
    w = nerf_np.make_workload("chunk")
    out = nerf_np.nerf_forward_backward(w.X, w.ws, w.bs, w.dists, w.target, w.S, seed=1.0)
    np.savez_compressed(os.path.join(HERE, "chunk_4x30.npz"), **pack(w, out))
    # 2. the bench MLP's depth (8 layers) at width 64 (33->64x7->4) on 2 rays x 64 samples
    w = nerf_np.make_workload("cfg3", rays=2, filter_size=64)
    out = nerf_np.nerf_forward_backward(w.X, w.ws, w.bs, w.dists, w.target, w.S, seed=1.0)
    np.savez_compressed(os.path.join(HERE, "deep8_w64_2x64.npz"), **pack(w, out))
    # 3. the reference's saved weights (3->16->16->4, no PE) on raw sample positions
    ref = "/root/reference/models"
    if os.path.exists(os.path.join(ref, "weights.npy")):
        wp = np.load(os.path.join(ref, "weights.npy"), allow_pickle=False).astype(np.float32)
        bp = np.load(os.path.join(ref, "biases.npy"), allow_pickle=False).astype(np.float32)
        shapes = [(3, 16), (16, 16), (16, 4)]
        ws = [wp[l, :k, :n] for l, (k, n) in enumerate(shapes)]
        bs = [bp[l, :n] for l, (k, n) in enumerate(shapes)]
        base = nerf_np.make_workload("chunk", rays=8, samples=16, num_functions=0)
        X = base.pts.reshape(-1, 3).astype(np.float32)
        out = nerf_np.nerf_forward_backward(X, ws, bs, base.dists, base.target, base.S, seed=1.0)
        w = nerf_np.Workload(base.pts, base.pts32, X, base.dists, base.target, ws, bs, wp, bp, 0,
                             base.S, base.N)
        np.savez_compressed(os.path.join(HERE, "trained_weights_8x16.npz"), **pack(w, out))
    # 4. mult_a_b known answer (fit_img.py:363-374)
    np.savez(os.path.join(HERE, "mult_a_b.npz"),
             a=np.array([[1, 2], [3, 4], [5, 6]], np.float32),
             b=np.array([[100], [200]], np.float32),
             c=np.array([[500], [1100], [1700]], np.float32))
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
