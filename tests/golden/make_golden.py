"""Generates the golden fixtures in tests/golden/ (committed; re-run to regenerate).

Expected outputs come from the float64 numpy restatement (oracle/nerf_np.py), which is
independent of the C oracle and of the HIP kernels -- except the edge-numerics fixtures, whose
expected values are the loma-order fp32 C oracle's (oracle/nerf_oracle.c: NaN adjoints and fp32
underflow are properties of the reference's fp32 semantics), with the float64 values alongside
(f64_*); the inputs reproduce the reference's own
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


# Edge-numerics fixtures. An identity MLP 8 -> 8 -> 8 -> 4 (W0 = W1 = I, W2[c][c] = 1,
# W2[c+4][c] = -1, zero biases) makes every head pre-activation z_c = relu(x_c) - relu(x_{c+4}),
# so each sample's rgb / sigma is set directly by its input row; 8 samples per ray, dists of
# linspace(2, 6, 8) with the reference's trailing 1e8 (train_nerf.py:306).
#   sigma0     sigma = ReLU(-1) = 0 on every sample (alpha 0, T stays 1)
#   tiny       sigma = (j+1) 1e-9 with every feature of the sample as small (a value 2^-40 below
#              its row's largest is a ReLU tie at fp32 resolution in any real MLP, so each row is
#              kept to one magnitude): alpha underflows to 0
#              for delta 0.57 in fp32, the last sample's sigma * 1e8 = 0.8 (dsigma ~ 1e8 gα)
#   denormal   sigma = 24.2: c = (1 - alpha) + 1e-10 ~ 1e-6, so P_j = prod c runs through the
#              fp32 subnormals (P_6 ~ 1e-42) and underflows to 0 (nerf.py:218-232)
#   opaque     sigma = 50: alpha rounds to 1, c = 1e-10 exactly, P_3 = 1e-40 subnormal, then 0
#   saturated  rgb pre-activations +-30 (sigmoid 1 / 9e-14), sigma alternating 0 and 3
#   sigma_tiny sigma = 1e-30 (the row as small): alpha = 0, dsigma = gα 1e8
#   nan        z_r = -100 on sample 3: expf(100) overflows, loma's sigmoid adjoint
#              (x (1 - x) through 1/(1 + e)^2 e, nerf.py:157-165 under rev_diff) is NaN, like
#              the reference (train_nerf.py:486-489 guards for exactly this)
EDGE_FINITE = ("sigma0", "tiny", "denormal", "opaque", "saturated", "sigma_tiny")
EDGE_NAN = ("sigma0", "nan", "saturated")


def edge_ray(kind, rng, S=8):
    x = np.zeros((S, 8), np.float32)
    rgb = rng.uniform(-2, 2, (S, 3)).astype(np.float32)
    x[:, 0:3] = np.maximum(rgb, 0)
    x[:, 4:7] = np.maximum(-rgb, 0)
    sig = {"sigma0": -np.ones(S), "denormal": np.full(S, 24.2), "opaque": np.full(S, 50.0),
           "sigma_tiny": np.full(S, 1e-30), "nan": rng.uniform(0.5, 2, S),
           "saturated": np.where(np.arange(S) % 2 == 0, 0.0, 3.0),
           "tiny": (np.arange(S) + 1) * 1e-9}[kind]
    x[:, 3] = np.maximum(sig, 0)
    x[:, 7] = np.maximum(-sig, 0)
    if kind in ("tiny", "sigma_tiny"):   # the whole row as small as sigma (its own exponent group)
        x[:, [0, 1, 2, 4, 5, 6]] *= 1e-9 if kind == "tiny" else 1e-30
    if kind == "saturated":
        x[:, 0:3] = np.where(rng.uniform(size=(S, 3)) < 0.5, 30.0, 0.0)
        x[:, 4:7] = np.where(x[:, 0:3] > 0, 0.0, 30.0)
    if kind == "nan":
        x[3, 0], x[3, 4] = 0.0, 100.0
    return x


def edge_fixture(kinds, S=8):
    import oracle
    rng = np.random.RandomState(11)
    X = np.concatenate([edge_ray(k, rng, S) for k in kinds]).astype(np.float32)
    N = len(kinds)
    I = np.eye(8, dtype=np.float32)
    W2 = np.zeros((8, 4), np.float32)
    for c in range(4):
        W2[c, c], W2[c + 4, c] = 1.0, -1.0
    ws = [I, I.copy(), W2]
    bs = [np.zeros(8, np.float32), np.zeros(8, np.float32), np.zeros(4, np.float32)]
    wp, bp = nerf_np.pad_weights(ws, bs)
    t = np.linspace(2.0, 6.0, S)
    dists = np.repeat(np.concatenate([t[1:] - t[:-1], [1e8]])[None, :], N, 0).astype(np.float32)
    target = rng.uniform(0, 1, (N, 3)).astype(np.float32)
    shapes = [w.shape for w in ws]
    c = oracle.standard_forward_backward(X, wp, bp, shapes, dists, target, S, seed=1.0, dX=True)
    f = nerf_np.nerf_forward_backward(X, ws, bs, dists, target, S, seed=1.0)
    L = len(ws)
    dW64 = np.zeros(wp.shape)
    dB64 = np.zeros(bp.shape)
    for l in range(L):
        k, n = ws[l].shape
        dW64[l, :k, :n] = f["dW"][l]
        dB64[l, :n] = f["db"][l]
    return dict(kinds=np.array(kinds), X=X, dists=dists, target=target, wp=wp, bp=bp,
                shapes=np.array(shapes, np.int32), S=np.int32(S),
                loss=np.float64(c["loss"]), acc=c["acc"], dW=c["dW"], dB=c["dB"], dX=c["dX"],
                d_dists=c["d_dists"], d_target=c["d_target"],
                f64_loss=np.float64(f["loss"]), f64_acc=f["acc"], f64_dW=dW64, f64_dB=dB64,
                f64_d_dists=f["d_dists"], f64_d_target=f["d_target"], f64_dX=f["dX"])


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
    # 5. edge numerics (scripts/nerf.py:157-165,200-232, train_nerf.py:306-311)
    for name, rays in (("edge_finite_6x8.npz", EDGE_FINITE), ("edge_nan_3x8.npz", EDGE_NAN)):
        np.savez_compressed(os.path.join(HERE, name), **edge_fixture(rays))
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
