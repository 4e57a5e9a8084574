"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference NeRF hot path (the checker).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product path (loma-nerf_amd/) never does.

Parity status: "parity unpinned" against the reference binary (no golden vectors exist for this
path and running the loma compiler was denied). This float64 restatement is
independent of the C restatement in nerf_oracle.c; tests cross-check the two, torch autograd and
finite differences.

Contents (each function cites the reference code it restates):
  * get_rays                  train_nerf.py:23-62
  * positional_encoding_3d    pos_encoding.py:38-69
  * get_sample_mlp / pad      mlp_utils.py:166-204, :272-313
  * sample_rays               train_nerf.py:289-311 (linspace depths, dists with trailing 1e8)
  * nerf_forward_backward     scripts/nerf.py:1-304 + its reverse-mode gradient (:306), float64,
                              "standard semantics" (zero-initialised buffers, io rows = real rows)
  * make_workload             the synthetic configs of SURVEY.md §8d
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# --------------------------------------------------------------------------------------------
# host-side producers (train_nerf.py / pos_encoding.py / mlp_utils.py restatements)
# --------------------------------------------------------------------------------------------


def get_rays(height: int, width: int, normalized_K: np.ndarray, c2w: np.ndarray):
    """train_nerf.py:23-62. Pixel grid linspace(0,1,W) (note: `height` is unused there too),
    directions [(i-cx)/fx, -(j-cy)/fy, -1] (not normalised), rotated by c2w[:3,:3]."""
    rng = np.linspace(0, 1, width)
    i, j = np.meshgrid(rng, rng, indexing="xy")
    i, j = i.flatten(), j.flatten()
    dirs = np.stack([(i - normalized_K[0, 2]) / normalized_K[0, 0],
                     -(j - normalized_K[1, 2]) / normalized_K[1, 1],
                     -np.ones_like(i)], axis=-1)
    R = c2w[:3, :3]
    T = c2w[:3, 3]
    return T[None, :].repeat(dirs.shape[0], 0), dirs @ R.T


def positional_encoding_3d(x: np.ndarray, num_functions: int = 5) -> np.ndarray:
    """pos_encoding.py:38-69: block-major [x, sin(2^0 x), cos(2^0 x), ...], f64 -> f32."""
    parts = [x]
    for f in range(num_functions):
        parts.append(np.sin((2.0 ** f) * x))
        parts.append(np.cos((2.0 ** f) * x))
    comb = np.transpose(np.array(parts), (1, 2, 0, 3))
    return comb.reshape(comb.shape[0], comb.shape[1], -1).astype(np.float32)


def get_sample_mlp(in_channels: int, out_channels: int, num_layers: int, filter_size: int):
    """mlp_utils.py:166-204: W ~ N(0, sqrt(2/in)) (in, out) f32, then b ~ N(0, 0.5) f32, per layer,
    drawn from numpy's global RandomState in that order."""
    ws, bs = [], []
    cin = in_channels
    for i in range(num_layers):
        cout = out_channels if i == num_layers - 1 else filter_size
        ws.append(np.random.normal(size=(cin, cout), loc=0, scale=(2 / cin) ** 0.5).astype(np.float32))
        bs.append(np.random.normal(size=cout, loc=0, scale=0.5).astype(np.float32))
        cin = cout
    return ws, bs


def pad_weights(ws, bs):
    """mlp_utils.py:272-313 for the (L, Kmax, Nmax) / (L, Nmax) padded layout."""
    L = len(ws)
    kmax = max(w.shape[0] for w in ws)
    nmax = max(max(w.shape[1] for w in ws), max(b.shape[0] for b in bs))
    wp = np.zeros((L, kmax, nmax), np.float32)
    bp = np.zeros((L, nmax), np.float32)
    for l, (w, b) in enumerate(zip(ws, bs)):
        wp[l, : w.shape[0], : w.shape[1]] = w
        bp[l, : b.shape[0]] = b
    return wp, bp


def look_at_pose(radius: float = 4.0, azimuth_deg: float = 45.0, elevation_deg: float = 30.0):
    """A Blender-synthetic style camera-to-world pose: camera at `radius` looking at the origin,
    +z of the camera frame pointing away from the target (the camera looks down -z, as the
    directions of train_nerf.py:41-48 assume)."""
    az, el = math.radians(azimuth_deg), math.radians(elevation_deg)
    eye = radius * np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
    z = eye / np.linalg.norm(eye)
    up = np.array([0.0, 0.0, 1.0])
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = x, y, z, eye
    return c2w


def sample_rays(rays_o: np.ndarray, rays_d: np.ndarray, num_samples: int, near=2.0, far=6.0):
    """train_nerf.py:289-311: t = linspace(near, far, S) (no jitter), points o + d t (f64),
    dists = [diff(t), 1e8] repeated per ray."""
    t = np.linspace(near, far, num_samples)
    pts = rays_o[:, None, :] + rays_d[:, None, :] * t[None, :, None]
    dists = np.concatenate((t[1:] - t[:-1], np.ones_like(t[:1]) * 1e8))[None, :].repeat(rays_o.shape[0], 0)
    return pts, dists


# --------------------------------------------------------------------------------------------
# synthetic workloads (seeds: rays 0, targets 1, weights 215)
# --------------------------------------------------------------------------------------------

CONFIGS = {
    # name: (image side, rays, samples, F, layers, filter)
    "cfg2": (100, 1024, 32, 5, 3, 30),   # train_nerf.py-sized MLP 33->30->30->4
    "cfg3": (400, 4096, 64, 5, 8, 256),  # 33->256x7->4, the headline bench workload
    "chunk": (64, 4, 30, 5, 3, 30),      # the train_nerf.py chunk: 4 rays x 30 samples
}


@dataclass
class Workload:
    pts: np.ndarray        # (N, S, 3) float64 sample positions
    pts32: np.ndarray      # (N, S, 3) float32 (what the device POINTS mode consumes)
    X: np.ndarray          # (N*S, C_in) float32 = PE(pts) from float64 (the loma layer_input)
    dists: np.ndarray      # (N, S) float32 (c_float at the ABI)
    target: np.ndarray     # (N, 3) float32
    ws: list               # per-layer (K, N) float32
    bs: list               # per-layer (N,) float32
    wp: np.ndarray         # padded (L, Kmax, Nmax)
    bp: np.ndarray         # padded (L, Nmax)
    F: int
    S: int
    N: int


def make_workload(name: str = "cfg2", rays: int | None = None, samples: int | None = None,
                  layers: int | None = None, filter_size: int | None = None,
                  num_functions: int | None = None) -> Workload:
    side, N, S, F, L, H = CONFIGS[name]
    N = rays or N
    S = samples or S
    L = layers or L
    H = filter_size or H
    F = F if num_functions is None else num_functions
    focal = 0.5 / np.tan(0.5 * 0.6911112)  # dataloader.py:55 with lego's camera_angle_x
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]]).astype(np.float32)  # :265-267
    o, d = get_rays(side, side, K, look_at_pose())
    sel = np.random.RandomState(0).choice(o.shape[0], size=N, replace=N > o.shape[0])
    pts, dists = sample_rays(o[sel], d[sel], S)
    X = positional_encoding_3d(pts, F).reshape(-1, 3 + 6 * F)
    target = np.random.RandomState(1).uniform(0, 1, size=(N, 3)).astype(np.float32)
    state = np.random.get_state()
    np.random.seed(215)
    ws, bs = get_sample_mlp(3 + 6 * F, 4, L, H)
    np.random.set_state(state)
    wp, bp = pad_weights(ws, bs)
    pts32 = pts.astype(np.float32)
    return Workload(pts, pts32, X, dists.astype(np.float32), target, ws, bs, wp, bp, F, S, N)


def relu_tie_rays(w: Workload, thresh: float = 5e-7) -> np.ndarray:
    """Rays holding a hidden pre-activation z with |z| < thresh * sum|terms| (float64 forward).

    Such a ReLU decision sits below fp32 resolution (thresh ~ 8 ulp): any fp32 summation order
    may decide it either way, and a flipped decision moves that sample's whole gradient row, far
    past the 1e-4 parity tolerance ("ReLU-mask flips ... reported separately")."""
    A = positional_encoding_3d(w.pts32.astype(np.float64), w.F).reshape(w.N * w.S, -1) \
        if w.X.shape[1] == 3 + 6 * w.F else w.X.astype(np.float64)
    bad = np.zeros(w.N * w.S, bool)
    for l in range(len(w.ws) - 1):
        W = w.ws[l].astype(np.float64)
        b = w.bs[l].astype(np.float64)
        Z = A @ W + b
        T = np.abs(A) @ np.abs(W) + np.abs(b)
        bad |= (np.abs(Z) < thresh * T).any(axis=1)
        A = np.maximum(Z, 0.0)
    return np.unique(np.nonzero(bad)[0] // w.S)


def subset_rays(w: Workload, rays) -> Workload:
    rays = np.asarray(rays, np.int64)
    rows = (rays[:, None] * w.S + np.arange(w.S)[None, :]).ravel()
    return Workload(w.pts[rays], w.pts32[rays], w.X[rows], w.dists[rays], w.target[rays], w.ws, w.bs,
                    w.wp, w.bp, w.F, w.S, len(rays))


def without_relu_ties(w: Workload, thresh: float = 5e-7) -> Workload:
    """The workload minus its relu_tie_rays (parity tests against an fp32 oracle)."""
    ties = set(relu_tie_rays(w, thresh).tolist())
    return subset_rays(w, [r for r in range(w.N) if r not in ties])


# --------------------------------------------------------------------------------------------
# float64 forward + hand-derived backward (standard semantics)
# --------------------------------------------------------------------------------------------


def nerf_forward_backward(X, ws, bs, dists, target, S, seed=1.0, masks=None):
    """scripts/nerf.py:1-304 forward and the exact derivative its rev_diff computes (SURVEY §8a
    "Backward the build implements"), in float64. Returns a dict with loss, acc_color (N,3),
    dW/db per layer, dX, d_dists, d_target, and the per-sample rgba.

    seed=None seeds the reverse pass with the loss itself (train_nerf.py:477). masks (optional):
    per hidden layer l a bool (R, n_l) array of ReLU decisions to use instead of z > 0 in both
    passes (nerf.py:141-144) -- the derivative at another implementation's decisions, for
    comparing with it on rays whose pre-activations sit at |z| ~ 0 (ReLU ties). Also returns the
    hidden pre-activations Z[l] and their term magnitudes T[l] = |A||W| + |b|, and the operands of
    every weight adjoint: A[l] (layer l's input, X for l = 0) and G[l] = dL/dZ_l, dW[l] = A^T G."""
    X = np.asarray(X, np.float64)
    L = len(ws)
    A = [X]
    Z = []
    Tm = []
    for l in range(L):
        W64 = np.asarray(ws[l], np.float64)
        b64 = np.asarray(bs[l], np.float64)
        z = A[-1] @ W64 + b64[None, :]
        Z.append(z)
        if l < L - 1:
            Tm.append(np.abs(A[-1]) @ np.abs(W64) + np.abs(b64)[None, :])
            m = (z > 0) if masks is None else np.asarray(masks[l], bool)
            A.append(np.where(m, z, 0.0))
    zl = Z[-1]
    sig = 1.0 / (1.0 + np.exp(-zl[:, :3]))
    sigma = np.where(zl[:, 3] > 0, zl[:, 3], 0.0)
    N = X.shape[0] // S
    rgb = sig.reshape(N, S, 3)
    sg = sigma.reshape(N, S)
    dl = np.asarray(dists, np.float64).reshape(N, S)
    e = np.exp(-sg * dl)
    alpha = 1.0 - e
    c = (1.0 - alpha) + 1e-10
    P = np.cumprod(c, axis=1)
    T = P.copy()
    T[:, 0] = 1.0            # inclusive product with T_0 = 1 (nerf.py:226-272)
    w = alpha * T
    C = (w[:, :, None] * rgb).sum(1)
    t = np.asarray(target, np.float64)
    loss = ((C - t) ** 2).sum()
    if seed is None:
        seed = loss

    gC = 2.0 * seed * (C - t)
    gw = (gC[:, None, :] * rgb).sum(2)
    grgb = w[:, :, None] * gC[:, None, :]
    dP = alpha * gw
    dP[:, 0] = 0.0
    dc = np.zeros_like(c)
    for j in range(S - 1, 0, -1):
        dP[:, j - 1] += dP[:, j] * c[:, j]
        dc[:, j] += dP[:, j] * P[:, j - 1]
    dc[:, 0] += dP[:, 0]
    galpha = T * gw - dc
    gsigma = galpha * e * dl
    gdist = galpha * e * sg
    dz = np.zeros_like(zl)
    s3 = sig.reshape(-1, 3)
    dz[:, :3] = grgb.reshape(-1, 3) * s3 * (1.0 - s3)
    dz[:, 3] = np.where(zl[:, 3] > 0, gsigma.reshape(-1), 0.0)
    dW = [None] * L
    db = [None] * L
    G = [None] * L
    g = dz
    dX = None
    for l in range(L - 1, -1, -1):
        G[l] = g
        dW[l] = A[l].T @ g
        db[l] = g.sum(0)
        ga = g @ np.asarray(ws[l], np.float64).T
        if l > 0:
            m = (Z[l - 1] > 0) if masks is None else np.asarray(masks[l - 1], bool)
            g = np.where(m, ga, 0.0)
        else:
            dX = ga
    return dict(loss=loss, acc=C, dW=dW, db=db, dX=dX, d_dists=gdist, d_target=-gC,
                rgb=rgb, sigma=sg, weights=w, alpha=alpha, Z=Z[:-1], T=Tm, A=A, G=G)


def nerf_forward_backward_chunked(X, ws, bs, dists, target, S, seed, masks=None, rays_per_chunk=256):
    """nerf_forward_backward over ray chunks (bounded memory at the full bench size), summing the
    batch quantities. `seed` must be a number here (the gradient is linear in it); returns loss,
    acc, dW, db, d_dists, d_target and, per hidden layer, the decisions that differ from z > 0
    with their margins |z| / T (flip_margins)."""
    X = np.asarray(X)
    N = X.shape[0] // S
    L = len(ws)
    out = dict(loss=0.0, acc=[], dW=[0.0] * L, db=[0.0] * L, d_dists=[], d_target=[],
               flip_margins=[[] for _ in range(L - 1)])
    for lo in range(0, N, rays_per_chunk):
        hi = min(N, lo + rays_per_chunk)
        rows = slice(lo * S, hi * S)
        ms = None if masks is None else [np.asarray(m[rows], bool) for m in masks]
        r = nerf_forward_backward(X[rows], ws, bs, dists[lo:hi], target[lo:hi], S, seed=seed, masks=ms)
        out["loss"] += r["loss"]
        out["acc"].append(r["acc"])
        out["d_dists"].append(r["d_dists"])
        out["d_target"].append(r["d_target"])
        for l in range(L):
            out["dW"][l] = out["dW"][l] + r["dW"][l]
            out["db"][l] = out["db"][l] + r["db"][l]
        if ms is not None:
            for l in range(L - 1):
                flip = (r["Z"][l] > 0) != ms[l]
                out["flip_margins"][l].append(np.abs(r["Z"][l][flip]) / np.maximum(r["T"][l][flip], 1e-300))
    for k in ("acc", "d_dists", "d_target"):
        out[k] = np.concatenate(out[k])
    out["flip_margins"] = [np.concatenate(f) if f else np.zeros(0) for f in out["flip_margins"]]
    return out
