"""Host-side producers of the reference's training step (rays, samples, MLP init) and the
synthetic workloads the bench runs (seeds: rays 0, targets 1, weights 215).

Restates, for the product/bench path (the oracle keeps its own independent copy):
  get_rays           train_nerf.py:23-62
  sample points      train_nerf.py:289-311 (linspace t, no jitter, dists with trailing 1e8)
  get_sample_mlp     mlp_utils.py:166-204, pad_array :272-313
The data/lego dataset is absent in this environment, so the camera is a Blender-style look-at
pose at radius 4 with lego's camera_angle_x (dataloader.py:55).
"""
from __future__ import annotations

import math

import numpy as np

CONFIGS = {
    # name: (image side, rays, samples, F, layers, filter)
    "cfg2": (100, 1024, 32, 5, 3, 30),
    "cfg3": (400, 4096, 64, 5, 8, 256),
    "cfg5": (800, 640000, 128, 5, 8, 256),
}
CAMERA_ANGLE_X = 0.6911112


def look_at_pose(radius=4.0, azimuth_deg=45.0, elevation_deg=30.0):
    az, el = math.radians(azimuth_deg), math.radians(elevation_deg)
    eye = radius * np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
    z = eye / np.linalg.norm(eye)
    x = np.cross(np.array([0.0, 0.0, 1.0]), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    c2w = np.eye(4)
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2], c2w[:3, 3] = x, y, z, eye
    return c2w


def get_rays(width, K, c2w):
    t = np.linspace(0, 1, width)
    i, j = np.meshgrid(t, t, indexing="xy")
    i, j = i.ravel(), j.ravel()
    d = np.stack([(i - K[0, 2]) / K[0, 0], -(j - K[1, 2]) / K[1, 1], -np.ones_like(i)], -1)
    return np.repeat(c2w[None, :3, 3], d.shape[0], 0), d @ c2w[:3, :3].T


def init_mlp(in_channels, out_channels, num_layers, filter_size, seed=215):
    rs = np.random.RandomState(seed)
    ws, bs = [], []
    cin = in_channels
    for l in range(num_layers):
        cout = out_channels if l == num_layers - 1 else filter_size
        ws.append(rs.normal(size=(cin, cout), loc=0, scale=(2 / cin) ** 0.5).astype(np.float32))
        bs.append(rs.normal(size=cout, loc=0, scale=0.5).astype(np.float32))
        cin = cout
    L = num_layers
    kmax = max(w.shape[0] for w in ws)
    nmax = max(w.shape[1] for w in ws)
    wp = np.zeros((L, kmax, nmax), np.float32)
    bp = np.zeros((L, nmax), np.float32)
    for l, (w, b) in enumerate(zip(ws, bs)):
        wp[l, : w.shape[0], : w.shape[1]] = w
        bp[l, : b.shape[0]] = b
    return [w.shape for w in ws], wp, bp


def make_batch(name="cfg3", rays=None, samples=None, rank=0):
    """Synthetic batch: pts (N*S, 3) float32, dists (N, S) float32, target (N, 3) float32.
    `rank` offsets the ray selection seed so data-parallel ranks get different rays."""
    side, N, S, F, L, H = CONFIGS[name]
    N = rays or N
    S = samples or S
    focal = 0.5 / np.tan(0.5 * CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]]).astype(np.float32)
    o, d = get_rays(side, K, look_at_pose())
    sel = np.random.RandomState(rank).choice(o.shape[0], size=N, replace=N > o.shape[0])
    t = np.linspace(2.0, 6.0, S)
    pts = o[sel][:, None, :] + d[sel][:, None, :] * t[None, :, None]
    dists = np.concatenate((t[1:] - t[:-1], [1e8]))[None, :].repeat(N, 0)
    target = np.random.RandomState(1 + 1000 * rank).uniform(0, 1, size=(N, 3)).astype(np.float32)
    rays = np.concatenate([o[sel], d[sel]], 1).astype(np.float32)   # LNERF_INPUT_RAYS rows
    return dict(pts=pts.reshape(-1, 3).astype(np.float32), dists=dists.astype(np.float32),
                rays=rays, target=target, F=F, S=S, N=N, L=L, H=H)


def shard_batch(b, lo, hi):
    """Rays [lo, hi) of a make_batch() batch (config 4 strong scaling: one batch split over the
    ranks by dp.shard_rays). N_total keeps the whole batch's ray count."""
    S = b["S"]
    out = dict(b)
    out.update(pts=b["pts"][lo * S:hi * S], dists=b["dists"][lo:hi], rays=b["rays"][lo:hi],
               target=b["target"][lo:hi], N=hi - lo, N_total=b["N"])
    return out


def compute_psnr(img1, img2, max_val=1.0):
    """train_nerf.py:163-183: 20 log10(max / sqrt(mean((img1 - img2)^2))), numpy or torch."""
    mse = ((img1 - img2) ** 2).mean()
    return 20.0 * math.log10(max_val / math.sqrt(float(mse)))


def render_image(engine, mlp, ws, bs, width, K, c2w, samples, num_freqs, near=2.0, far=6.0,
                 flags=0, target=None, rays=None):
    """The eval render of train_nerf.py:558-712 on the device: get_rays for the full width x width
    frame, sampling + encoding + MLP + compositing per ray (LNERF_INPUT_RAYS), one call.
    Returns (width*width, 3) colours (device tensor)."""
    import lnerf
    if rays is None:
        rays = engine.get_rays(width, K, c2w)
    if target is None:
        target = engine.torch.zeros(rays.shape[0], 3, dtype=engine.torch.float32, device=rays.device)
    _, acc = engine.render(mlp, ws, bs, rays, None, target, samples=samples,
                           input_mode=lnerf.INPUT_RAYS, num_freqs=num_freqs, near=near, far=far,
                           flags=flags)
    return acc


def step_flops(shapes):
    """Canonical algorithmic FLOPs per sample: fwd 2KN every layer, bwd dW 2KN
    every layer, bwd dX 2KN for l >= 1."""
    s = sum(k * n for k, n in shapes)
    return 6 * s - 2 * shapes[0][0] * shapes[0][1]


def fused_kernel_flops(shapes):
    """Algorithmic FLOPs per sample of the fused forward + reverse-chain kernel (k1)."""
    s = sum(k * n for k, n in shapes)
    return 4 * s - 2 * shapes[0][0] * shapes[0][1]


def dw_kernel_flops(shapes):
    return 2 * sum(k * n for k, n in shapes)
