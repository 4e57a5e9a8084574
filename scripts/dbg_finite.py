# Debug helper: one cfg3 fused training step (256 rays), per-layer finiteness and size of dW / db.
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "loma-nerf_amd")):
    sys.path.insert(0, p)
import torch
import lnerf
import nerf_np
eng = lnerf.Engine()
w = nerf_np.make_workload("cfg3", rays=256)
shapes = [x.shape for x in w.ws]
mlp = lnerf.make_mlp(shapes, w.wp.shape[1], w.wp.shape[2])
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0")
r = eng.train_step(mlp, t(w.wp), t(w.bp), t(w.pts32.reshape(-1, 3)), t(w.dists), t(w.target), samples=w.S,
                   num_freqs=w.F, seed=1.0, flags=lnerf.FAST)
torch.cuda.synchronize()
dW = r.d_ws.cpu().numpy(); dB = r.d_bs.cpu().numpy()
ref = nerf_np.nerf_forward_backward(w.X, w.ws, w.bs, w.dists, w.target, w.S)
print("lib", lnerf.LIB_PATH, "loss", float(r.loss.item()), "ref", ref["loss"], eng.last_path())
for l, (k, n) in enumerate(shapes):
    g = dW[l, :k, :n]; want = ref["dW"][l]
    print(l, (k, n), "finite", bool(np.isfinite(g).all()), "nonfinite", int((~np.isfinite(g)).sum()),
          "max|err|/max", float(np.nanmax(np.abs(g - want)) / np.abs(want).max()), "db finite", bool(np.isfinite(dB[l, :n]).all()))
for l in (1, 7):
    k, n = shapes[l]
    g = dW[l, :k, :n]
    bad = ~np.isfinite(g)
    print("layer", l, "nonfinite rows per 32-row tile", [int(bad[i:i + 32].any(axis=1).sum()) for i in range(0, k, 32)],
          "cols per 32-col tile", [int(bad[:, j:j + 32].any(axis=0).sum()) for j in range(0, n, 32)])
    fin = np.isfinite(g)
    want = ref["dW"][l]
    print("  finite elems max rel err", float(np.abs(np.where(fin, g - want, 0)).max() / np.abs(want).max()))
