"""Debug: the bench-size tiny-sigma workload on fused fp16x3 / bf16x6 and the generic (loma-order fp32)
path, dW columns compared among them and with float64 (test infrastructure)."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__)); REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "loma-nerf_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import torch, lnerf, nerf_np
from fused_parity import run_fused, encoded_input, padded
eng = lnerf.Engine(0)
w = nerf_np.make_workload("cfg3", rays=int(sys.argv[1]) if len(sys.argv) > 1 else 2048)
ws = [x.copy() for x in w.ws]; bs = [x.copy() for x in w.bs]
ws[-1][:, 3] *= 1e-8; bs[-1][3] = 0.0
sub = nerf_np.subset_rays(w, range(256))
r0 = nerf_np.nerf_forward_backward(sub.X, ws, bs, sub.dists, sub.target, sub.S, seed=1.0)
bs[-1][3] = np.float32(-np.median(r0["A"][-1] @ ws[-1][:, 3].astype(np.float64)))
wp, bp = nerf_np.pad_weights(ws, bs)
w = nerf_np.Workload(w.pts, w.pts32, w.X, w.dists, w.target, ws, bs, wp, bp, w.F, w.S, w.N)
a = run_fused(eng, w, seed=1.0)
b = run_fused(eng, w, seed=1.0, flags=lnerf.MFMA_BF16X6)
dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")
mlp = lnerf.make_mlp([x.shape for x in ws], wp.shape[1], wp.shape[2])
g = eng.train_step(mlp, dev(wp), dev(bp), dev(w.pts32.reshape(-1, 3)), dev(w.dists), dev(w.target), samples=w.S,
                   input_mode=lnerf.INPUT_POINTS, seed=1.0, flags=lnerf.GENERIC)
torch.cuda.synchronize()
gdW = g.d_ws.cpu().numpy()
X = encoded_input(w, True)
ref = nerf_np.nerf_forward_backward_chunked(X, ws, bs, w.dists, w.target, w.S, seed=1.0, masks=a["masks"])
ref0 = nerf_np.nerf_forward_backward_chunked(X, ws, bs, w.dists, w.target, w.S, seed=1.0)
dW = padded(ref["dW"], wp.shape); dW0 = padded(ref0["dW"], wp.shape)
for l, (k, n) in enumerate(x.shape for x in ws):
    cm = np.abs(dW[l, :k, :n]).max(0)
    def rel(x, y):
        return float((np.abs(x[l, :k, :n] - y[l, :k, :n]).max(0) / np.maximum(cm, 1e-300)).max())
    print(f"layer {l}: fp16x3-f64@mask {rel(a['dW'], dW):.3g}  bf16x6-f64@mask {rel(b['dW'], dW):.3g}  "
          f"generic-f64 {rel(gdW, dW0):.3g}  fp16x3-generic {rel(a['dW'], gdW):.3g}  fp16x3-bf16x6 {rel(a['dW'], b['dW']):.3g}"
          f"  f64@mask-f64 {rel(dW, dW0):.3g}")
print("loss", a["loss"], b["loss"], float(g.loss.item()), ref["loss"])
