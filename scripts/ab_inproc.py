"""In-process interleaved A/B of engine library builds (GPU box): every library is loaded into ONE
process (ctypes, RTLD_LOCAL) with its own context and its own copy of the cfg3 training state, and
the libraries take turns in short blocks of steps, so clock, power and thermal state are shared
(bench.py runs per library on one box spread ±2-3 % between identical builds).

  python scripts/ab_inproc.py lib/libloma_nerf.so lib/libloma_nerf_X.so [--rounds 12 --block 8]

Prints per library the median and mean of k1 (`fused`), k2 (`dw`) and the whole step by HIP
events, over every timed step of every round."""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "loma-nerf_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--block", type=int, default=8)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--render", action="store_true", help="the config-5 frame (kr) instead of cfg3 training")
    ap.add_argument("--lr", type=float, default=None,
                    help="Adam learning rate (0: the weights never move, so timing-knob builds with wrong "
                         "gradients keep running on the same sane weights as the product)")
    a = ap.parse_args()
    import torch
    import bench
    import lnerf

    class LibEngine(lnerf.Engine):
        def __init__(self, path, device=0):
            self.torch = torch
            self.lib = lnerf.load_library(path)
            self.device = device
            h = ctypes.c_void_p()
            if self.lib.lnerf_ctx_create(ctypes.byref(h), device) != 0:
                raise RuntimeError("lnerf_ctx_create failed for " + path)
            self.ctx = h

    saved = sys.argv
    sys.argv = [saved[0]]   # bench.py's defaults (RAYS input, Adam in the step)
    args = bench.parse()
    sys.argv = saved
    if a.lr is not None:
        args.lr = a.lr
    if a.render:
        return render_ab(a, LibEngine)
    trainers = []
    for p in a.libs:
        t = bench.Trainer(args, a.config, 0, 0, 1, None)
        t.eng.close()
        t.eng = LibEngine(os.path.abspath(p))
        t.grads = t.eng.alloc_grads(len(t.shapes), t.ws.shape[1], t.ws.shape[2])
        for _ in range(3):
            t.step()
        trainers.append(t)
    torch.cuda.synchronize()
    res = {p: {"fused": [], "dw": [], "total": [], "step_ms": []} for p in a.libs}
    for r in range(a.rounds):
        order = list(range(len(a.libs)))
        if r % 2:
            order.reverse()
        for i in order:
            t, p = trainers[i], a.libs[i]
            t.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.block):
                t.step()
            torch.cuda.synchronize()
            res[p]["step_ms"].append((time.perf_counter() - t0) * 1e3 / a.block)
            for _ in range(2):
                t.step(timing=True)
                k = t.eng.timings()
                for key in ("fused", "dw", "total"):
                    if key in k:
                        res[p][key].append(k[key])
        print(f"round {r + 1}/{a.rounds}", flush=True)
    out = {}
    for p in a.libs:
        out[os.path.basename(p)] = {k: {"median": round(statistics.median(v), 4), "mean": round(statistics.fmean(v), 4),
                                        "n": len(v)} for k, v in res[p].items() if v}
    print(json.dumps(out, indent=1))
    for t in trainers:
        t.close()


def render_ab(a, LibEngine):
    """The config-5 frame (bench.py bench_render's inputs) per library, alternating one frame each:
    the render kernel's HIP-event time and the frame's wall time."""
    import numpy as np
    import torch
    import lnerf
    import scene
    side, _, S, F, L, H = scene.CONFIGS["cfg5"]
    shapes, wp, bp = scene.init_mlp(3 + 6 * F, 4, L, H)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    ws = torch.from_numpy(wp).to("cuda:0")
    bs = torch.from_numpy(bp).to("cuda:0")
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    engs = [LibEngine(os.path.abspath(p)) for p in a.libs]
    rays = engs[0].get_rays(side, K, scene.look_at_pose())
    N = rays.shape[0]
    target = torch.zeros(N, 3, dtype=torch.float32, device="cuda:0")
    acc = torch.empty(N, 3, dtype=torch.float32, device="cuda:0")
    loss = torch.empty(1, dtype=torch.float32, device="cuda:0")
    res = {p: {"fused": [], "frame_ms": []} for p in a.libs}

    def frame(e, timing):
        e.render(mlp, ws, bs, rays, None, target, samples=S, input_mode=lnerf.INPUT_RAYS, num_freqs=F,
                 flags=lnerf.FAST | lnerf.MFMA_BF16 | (lnerf.TIMING if timing else 0), acc=acc, loss=loss)

    for e in engs:
        frame(e, False)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        order = list(range(len(a.libs)))
        if r % 2:
            order.reverse()
        for i in order:
            e, p = engs[i], a.libs[i]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            frame(e, True)
            torch.cuda.synchronize()
            res[p]["frame_ms"].append((time.perf_counter() - t0) * 1e3)
            res[p]["fused"].append(e.timings()["fused"])
        print(f"round {r + 1}/{a.rounds}", flush=True)
    out = {os.path.basename(p): {k: {"median": round(statistics.median(v), 4), "mean": round(statistics.fmean(v), 4),
                                     "n": len(v)} for k, v in res[p].items()} for p in a.libs}
    print(json.dumps(out, indent=1))
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
