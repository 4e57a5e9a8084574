#!/usr/bin/env python3
"""Experiment (not product code): does a dw16 pass overlap a k1 pass on the GPU?

Half-batches (2048 rays x 64 samples of cfg3) on two engines. Sequential: every half-step on one
stream. Overlapped: two streams, the second delayed by about one k1 so that one half's k1 runs
while the other half's dW kernel streams its slabs. Prints ms per half-step for both.

    python scripts/exp_overlap.py
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "loma-nerf_amd"))


def main():
    import torch
    import lnerf
    import scene
    dev = "cuda:0"
    b = scene.make_batch("cfg3", rays=2048)
    shapes, wp, bp = scene.init_mlp(3 + 6 * b["F"], 4, b["L"], b["H"])
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    ws = torch.from_numpy(wp).to(dev)
    bs = torch.from_numpy(bp).to(dev)
    x = torch.from_numpy(b["rays"]).to(dev)
    tg = torch.from_numpy(b["target"]).to(dev)
    engs = [lnerf.Engine(0), lnerf.Engine(0)]
    grads = [e.alloc_grads(len(shapes), wp.shape[1], wp.shape[2]) for e in engs]
    accs = [torch.empty(2048, 3, device=dev) for _ in engs]

    def half(i):
        engs[i].train_step(mlp, ws, bs, x, None, tg, samples=b["S"], num_freqs=b["F"],
                           input_mode=lnerf.INPUT_RAYS, seed=None, flags=lnerf.FAST, grads=grads[i],
                           acc_color=accs[i])

    # per-kernel times of one half-step
    engs[0].train_step(mlp, ws, bs, x, None, tg, samples=b["S"], num_freqs=b["F"],
                       input_mode=lnerf.INPUT_RAYS, seed=None, flags=lnerf.FAST | lnerf.TIMING,
                       grads=grads[0], acc_color=accs[0])
    kt = engs[0].timings()
    print("half-step kernels ms", {k: round(v, 4) for k, v in kt.items()}, flush=True)
    n = 40
    for _ in range(5):
        half(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        half(i & 1)
    torch.cuda.synchronize()
    seq = (time.perf_counter() - t0) / n * 1e3
    print(f"sequential: {seq:.4f} ms per half-step", flush=True)

    s = [torch.cuda.Stream(), torch.cuda.Stream()]
    cyc = int(kt["fused"] * 1e-3 * 2.1e9)   # torch.cuda._sleep spins on the shader clock
    for delay_frac in (0.0, 0.5, 1.0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s[1]):
            if delay_frac:
                torch.cuda._sleep(int(cyc * delay_frac))
        for i in range(n // 2):
            for j in (0, 1):
                with torch.cuda.stream(s[j]):
                    half(j)
        torch.cuda.synchronize()
        ov = (time.perf_counter() - t0) / n * 1e3
        print(f"two streams (delay {delay_frac} x k1 nominal): {ov:.4f} ms per half-step", flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
