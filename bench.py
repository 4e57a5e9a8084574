#!/usr/bin/env python3
"""Headline benchmark: ray-samples/s of one fwd+bwd training step (BASELINE.json `metric`).

Workload (BASELINE.json configs[2]): synthetic Lego-style 400x400 camera,
4096 rays x 64 samples per GPU, positional encoding F=5 (33 inputs), MLP 33->256x7->4, fp32,
random-init weights (mlp_utils.py:166-204, seed 215). A step = sampling the rays (linspace depths,
points, dists; train_nerf.py:289-306) + positional encoding + MLP forward + compositing +
sum-of-squares loss + the reverse pass over every MLP weight (the work of one
nerf_evaluate_and_march + grad_nerf_evaluate_and_march pair on the batch) + the reference's Adam
update of every weight and bias on the device (train_nerf.py:133-161; --no-optimizer drops it), on
rays already resident in HBM (--input points: host-sampled points instead). With N > 1 GPUs (one process per GPU, torchrun) every rank runs its own 4096-ray
batch (weak scaling) and the packed [dW, db, loss] buffer is all-reduced (SUM) over RCCL, then
scaled by the global loss (the reference seeds its gradient with the loss, train_nerf.py:477).

Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "loma-nerf_amd"))

METRIC = "ray-samples/sec fwd+bwd, 4096 rays×64 samples, 1/2/4/8 MI355X"
# bf16 MFMA dense: 256 CU x 4 SIMD x 1024 FLOP/clk (v_mfma_f32_32x32x16_bf16: 32768 FLOP / 32 clk)
# x 2.4 GHz = 2516.6 TF; the bf16x6 split spends 6 bf16 MFMA products per fp32 multiply-add
PEAK_BF16_TFLOPS = 2516.6
PEAK_X6_TFLOPS = PEAK_BF16_TFLOPS / 6
PEAK_F16X3_TFLOPS = PEAK_BF16_TFLOPS / 3   # fp16 MFMA runs at the bf16 rate
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rays", type=int, default=None, help="rays per GPU (default: config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rays", type=int, default=128, help="rays in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--generic", action="store_true", help="time the loma-order kernels instead")
    ap.add_argument("--input", choices=("rays", "points"), default="rays",
                    help="rays: (rays, 6) origins+directions, the engine samples points, dists and "
                         "the encoding on the GPU (LNERF_INPUT_RAYS); points: host-sampled positions")
    ap.add_argument("--render", action="store_true",
                    help="config 5 instead: forward-only eval render of an 800x800 frame at 128 "
                         "samples/ray (bf16 MFMA unless --x6), rays sharded over ranks")
    ap.add_argument("--x6", action="store_true",
                    help="render with the fp32-class default split (fp16x3) instead of plain bf16")
    ap.add_argument("--x6-train", action="store_true",
                    help="fused path with the bf16x6 split instead of the default fp16x3 split")
    ap.add_argument("--k16-w4", action="store_true",
                    help="A/B: k16 on 4-wave 64-sample workgroups, two per CU (lnerf.K16_W4)")
    ap.add_argument("--strong", action="store_true",
                    help="config 4 strong scaling: one batch of the config's rays (4096) sharded "
                         "over the ranks (contiguous ray ranges, 512 per GPU at N=8) instead of a "
                         "full batch per GPU")
    ap.add_argument("--no-optimizer", action="store_true",
                    help="fwd+bwd only: skip the on-device Adam update (train_nerf.py:133-161) "
                         "that every timed step otherwise applies after the gradient exchange")
    ap.add_argument("--lr", type=float, default=5e-4, help="Adam learning rate (train_nerf.py)")
    ap.add_argument("--no-render", action="store_true",
                    help="skip the config-5 render record the default N=1 line carries")
    return ap.parse_args()


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/<round>_pmc.json, written by scripts/summarize_profile.py from separate FETCH_SIZE /
    WRITE_SIZE passes of this same command, gfx950-corrected), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "r*_pmc.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    if d.get("workload") != config:
        return None
    for name, v in d["kernels"].items():
        if name.startswith(kernel):
            return {"bytes": v["hbm_bytes_per_launch"], "read": v["hbm_read_bytes"],
                    "write": v["hbm_write_bytes"], "source": os.path.relpath(files[-1], HERE)}
    return None


def sq_counters(kernel):
    """MFMA-busy and LDS figures for `kernel` from the newest committed SQ counter summary
    (profiles/<round>_sq.json, scripts/gpu_sq.sh + scripts/summarize_sq.py: separate rocprofv3
    --pmc passes of this bench), or None. mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8
    x 1024 SIMDs), rocprof's MfmaUtil."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "r*_sq.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    for name, v in d["kernels"].items():
        if name.startswith(kernel):
            der = v["derived"]
            return {"mfma_busy": der.get("mfma_busy"), "lds_busy": der.get("lds_busy"),
                    "lds_bank_conflict": der.get("lds_conflict"), "clock_ghz": der.get("clock_ghz"),
                    "source": os.path.relpath(files[-1], HERE)}
    return None


def cpu_baseline(args, cfg):
    """The C oracle (loma-order scalar fp32 restatement, -O2, no FMA) timed on this host on a
    bounded sample of the same workload. Test infrastructure, used only as the reported baseline."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import numpy as np
    import oracle
    import scene
    b = scene.make_batch(cfg, rays=args.cpu_rays)
    shapes, wp, bp = scene.init_mlp(3 + 6 * b["F"], 4, b["L"], b["H"])
    res = {}
    for threads, rays in ((1, args.cpu_rays), (args.cpu_threads, args.cpu_rays * args.cpu_threads)):
        bb = scene.make_batch(cfg, rays=rays)
        Xb = oracle.positional_encoding_3d(bb["pts"].astype(np.float64), bb["F"])
        oracle.train_step(Xb[: 2 * bb["S"]], wp, bp, shapes, bb["dists"][:2], bb["target"][:2],
                          bb["S"], threads=1)  # warm the library
        t0 = time.perf_counter()
        oracle.train_step(Xb, wp, bp, shapes, bb["dists"], bb["target"], bb["S"], threads=threads)
        dt = time.perf_counter() - t0
        res[threads] = (rays * bb["S"] / dt, rays, dt)
    v1, r1, t1 = res[1]
    vn, rn, tn = res[args.cpu_threads]
    return ({"value": v1, "unit": "ray-samples/s", "cores": 1, "kind": "port",
             "sample": f"{r1} rays x {b['S']} samples of {cfg}, one fwd+grad step, scalar "
                       f"loma-order C oracle (-O2, no FMA), {t1:.1f}s"},
            {"value": vn, "unit": "ray-samples/s", "cores": args.cpu_threads, "kind": "port",
             "sample": f"{rn} rays x {b['S']} samples, OpenMP over rays, {tn:.1f}s"})


def bench_render(args, world, rank, local, dist, steps=None, warmup=None):
    """Config 5: 800x800 frame, 128 samples/ray, MLP 33->256x7->4, forward only.
    The frame's 640 000 rays come from the device get_rays; each rank renders a contiguous share
    (replicas, no collective in the timed region). Returns rank 0's JSON record (None elsewhere)."""
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    import numpy as np
    import torch
    import dp
    import lnerf
    import scene
    side, _, S, F, L, H = scene.CONFIGS["cfg5"]
    dev = f"cuda:{local}"
    eng = lnerf.Engine(local)
    shapes, wp, bp = scene.init_mlp(3 + 6 * F, 4, L, H)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    ws = torch.from_numpy(wp).to(dev)
    bs = torch.from_numpy(bp).to(dev)
    focal = 0.5 / np.tan(0.5 * scene.CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5], [0, focal, 0.5], [0, 0, 1]])
    rays_all = eng.get_rays(side, K, scene.look_at_pose())
    lo, hi = dp.shard_rays(rays_all.shape[0], world, rank)
    rays = rays_all[lo:hi].contiguous()
    N = rays.shape[0]
    target = torch.zeros(N, 3, dtype=torch.float32, device=dev)
    acc = torch.empty(N, 3, dtype=torch.float32, device=dev)
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    flags = lnerf.FAST | (0 if args.x6 else lnerf.MFMA_BF16)

    def step():
        eng.render(mlp, ws, bs, rays, None, target, samples=S, input_mode=lnerf.INPUT_RAYS,
                   num_freqs=F, flags=flags, acc=acc, loss=loss)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / steps * 1e3
    total = side * side * S
    fwd_flops = 2 * sum(k * n for k, n in shapes)
    rec = None
    if rank == 0:
        mode = "fp16x3" if args.x6 else "bf16"
        peak = PEAK_F16X3_TFLOPS if args.x6 else PEAK_BF16_TFLOPS
        ach = fwd_flops * N * S / (ms / 1e3) / 1e12
        rec = {
            "metric": "ray-samples/sec fwd (eval render), 800x800 frame x 128 samples",
            "value": total / (ms / 1e3), "unit": "ray-samples/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": mode, "data": "synthetic (device get_rays of a look-at camera, random-init "
                                   "MLP seed 215)",
            "config": {"workload": "cfg5: 800x800 rays x 128 samples per frame, PE F=5, "
                                   "MLP 33->256x7->4, forward only",
                       "rays_per_gpu": N, "parallelism": f"replicas{world}"},
            "roofline": {"bound": "mfma",
                         "kernel": "k16_fwd_bwd_kernel (forward only)",
                         "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
                         "traffic": None,
                         "note": "rank-0 per-GPU rate: 2*sum(KN) FLOP/sample x its samples / "
                                 "step time (includes get_rays-free sampling + PE + compositing)"},
        }
    eng.close()
    return rec


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import dp
    import lnerf
    import scene

    torch.cuda.set_device(local)
    dist = None
    # under torchrun (WORLD_SIZE set) the RCCL data-parallel step runs even at world size 1, so the
    # N>1 code path can be rehearsed on a single GPU
    if world > 1 or "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    if args.render:
        rec = bench_render(args, world, rank, local, dist)
        if rec:
            print(json.dumps(rec), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    dev = f"cuda:{local}"
    if args.strong:
        # config 4: ONE batch (the same rays on every rank), rank r takes its
        # contiguous share (dp.shard_rays); the all-reduce SUM restores the whole batch's gradient
        b = scene.shard_batch(scene.make_batch(args.config, rays=args.rays, rank=0),
                              *dp.shard_rays(args.rays or scene.CONFIGS[args.config][1], world, rank))
    else:
        b = scene.make_batch(args.config, rays=args.rays, rank=rank)
    shapes, wp, bp = scene.init_mlp(3 + 6 * b["F"], 4, b["L"], b["H"])
    N, S = b["N"], b["S"]
    eng = lnerf.Engine(local)
    mlp = lnerf.make_mlp(shapes, wp.shape[1], wp.shape[2])
    # weights and biases packed like the gradient buffer [dW | db], so that one Adam launch
    # updates both (padding entries have zero gradients and never move)
    params = torch.cat([torch.from_numpy(wp).reshape(-1), torch.from_numpy(bp).reshape(-1)]).to(dev)
    ws = params[:wp.size].view(wp.shape)
    bs = params[wp.size:].view(bp.shape)
    adam_m = torch.zeros_like(params)
    adam_v = torch.zeros_like(params)
    adam_t = [0]
    if args.input == "rays":
        x = torch.from_numpy(b["rays"]).to(dev)
        dists = None
        mode = lnerf.INPUT_RAYS
    else:
        x = torch.from_numpy(b["pts"]).to(dev)
        dists = torch.from_numpy(b["dists"]).to(dev)
        mode = lnerf.INPUT_POINTS
    target = torch.from_numpy(b["target"]).to(dev)
    grads = eng.alloc_grads(len(shapes), wp.shape[1], wp.shape[2])
    gbuf = grads[0]
    acc = torch.empty(N, 3, device=dev)
    flags = lnerf.GENERIC if args.generic else lnerf.FAST
    if args.x6_train:
        flags |= lnerf.MFMA_BF16X6
    if args.k16_w4:
        flags |= lnerf.K16_W4

    def step(timing=False):
        f = flags | (lnerf.TIMING if timing else 0)
        if dist is None:
            eng.train_step(mlp, ws, bs, x, dists, target, samples=S, num_freqs=b["F"], input_mode=mode,
                           seed=None, flags=f, grads=grads, acc_color=acc)
        else:
            eng.train_step(mlp, ws, bs, x, dists, target, samples=S, num_freqs=b["F"], input_mode=mode,
                           seed=1.0, flags=f, grads=grads, acc_color=acc)
            # [dW, db, loss] SUM over ranks (RCCL), then the loss seed (loma-nerf_amd/dp.py)
            dp.allreduce_loss_seeded(gbuf, dist, eng.scale_by_device_scalar)
        if not args.no_optimizer:
            # the reference's Adam step on the device (replicated on every rank after the
            # all-reduce, so weights stay identical)
            adam_t[0] += 1
            eng.adam_update(params, gbuf[:-1], adam_m, adam_v, adam_t[0], args.lr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_host = time.perf_counter() - t0   # host enqueue time of the K steps (no sync inside)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    total_rays = b["N_total"] if args.strong else world * N
    value = total_rays * S / (ms / 1e3)

    # per-kernel HIP-event times over extra timed steps (same stream, same kernels)
    kt = {}
    if not args.generic:
        reps = max(3, min(args.steps, 10))
        acc_t = {}
        for _ in range(reps):
            step(timing=True)
            for k, v in eng.timings().items():
                acc_t[k] = acc_t.get(k, 0.0) + v
        kt = {k: v / reps for k, v in acc_t.items()}
    fused_flops = scene.fused_kernel_flops(shapes) * N * S
    dw_flops = scene.dw_kernel_flops(shapes) * N * S
    step_flops = scene.step_flops(shapes) * N * S

    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "ray-samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None, "dtype": "f32",
            "mfma": ("generic (no MFMA)" if args.generic else
                     "bf16x6 (fp32 operands split hi+mid+lo, fp32 accumulate)" if args.x6_train else
                     "fp16x3 (fp32 operands x 2^e split hi+lo in fp16, 3 products, fp32 accumulate)"),
            "data": "synthetic (look-at camera rays, uniform targets, random-init MLP seed 215)",
            "config": {"workload": (f"cfg4 (strong): one {total_rays}-ray x {S}-sample batch sharded "
                                    f"over {world} GPU(s), {N} rays on rank 0" if args.strong else
                                    f"{args.config}: {N} rays x {S} samples per GPU")
                                   + f", PE F={b['F']}, MLP {shapes[0][0]}->{b['H']}x{b['L'] - 1}->4, fp32",
                       "rays_per_gpu": N, "samples": S, "layers": b["L"], "width": b["H"],
                       "parallelism": f"dp{world}", "path": "generic" if args.generic else "fused",
                       "optimizer": (None if args.no_optimizer else
                                     f"adam lr {args.lr} on device (train_nerf.py:133-161), in the step"),
                       "input": ("rays: sampling, dists and positional encoding on the GPU"
                                 if args.input == "rays" else "points: sampled on the host")},
            "step_tflops": step_flops / (ms / 1e3) / 1e12,
            "host_enqueue_ms_per_step": t_host / args.steps * 1e3,
        }
        if kt:
            fus_ms = kt["fused"]
            peak = PEAK_X6_TFLOPS if args.x6_train else PEAK_F16X3_TFLOPS
            assert eng.last_path()["k16"], eng.last_path()
            k1 = "k16_fwd_bwd_kernel"
            out["roofline"] = {"bound": "mfma", "kernel": k1,
                               "achieved": fused_flops / (fus_ms / 1e3) / 1e12,
                               "peak": peak, "unit": "TFLOP/s",
                               "frac": fused_flops / (fus_ms / 1e3) / 1e12 / peak,
                               "traffic": None,
                               "flops_per_launch": fused_flops, "avg_ms": fus_ms,
                               "peak_basis": ("bf16 MFMA dense 2516.6 TF / 6 (bf16x6: six bf16 "
                                              "products per fp32-accurate multiply-add)" if args.x6_train
                                              else "fp16 MFMA dense 2516.6 TF / 3 (fp16x3: three fp16 "
                                              "products per multiply-add)")}
            full = args.rays is None and not args.strong
            tr = pmc_traffic(k1, args.config) if full else None
            if tr:
                out["roofline"]["traffic"] = tr["bytes"]
                out["roofline"]["traffic_unit"] = "bytes/launch"
                out["roofline"]["traffic_source"] = tr["source"]
                out["roofline"]["traffic_gbs"] = tr["bytes"] / (fus_ms / 1e3) / 1e9
            sq = sq_counters(k1) if full and not args.x6_train else None
            if sq:
                out["roofline"]["mfma_busy"] = sq["mfma_busy"]
                out["roofline"]["counters"] = sq
            out["kernels_ms"] = kt
            out["dw_kernel_tflops"] = dw_flops / (kt["dw"] / 1e3) / 1e12
            out["dw_kernel_frac"] = out["dw_kernel_tflops"] / peak
            # k2 streams the slabs k1 wrote: algorithmic bytes = every slab value read once
            # (X, A_l for l < L-1, G_l for every l; 32-feature tiles, fp32)
            slab_b = 4 * 32 * (-(-shapes[0][0] // 32) + sum(-(-n // 32) for _, n in shapes[:-1])
                               + sum(-(-n // 32) for _, n in shapes))
            out["dw_kernel_hbm"] = {"bytes_per_sample": slab_b, "bytes_per_launch": slab_b * N * S,
                                    "achieved_gbs": slab_b * N * S / (kt["dw"] / 1e3) / 1e9,
                                    "peak_gbs": PEAK_HBM_GBS,
                                    "frac": slab_b * N * S / (kt["dw"] / 1e3) / 1e9 / PEAK_HBM_GBS}
        if world == 1 and not (args.no_render or args.generic or args.strong or args.rays):
            # config 5 (forward-only 800x800x128 bf16 eval render) on the same GPU, timed the same
            # way (its own warmup, barrier + synchronize brackets), so that it has a driver record
            eng.close()
            r5 = bench_render(argparse.Namespace(x6=False), 1, 0, local, None,
                              steps=5, warmup=2)
            out["config5_render"] = {k: r5[k] for k in ("metric", "value", "unit", "ms_per_step", "steps",
                                                         "warmup", "dtype", "config", "roofline")}
        if world == 1 and not args.no_cpu_baseline:
            c1, cn = cpu_baseline(args, args.config)
            out["cpu_baseline"] = c1
            out["cpu_baseline_mt"] = cn
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
