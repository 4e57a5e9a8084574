#!/usr/bin/env python3
"""Headline benchmark: ray-samples/s of one fwd+bwd training step (BASELINE.json `metric`).

Workload (BASELINE.json configs[2]): synthetic Lego-style 400x400 camera,
4096 rays x 64 samples per GPU, positional encoding F=5 (33 inputs), MLP 33->256x7->4, fp32,
random-init weights (mlp_utils.py:166-204, seed 215). A step = sampling the rays (linspace depths,
points, dists; train_nerf.py:289-306) + positional encoding + MLP forward + compositing +
sum-of-squares loss + the reverse pass over every MLP weight (the work of one
nerf_evaluate_and_march + grad_nerf_evaluate_and_march pair on the batch) + the reference's Adam
update of every weight and bias on the device (train_nerf.py:133-161; --no-optimizer drops it), on
rays already resident in HBM (--input points: host-sampled points instead). With N > 1 GPUs (one
process per GPU, torchrun) every rank runs its own 4096-ray batch (weak scaling) and the packed
[dW, db, loss] buffer is all-reduced (SUM) over RCCL, then scaled by the global loss (the reference
seeds its gradient with the loss, train_nerf.py:477).

The default N=1 line also carries, each timed with its own warmup and barrier/synchronize brackets
after the headline timing:
  * config2         configs[1]: 1024 rays x 32 samples, MLP 33->30->30->4 (train_nerf.py:189-203)
  * config5_render  configs[4]: the 800x800 x 128-sample forward-only eval render (bf16 MFMA)
  * cpu_baseline    the loma-order C restatement on one host core, and cpu_baseline_mt on every
                    core this process may run on (host model and counts recorded)
Counter-derived fields (HBM traffic, MFMA busy) come from the committed rocprofv3 summaries under
profiles/ and are quoted only when their recorded library hash equals the loaded library's.

Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
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
# the k16 instantiations the bench runs (template <hidden tiles, planes, waves>)
K1_TRAIN = "k16_fwd_bwd_kernel<16, 2, 8>"
K1_RENDER = "k16_fwd_bwd_kernel<16, 1, 8>"       # the render on k16's forward (--render-k16)
K1_RENDER_KR = "kr_fwd_kernel<16>"                 # the render kernel (lnerf_render.hip)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--rays", type=int, default=None, help="rays per GPU (default: config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target wall time of each CPU-baseline leg (bounded sample)")
    ap.add_argument("--generic", action="store_true", help="time the loma-order kernels instead")
    ap.add_argument("--input", choices=("rays", "points"), default="rays",
                    help="rays: (rays, 6) origins+directions, the engine samples points, dists and "
                         "the encoding on the GPU (LNERF_INPUT_RAYS); points: host-sampled positions")
    ap.add_argument("--render", action="store_true",
                    help="config 5 instead: forward-only eval render of an 800x800 frame at 128 "
                         "samples/ray (bf16 MFMA unless --x6), rays sharded over ranks, the frame "
                         "gathered on every rank inside the timed region")
    ap.add_argument("--x6", action="store_true",
                    help="render with the fp32-class default split (fp16x3) instead of plain bf16")
    ap.add_argument("--render-k16", action="store_true",
                    help="A/B: render (plain bf16) on k16's forward instead of kr (lnerf.RENDER_K16)")
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
    ap.add_argument("--zero-weights", action="store_true",
                    help="diagnostic only (not a benchmark): all weights and biases zero, to measure how "
                         "much of the step is the chip's power-limited clock (MI355X_MICROARCH.md DVFS)")
    ap.add_argument("--dw-grid", type=int, default=0,
                    help="dW kernel workgroups per step (lnerf_ctx_set_option OPT_DW_GRID; 0 = default 512)")
    ap.add_argument("--no-render", action="store_true",
                    help="skip the config-5 render record the default N=1 line carries")
    ap.add_argument("--no-cfg2", action="store_true",
                    help="skip the config-2 record the default N=1 line carries")
    return ap.parse_args()


# ---- counters from the committed rocprofv3 summaries, bound to the library they profiled --------

def lib_sha16(path=None):
    """First 16 hex digits of the SHA-256 of the engine library (the one lnerf loads)."""
    import lnerf
    path = path or lnerf.LIB_PATH
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def _summaries(kind, workload, sha):
    """Newest profiles/r*_{kind}.json for `workload` whose lib_sha16 is `sha`: (dict, relpath), or
    (None, why)."""
    files = sorted(glob.glob(os.path.join(HERE, "profiles", f"r*_{kind}.json")))
    stale = []
    for f in reversed(files):
        d = json.load(open(f))
        if d.get("workload") != workload:
            continue
        if d.get("lib_sha16") != sha:
            stale.append(os.path.relpath(f, HERE))
            continue
        return d, os.path.relpath(f, HERE)
    return None, ("no summary profiled this library (" + ", ".join(stale[:3]) + " profiled others)"
                  if stale else "no summary for this workload")


def _kernel_entry(d, kernel):
    k = d["kernels"].get(kernel)
    if k is None:   # older summaries key by the template-free name
        k = next((v for n, v in d["kernels"].items() if n.startswith(kernel.split("<")[0])), None)
    return k


def pmc_traffic(kernel, workload, sha):
    """HBM bytes per launch of `kernel` from separate FETCH_SIZE / WRITE_SIZE passes of this same
    command (scripts/summarize_profile.py, gfx950-corrected), or (None, why)."""
    d, src = _summaries("pmc", workload, sha)
    if d is None:
        return None, src
    v = _kernel_entry(d, kernel)
    if v is None:
        return None, f"{kernel} not in {src}"
    return {"bytes": v["hbm_bytes_per_launch"], "read": v["hbm_read_bytes"], "write": v["hbm_write_bytes"],
            "source": src}, None


def sq_counters(kernel, workload, sha):
    """MFMA-busy and LDS figures of `kernel` from SQ/GRBM --pmc passes of this bench
    (scripts/gpu_sq.sh + summarize_sq.py), or (None, why). mfma_busy =
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs), rocprof's MfmaUtil."""
    d, src = _summaries("sq", workload, sha)
    if d is None:
        return None, src
    v = _kernel_entry(d, kernel)
    if v is None:
        return None, f"{kernel} not in {src}"
    der = v["derived"]
    return {"mfma_busy": der.get("mfma_busy"), "lds_busy": der.get("lds_busy"),
            "lds_bank_conflict": der.get("lds_conflict"), "clock_ghz": der.get("clock_ghz"),
            "source": src}, None


def attach_counters(roof, kernel, workload, sha, with_sq=True, work=None):
    """Counter fields of the committed, hash-matched summaries. `work` (FLOP or bytes per launch,
    the unit of roof["peak"]): also frac_rocprof = work / the rocprofv3 kernel-trace average of the
    same library (profiles/*_pmc.json avg_ms, from *_kernel_stats.csv) / peak, and, with SQ
    counters, frac_at_clock = the HIP-event frac scaled by 2.4 GHz / the SQ-derived clock the
    kernel ran at under the profiler (the fraction of what the chip's clock allowed)."""
    tr, why = pmc_traffic(kernel, workload, sha)
    if tr:
        roof["traffic"] = tr["bytes"]
        roof["traffic_unit"] = "bytes/launch"
        roof["traffic_source"] = tr["source"]
        roof["traffic_gbs"] = tr["bytes"] / (roof["avg_ms"] / 1e3) / 1e9
        d, _ = _summaries("pmc", workload, sha)
        ent = _kernel_entry(d, kernel) if d else None
        if work is not None and ent and ent.get("avg_ms"):
            scale = 1e12 if roof.get("unit") == "TFLOP/s" else 1e9
            roof["avg_ms_rocprof"] = ent["avg_ms"]
            roof["frac_rocprof"] = work / (ent["avg_ms"] / 1e3) / scale / roof["peak"]
    else:
        roof["traffic_note"] = why
    if with_sq:
        sq, why = sq_counters(kernel, workload, sha)
        if sq:
            roof["mfma_busy"] = sq["mfma_busy"]
            roof["counters"] = sq
            base = roof.get("kernel_frac", roof.get("frac"))
            if sq.get("clock_ghz") and base is not None:
                roof["clock_ghz_profiled"] = sq["clock_ghz"]
                roof["frac_at_clock"] = base * 2.4 / sq["clock_ghz"]
        else:
            roof["counters_note"] = why


# ---- CPU baseline ------------------------------------------------------------------------------

def host_info():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    # a CPU quota (cgroup v2 cpu.max "quota period", or v1 cfs files) caps the CPUs this process
    # can actually keep busy below its affinity mask (the GPU box grants one GPU's share)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.5)))
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_cpu_quota": quota, "usable_cpus": usable,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(args, cfg):
    """The C oracle (loma-order scalar fp32 restatement of scripts/nerf.py's generated C, -O2, no
    FMA) timed on this host on a bounded sample of the same workload: one core, then OpenMP over
    rays on every CPU this process may run on (sched_getaffinity). Each sample is sized from a
    short calibration run so that the leg takes about --cpu-seconds. The thread count is the CPUs
    the process can keep busy: its affinity mask capped by its cgroup CPU quota (on the GPU box
    the mask names all 256 CPUs but the quota grants one GPU's share). Test infrastructure, used
    only as the reported baseline, after the GPU timing."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import numpy as np
    import oracle
    import scene
    info = host_info()
    _, _, S, F, L, H = scene.CONFIGS[cfg]
    shapes, wp, bp = scene.init_mlp(3 + 6 * F, 4, L, H)

    def run(rays, threads):
        bb = scene.make_batch(cfg, rays=rays)
        Xb = oracle.positional_encoding_3d(bb["pts"].astype(np.float64), bb["F"])
        t0 = time.perf_counter()
        oracle.train_step(Xb, wp, bp, shapes, bb["dists"], bb["target"], bb["S"], threads=threads)
        dt = time.perf_counter() - t0
        return rays * bb["S"] / dt, dt

    run(2, 1)   # warm the library
    res = {}
    # multi-core candidates: the usable CPUs, and the box's OMP_NUM_THREADS share when it differs
    # (a quota the process cannot read shows up as poor scaling past it); the faster one is kept
    cands = [info["usable_cpus"]]
    try:
        omp = int(info["omp_num_threads_env"] or 0)
        if 1 < omp < cands[0]:
            cands.append(omp)
    except ValueError:
        pass
    for threads in [1] + cands:
        probe = max(threads, 8)
        rate, _ = run(probe, threads)                       # calibration
        secs = args.cpu_seconds if threads == 1 else args.cpu_seconds / len(cands)
        rays = max(probe, int(rate * secs / S))
        rate, dt = run(rays, threads)
        res[threads] = (rate, rays, dt)
    v1, r1, t1 = res[1]
    best = max(cands, key=lambda t: res[t][0])
    vn, rn, tn = res[best]
    info = dict(info, mt_rates={str(t): res[t][0] for t in cands})
    one = {"value": v1, "unit": "ray-samples/s", "cores": 1, "kind": "port",
           "sample": f"{r1} rays x {S} samples of {cfg}, one fwd+grad step, scalar loma-order C "
                     f"oracle (-O2, no FMA), {t1:.1f}s", "host": info}
    mt = {"value": vn, "unit": "ray-samples/s", "cores": best, "kind": "port",
          "sample": f"{rn} rays x {S} samples, OpenMP over rays on {best} threads (the faster of the "
                    f"CPUs this process can keep busy -- affinity capped by cgroup quota -- and "
                    f"OMP_NUM_THREADS), {tn:.1f}s", "host": info}
    return one, mt


# ---- timing helpers ----------------------------------------------------------------------------

def timed(step, steps, warmup, dist=None, dev=None):
    """W untimed steps, then K steps bracketed by barrier + synchronize; MAX over ranks. Returns
    (seconds, host enqueue seconds)."""
    import torch
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, t_host


class Trainer:
    """One configuration's training step on one rank: the engine's fused (or generic) fwd+bwd,
    the RCCL exchange when distributed, and the on-device Adam update."""

    def __init__(self, args, config, local, rank, world, dist, rays=None, strong=False):
        import torch
        import dp
        import lnerf
        import scene
        self.dist, self.args, self.world = dist, args, world
        dev = self.dev = f"cuda:{local}"
        if strong:
            # config 4: ONE batch (the same rays on every rank), rank r takes its
            # contiguous share (dp.shard_rays); the all-reduce SUM restores the whole batch's gradient
            b = scene.shard_batch(scene.make_batch(config, rays=rays, rank=0),
                                  *dp.shard_rays(rays or scene.CONFIGS[config][1], world, rank))
        else:
            b = scene.make_batch(config, rays=rays, rank=rank)
        self.b = b
        self.shapes, wp, bp = scene.init_mlp(3 + 6 * b["F"], 4, b["L"], b["H"])
        self.N, self.S = b["N"], b["S"]
        self.eng = lnerf.Engine(local)
        if getattr(args, "dw_grid", 0):
            self.eng.set_option(lnerf.OPT_DW_GRID, args.dw_grid)
        self.mlp = lnerf.make_mlp(self.shapes, wp.shape[1], wp.shape[2])
        # weights and biases packed like the gradient buffer [dW | db], so that one Adam launch
        # updates both (padding entries have zero gradients and never move)
        self.params = torch.cat([torch.from_numpy(wp).reshape(-1), torch.from_numpy(bp).reshape(-1)]).to(dev)
        if getattr(args, "zero_weights", False):
            self.params.zero_()
        self.ws = self.params[:wp.size].view(wp.shape)
        self.bs = self.params[wp.size:].view(bp.shape)
        self.adam_m = torch.zeros_like(self.params)
        self.adam_v = torch.zeros_like(self.params)
        self.adam_t = 0
        if args.input == "rays":
            self.x, self.dists, self.mode = torch.from_numpy(b["rays"]).to(dev), None, lnerf.INPUT_RAYS
        else:
            self.x = torch.from_numpy(b["pts"]).to(dev)
            self.dists = torch.from_numpy(b["dists"]).to(dev)
            self.mode = lnerf.INPUT_POINTS
        self.target = torch.from_numpy(b["target"]).to(dev)
        self.grads = self.eng.alloc_grads(len(self.shapes), wp.shape[1], wp.shape[2])
        self.acc = torch.empty(self.N, 3, device=dev)
        flags = lnerf.GENERIC if args.generic else lnerf.FAST
        if args.x6_train:
            flags |= lnerf.MFMA_BF16X6
        if args.k16_w4:
            flags |= lnerf.K16_W4
        self.flags = flags

    def step(self, timing=False):
        import dp
        import lnerf
        f = self.flags | (lnerf.TIMING if timing else 0)
        seed = None if self.dist is None else 1.0
        self.eng.train_step(self.mlp, self.ws, self.bs, self.x, self.dists, self.target, samples=self.S,
                            num_freqs=self.b["F"], input_mode=self.mode, seed=seed, flags=f,
                            grads=self.grads, acc_color=self.acc)
        if self.dist is not None:
            # [dW, db, loss] SUM over ranks (RCCL), then the loss seed (loma-nerf_amd/dp.py)
            dp.allreduce_loss_seeded(self.grads[0], self.dist, self.eng.scale_by_device_scalar)
        if not self.args.no_optimizer:
            # the reference's Adam step on the device (replicated on every rank after the
            # all-reduce, so weights stay identical)
            self.adam_t += 1
            self.eng.adam_update(self.params, self.grads[0][:-1], self.adam_m, self.adam_v, self.adam_t,
                                 self.args.lr)

    def kernel_times(self, reps):
        """Per-kernel HIP-event times (ms, on the step's stream) averaged over `reps` extra steps."""
        acc = {}
        for _ in range(reps):
            self.step(timing=True)
            for k, v in self.eng.timings().items():
                acc[k] = acc.get(k, 0.0) + v
        return {k: v / reps for k, v in acc.items()}

    def close(self):
        self.eng.close()


def bench_config2(args, local):
    """BASELINE.json configs[1]: train_nerf.py's own shape -- 1024 rays x
    32 samples, MLP 33->30->30->4 (train_nerf.py:189-203) -- the same step (fwd+bwd+Adam, RAYS
    input). 32 768 samples are 256 k16 workgroups, one per CU and a single wave pair per SIMD, and
    the MLP is 30 wide: a latency-bound step (launches and serial phases, not MFMA or HBM)."""
    import scene
    t = Trainer(args, "cfg2", local, 0, 1, None)
    steps, warmup = 50, 10
    dt, t_host = timed(t.step, steps, warmup)
    ms = dt / steps * 1e3
    kt = t.kernel_times(10)
    t.close()
    return {"metric": "ray-samples/sec fwd+bwd, 1024 rays×32 samples (config 2)",
            "value": t.N * t.S / (ms / 1e3), "unit": "ray-samples/s", "ms_per_step": ms, "steps": steps,
            "warmup": warmup, "dtype": "f32",
            "config": {"workload": f"cfg2: {t.N} rays x {t.S} samples, PE F=5, MLP 33->30->30->4, fp32, "
                                   "Adam in the step", "rays_per_gpu": t.N},
            "kernels_ms": kt, "host_enqueue_ms_per_step": t_host / steps * 1e3,
            "note": "latency-bound: 256 workgroups (one per CU), 30-wide layers; the step is its "
                    "launches and serial phases, not MFMA or HBM time",
            "step_tflops": scene.step_flops(t.shapes) * t.N * t.S / (ms / 1e3) / 1e12}


def bench_render(args, world, rank, local, dist, steps=None, warmup=None):
    """Config 5: 800x800 frame, 128 samples/ray, MLP 33->256x7->4, forward only.
    The frame's 640 000 rays come from the device get_rays; each rank renders a contiguous share
    and, at N > 1, the frame's colours are gathered on every rank (dp.gather_rows, the final
    gather of SURVEY §8e; train_nerf.py:659-681 assembles the eval image) inside the timed step.
    Returns rank 0's JSON record (None elsewhere)."""
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
    n_total = rays_all.shape[0]
    lo, hi = dp.shard_rays(n_total, world, rank)
    rays = rays_all[lo:hi].contiguous()
    N = rays.shape[0]
    target = torch.zeros(N, 3, dtype=torch.float32, device=dev)
    acc = torch.empty(N, 3, dtype=torch.float32, device=dev)
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    flags = lnerf.FAST | (0 if args.x6 else lnerf.MFMA_BF16) | (lnerf.RENDER_K16 if getattr(args, "render_k16", False) else 0)
    frame = [None]

    def step(timing=False):
        eng.render(mlp, ws, bs, rays, None, target, samples=S, input_mode=lnerf.INPUT_RAYS,
                   num_freqs=F, flags=flags | (lnerf.TIMING if timing else 0), acc=acc, loss=loss)
        if dist is not None and world > 1:
            frame[0] = dp.gather_rows(acc, n_total, dist)

    dt, _ = timed(step, steps, warmup, dist, dev)
    ms = dt / steps * 1e3
    # the render kernel alone (HIP events on the render's stream)
    kms = []
    for _ in range(3):
        step(timing=True)
        kms.append(eng.timings().get("fused"))
    kern_ms = None if None in kms else sum(kms) / len(kms)
    used_kr = eng.last_path()["kr"]
    total = side * side * S
    fwd_flops = 2 * sum(k * n for k, n in shapes)
    rec = None
    if rank == 0:
        mode = "fp16x3" if args.x6 else "bf16"
        peak = PEAK_F16X3_TFLOPS if args.x6 else PEAK_BF16_TFLOPS
        ach = fwd_flops * N * S / (ms / 1e3) / 1e12
        kernel = K1_TRAIN if args.x6 else K1_RENDER_KR if used_kr else K1_RENDER
        roof = {"bound": "mfma", "kernel": kernel + " (forward only)", "achieved": ach, "peak": peak,
                "unit": "TFLOP/s", "frac": ach / peak, "traffic": None,
                "note": "rank-0 per-GPU rate: 2*sum(KN) FLOP/sample x its samples / step time "
                        "(includes the device sampling + PE + compositing)"}
        if kern_ms:
            roof["avg_ms"] = kern_ms
            roof["kernel_achieved"] = fwd_flops * N * S / (kern_ms / 1e3) / 1e12
            roof["kernel_frac"] = roof["kernel_achieved"] / peak
            if not args.x6 and not getattr(args, "render_k16", False) and world == 1:
                attach_counters(roof, kernel, "cfg5", lib_sha16(), work=fwd_flops * N * S)
        rec = {
            "metric": "ray-samples/sec fwd (eval render), 800x800 frame x 128 samples",
            "value": total / (ms / 1e3), "unit": "ray-samples/s", "n_gpus": world,
            "steps": steps, "warmup": warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": mode, "data": "synthetic (device get_rays of a look-at camera, random-init "
                                   "MLP seed 215)",
            "config": {"workload": "cfg5: 800x800 rays x 128 samples per frame, PE F=5, "
                                   "MLP 33->256x7->4, forward only",
                       "rays_per_gpu": N, "parallelism": f"replicas{world}",
                       "variant": [v for v in ("x6", "render-k16") if getattr(args, v.replace("-", "_"), False)] or None,
                       "gather": ("the whole frame's colours all-gathered on every rank inside the "
                                  "timed step (dp.gather_rows)" if world > 1 else None)},
            "roofline": roof,
        }
    eng.close()
    return rec


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, cmd=None, env=None, grace_s=10.0, poll_s=0.05) -> int:
    """`bench.py --gpus N` outside torchrun: start N rank processes of this same command (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set per child, rendezvous on
    127.0.0.1). Called before anything touches the GPU (this process never initialises HIP; the
    ranks are children, nothing is exec'd). Rank 0 prints the JSON line.

    Fail fast: the children are polled together, and the first one that exits non-zero makes the
    launcher terminate the rest (SIGTERM, then SIGKILL after `grace_s`) and return that status --
    a surviving rank would otherwise sit in an RCCL collective until the process-group timeout,
    longer than the driver's limit. SIGINT / SIGTERM sent to the launcher are
    forwarded to every rank. Returns 0 when every rank exits 0."""
    import signal
    import subprocess
    import time
    cmd = cmd or [sys.executable, os.path.abspath(__file__)]
    base = dict(os.environ if env is None else env)
    base.setdefault("MASTER_ADDR", "127.0.0.1")
    base.setdefault("MASTER_PORT", str(free_port()))
    procs = []

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass
        deadline = time.monotonic() + grace_s
        for p in procs:
            left = deadline - time.monotonic()
            try:
                p.wait(timeout=max(left, 0.01))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def forward(signum, _frame):
        stop_all(signal.SIGTERM)
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, forward) for s in (signal.SIGINT, signal.SIGTERM)}
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
            procs.append(subprocess.Popen(cmd + list(argv), env=e))
        while True:
            rcs = [p.poll() for p in procs]
            bad = next((rc for rc in rcs if rc is not None and rc != 0), None)
            if bad is not None:
                stop_all()
                return bad
            if all(rc == 0 for rc in rcs):
                return 0
            time.sleep(poll_s)
    finally:
        for s, h in old.items():
            signal.signal(s, h)


def variant_flags(args) -> list:
    """Every non-default measurement mode of this run: a bench line that carries any of them is not
    the headline configuration, says so in config.variant / data, and attaches no counters
    (those were profiled on the default configuration)."""
    v = []
    for name in ("zero_weights", "generic", "x6_train", "k16_w4", "no_optimizer", "strong", "render_k16", "x6"):
        if getattr(args, name, False):
            v.append(name.replace("_", "-"))
    if getattr(args, "dw_grid", 0):
        v.append(f"dw-grid={args.dw_grid}")
    if getattr(args, "input", "rays") != "rays":
        v.append(f"input={args.input}")
    if getattr(args, "rays", None):
        v.append(f"rays={args.rays}")
    if getattr(args, "config", "cfg3") != "cfg3":
        v.append(f"config={args.config}")
    if os.environ.get("LNERF_LIB"):
        v.append(f"lib={os.path.basename(os.environ['LNERF_LIB'])}")
    return v


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here (before any HIP call) instead of by torchrun
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report n_gpus={world}")
    import torch
    import scene

    torch.cuda.set_device(local)
    dist = None
    # under torchrun (WORLD_SIZE set) the RCCL data-parallel step runs even at world size 1, so the
    # N>1 code path can be rehearsed on a single GPU
    if world > 1 or "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        import datetime
        # a bounded rendezvous / collective wait: a dead peer ends this rank in minutes, not after the
        # 10-minute default, and launch_ranks then takes the whole launch down with it
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"),
                                timeout=datetime.timedelta(seconds=int(os.environ.get("LNERF_PG_TIMEOUT_S", "180"))))
    if args.render:
        rec = bench_render(args, world, rank, local, dist)
        if rec:
            print(json.dumps(rec), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    t = Trainer(args, args.config, local, rank, world, dist, rays=args.rays, strong=args.strong)
    dt, t_host = timed(t.step, args.steps, args.warmup, dist, t.dev)
    N, S, shapes = t.N, t.S, t.shapes
    ms = dt / args.steps * 1e3
    total_rays = t.b["N_total"] if args.strong else world * N
    value = total_rays * S / (ms / 1e3)
    # per-kernel HIP-event times over extra timed steps (same stream, same kernels)
    kt = {} if args.generic else t.kernel_times(max(3, min(args.steps, 10)))
    fused_flops = scene.fused_kernel_flops(shapes) * N * S
    dw_flops = scene.dw_kernel_flops(shapes) * N * S
    step_flops = scene.step_flops(shapes) * N * S
    last_path = None if args.generic else t.eng.last_path()
    # the last step's exceptional rows (lnerf_ctx_exceptional_rows; after the timed region)
    xrows = None
    if not args.generic and last_path and last_path.get("planes") == 2:
        n_x, n_last = t.eng.exceptional_rows(split=True)
        xrows = {"rows": n_x, "of_them_last_samples": n_last, "of": len(shapes) * N * S,
                 "floor_guard_fired": t.eng.guard_fired(),
                 "note": "rows (summed over layers) that dw16 multiplied on the bf16x6 split instead of "
                         "the fp16x3 one (lnerf_internal.h kXrowD0); floor_guard_fired: 1 if k1 met a hidden "
                         "G element below fp16x3's floor and the step re-ran on bf16x6 (kGuardExp); both "
                         "measured on the last step"}
    t.close()

    variants = variant_flags(args)
    if rank == 0:
        out = {
            "metric": (METRIC if not args.zero_weights else
                       "DIAGNOSTIC (not a benchmark: all-zero weights, DVFS check): " + METRIC),
            "value": value, "unit": "ray-samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None, "dtype": "f32",
            "mfma": ("generic (no MFMA)" if args.generic else
                     "bf16x6 (fp32 operands split hi+mid+lo, fp32 accumulate)" if args.x6_train else
                     "fp16x3 (fp32 operands x 2^e split hi+lo in fp16, 3 products, fp32 accumulate)"),
            "data": ("synthetic (look-at camera rays, uniform targets, random-init MLP seed 215)"
                     if not args.zero_weights else
                     "synthetic rays and targets, ALL-ZERO weights and biases (--zero-weights diagnostic)")
                    + ("" if not variants else f"; non-default run: {', '.join(variants)}"),
            "config": {"workload": (f"cfg4 (strong): one {total_rays}-ray x {S}-sample batch sharded "
                                    f"over {world} GPU(s), {N} rays on rank 0" if args.strong else
                                    f"{args.config}: {N} rays x {S} samples per GPU")
                                   + f", PE F={t.b['F']}, MLP {shapes[0][0]}->{t.b['H']}x{t.b['L'] - 1}->4, fp32",
                       "rays_per_gpu": N, "samples": S, "layers": t.b["L"], "width": t.b["H"],
                       "parallelism": f"dp{world}", "path": "generic" if args.generic else "fused",
                       "optimizer": (None if args.no_optimizer else
                                     f"adam lr {args.lr} on device (train_nerf.py:133-161), in the step"),
                       "input": ("rays: sampling, dists and positional encoding on the GPU"
                                 if args.input == "rays" else "points: sampled on the host"),
                       "variant": variants or None},
            "diagnostic": bool(args.zero_weights),
            "step_tflops": step_flops / (ms / 1e3) / 1e12,
            "host_enqueue_ms_per_step": t_host / args.steps * 1e3,
            "lib_sha16": lib_sha16(),
            "build_knobs": __import__("lnerf").build_knobs(),
        }
        if kt:
            fus_ms = kt["fused"]
            peak = PEAK_X6_TFLOPS if args.x6_train else PEAK_F16X3_TFLOPS
            assert last_path["k16"], last_path
            k1 = "k16_fwd_bwd_kernel<16, 3, 8>" if args.x6_train else K1_TRAIN
            roof = {"bound": "mfma", "kernel": k1,
                    "achieved": fused_flops / (fus_ms / 1e3) / 1e12,
                    "peak": peak, "unit": "TFLOP/s",
                    "frac": fused_flops / (fus_ms / 1e3) / 1e12 / peak,
                    "traffic": None,
                    "flops_per_launch": fused_flops, "avg_ms": fus_ms,
                    "peak_basis": ("bf16 MFMA dense 2516.6 TF / 6 (bf16x6: six bf16 products per "
                                   "fp32-accurate multiply-add)" if args.x6_train
                                   else "fp16 MFMA dense 2516.6 TF / 3 (fp16x3: three fp16 "
                                   "products per multiply-add)")}
            if not variants:
                attach_counters(roof, k1, "cfg3", out["lib_sha16"], work=fused_flops)
            out["roofline"] = roof
            out["kernels_ms"] = kt
            if xrows is not None:
                out["exceptional_rows"] = xrows
            out["dw_kernel_tflops"] = dw_flops / (kt["dw"] / 1e3) / 1e12
            out["dw_kernel_frac"] = out["dw_kernel_tflops"] / peak
            # k2 streams the slabs k1 wrote: algorithmic bytes = every slab value read once
            # (X, A_l for l < L-1: 3 B per value as int24 under fp16x3 training, else 4; G_l for
            # every l: 4 B; 32-feature tiles)
            a_b = 3 if last_path and last_path.get("a24") else 4
            slab_b = 32 * (a_b * (-(-shapes[0][0] // 32) + sum(-(-n // 32) for _, n in shapes[:-1]))
                           + 4 * sum(-(-n // 32) for _, n in shapes))
            out["dw_kernel_hbm"] = {"kernel": "dw16_kernel<2>", "avg_ms": kt["dw"],
                                    "slab_format": ("int24 activations + f32 gradients" if a_b == 3
                                                    else "f32 activations + f32 gradients"),
                                    "note": "issue-bound (split VALU + MFMA per half-block), not HBM-bound: "
                                            "fewer slab bytes moved it less than in proportion (DESIGN.md §3 k2)",
                                    "bytes_per_sample": slab_b, "bytes_per_launch": slab_b * N * S,
                                    "achieved_gbs": slab_b * N * S / (kt["dw"] / 1e3) / 1e9,
                                    "peak_gbs": PEAK_HBM_GBS,
                                    "frac": slab_b * N * S / (kt["dw"] / 1e3) / 1e9 / PEAK_HBM_GBS}
            if not variants:
                out["dw_kernel_hbm"]["unit"] = "GB/s"
                out["dw_kernel_hbm"]["peak"] = PEAK_HBM_GBS
                attach_counters(out["dw_kernel_hbm"], "dw16_kernel<2>", "cfg3", out["lib_sha16"],
                                work=slab_b * N * S)
        extras = world == 1 and not variants
        if extras and not args.no_cfg2:
            out["config2"] = bench_config2(args, local)
        if extras and not args.no_render:
            # config 5 (forward-only 800x800x128 bf16 eval render) on the same GPU, timed the same
            # way (its own warmup, barrier + synchronize brackets), so that it has a driver record
            r5 = bench_render(argparse.Namespace(x6=False, render_k16=False, steps=5, warmup=2), 1, 0, local, None)
            out["config5_render"] = {k: r5[k] for k in ("metric", "value", "unit", "ms_per_step", "steps",
                                                         "warmup", "dtype", "config", "roofline")}
        if world == 1 and not args.no_cpu_baseline:
            c1, cn = cpu_baseline(args, args.config)
            out["cpu_baseline"] = c1
            out["cpu_baseline_mt"] = cn
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
