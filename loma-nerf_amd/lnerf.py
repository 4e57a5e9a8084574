"""Python binding of libloma_nerf.so (include/lnerf.h) -- the host side of the MI355X engine.

Two surfaces:
  * `load_library()` returns the ctypes CDLL with argtypes for every exported symbol (the
    loma-compat ones are what `compiler.compile` hands to train_nerf.py / fit_img.py).
  * `Engine` drives the native batched API on torch device tensors (torch is used only for
    device memory and streams). There is no CPU fallback: without the library or a GPU the
    calls raise.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

HERE = os.path.dirname(os.path.abspath(__file__))
# LNERF_LIB: an alternative in-tree build (e.g. the LNERF_PROF phase-counter variant)
LIB_PATH = os.environ.get("LNERF_LIB") or os.path.join(HERE, "lib", "libloma_nerf.so")
MAX_LAYERS = 16

INPUT_ENCODED = 0
INPUT_POINTS = 1
INPUT_RAYS = 2
SEED_CONST = 0
SEED_LOSS = 1
ACCUMULATE = 2
WANT_DX = 4
GENERIC = 8
FAST = 16
TIMING = 32
MFMA_F32 = 64     # removed in round 4 (one-wave exact-f32 kernel): an error; exact fp32 is GENERIC
MFMA_BF16 = 128   # fused path: plain bf16 operands (reduced precision; inference)
MFMA_F16X3 = 256  # fused path: fp16x3 split (22-bit products, fp32 accumulate; the k16 default)
MFMA_BF16X6 = 512  # fused path: bf16x6 split (fp32-accurate products)
ONE_WAVE = 1024    # removed in round 4 (the one-wave-per-SIMD kernel pair): an error
K32 = 2048         # removed in round 4 (k32 lost to k16): an error
K16_W4 = 4096      # fused path: k16 on 4-wave 64-sample workgroups, two per CU (A/B)
HEAD_FIT = 8192    # the mlp_fit head (sigmoid on every output, no compositing; samples = 1)
RENDER_K16 = 16384  # render (plain bf16) on k16's forward instead of kr (A/B)

OPT_DW_GRID = 1    # lnerf_ctx_set_option: dW workgroups per step (0 = default 512)

# every symbol include/lnerf.h declares (tests check the library exports all of them)
EXPORTED_SYMBOLS = [
    "nerf_evaluate_and_march", "grad_nerf_evaluate_and_march", "mlp_fit", "grad_mlp_fit",
    "mult_a_b", "lnerf_last_error", "lnerf_version", "lnerf_ctx_create", "lnerf_ctx_destroy",
    "lnerf_workspace_bytes", "lnerf_train_step", "lnerf_render", "lnerf_scale_by_device_scalar",
    "lnerf_adam_update", "lnerf_ctx_timings", "lnerf_get_rays", "lnerf_ctx_last_path",
    "lnerf_ctx_set_option", "lnerf_ctx_relu_masks", "lnerf_build_knobs", "lnerf_ctx_exceptional_rows",
    "lnerf_ctx_guard_fired",
]

# lnerf_ctx_last_path bits
PATH_GENERIC = 1
PATH_FUSED = 2
PATH_K16 = 4
PATH_DW16 = 8
PATH_K32 = 16      # reserved (k32, removed in round 4)
PATH_K16_W4 = 32
PATH_KR = 64       # the render ran kr (lnerf_render.hip)
PATH_A24 = 128      # training kept the activation slabs as int24 (fp16x3)


class LnerfMLP(ctypes.Structure):
    _fields_ = [("num_layers", ctypes.c_int), ("k", ctypes.c_int * MAX_LAYERS),
                ("n", ctypes.c_int * MAX_LAYERS), ("w_k", ctypes.c_int), ("w_n", ctypes.c_int)]


class LnerfBatch(ctypes.Structure):
    _fields_ = [("rays", ctypes.c_int), ("samples", ctypes.c_int), ("input_mode", ctypes.c_int),
                ("num_freqs", ctypes.c_int), ("x", ctypes.c_void_p), ("dists", ctypes.c_void_p),
                ("target", ctypes.c_void_p), ("near_t", ctypes.c_float), ("far_t", ctypes.c_float)]


class LnerfOutputs(ctypes.Structure):
    _fields_ = [("loss", ctypes.c_void_p), ("acc_color", ctypes.c_void_p),
                ("d_ws", ctypes.c_void_p), ("d_bs", ctypes.c_void_p), ("d_x", ctypes.c_void_p),
                ("d_dists", ctypes.c_void_p), ("d_target", ctypes.c_void_p)]


_LIB = None

_F = ctypes.POINTER(ctypes.c_float)
_FF = ctypes.POINTER(_F)
_FFF = ctypes.POINTER(_FF)
_I = ctypes.POINTER(ctypes.c_int)
_II = ctypes.POINTER(_I)

# loma argtypes (compiler.py:25-51 mapping of the scripts/*.py signatures)
NERF_ARGTYPES = [_FF, ctypes.c_int, ctypes.c_int, _FFF, _FF, _FF, ctypes.c_int, ctypes.c_int,
                 ctypes.c_int, _II, _II, _II, _FFF, _FFF, ctypes.c_int, _FF, _FF, _FF, _FF, _FF]
MLP_FIT_ARGTYPES = [_FF, ctypes.c_int, ctypes.c_int, _FF, _FFF, _FF, _FF, ctypes.c_int,
                    ctypes.c_int, ctypes.c_int, _II, _II, _II, _FFF]
MULT_A_B_ARGTYPES = [_FF, ctypes.c_int, ctypes.c_int, _FF, ctypes.c_int, ctypes.c_int, _FF]


def rev_argtypes(fwd, ret_is_float=True):
    """reverse_diff.py:504-517: every In arg x is followed by an Out adjoint of x's type (arrays
    keep their pointer type, scalars become pointers); the float return adds a `_dreturn`."""
    out = []
    for t in fwd:
        out.append(t)
        out.append(t if issubclass(t, ctypes._Pointer) else ctypes.POINTER(t))
    if ret_is_float:
        out.append(ctypes.c_float)
    return out


def _preload_torch():
    # One HIP runtime per process: when torch is importable, let it load its libamdhip64 first so
    # ours resolves to the same SONAME instead of mapping a second copy.
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch absent
        pass


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libloma_nerf.so and set argtypes. Raises if the library is missing (no fallback)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libloma_nerf.so not built at {p} (run __graft_entry__.build())")
    _preload_torch()
    lib = ctypes.CDLL(p)
    configure(lib)
    if path is None:
        _LIB = lib
    return lib


def configure(lib: ctypes.CDLL) -> None:
    lib.nerf_evaluate_and_march.argtypes = NERF_ARGTYPES
    lib.nerf_evaluate_and_march.restype = ctypes.c_float
    lib.grad_nerf_evaluate_and_march.argtypes = rev_argtypes(NERF_ARGTYPES)
    lib.grad_nerf_evaluate_and_march.restype = None
    lib.mlp_fit.argtypes = MLP_FIT_ARGTYPES
    lib.mlp_fit.restype = ctypes.c_float
    lib.grad_mlp_fit.argtypes = rev_argtypes(MLP_FIT_ARGTYPES)
    lib.grad_mlp_fit.restype = None
    lib.mult_a_b.argtypes = MULT_A_B_ARGTYPES
    lib.mult_a_b.restype = None
    lib.lnerf_last_error.restype = ctypes.c_char_p
    lib.lnerf_version.restype = ctypes.c_char_p
    lib.lnerf_build_knobs.argtypes = []
    lib.lnerf_build_knobs.restype = ctypes.c_uint
    lib.lnerf_ctx_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
    lib.lnerf_ctx_destroy.argtypes = [ctypes.c_void_p]
    lib.lnerf_ctx_destroy.restype = None
    lib.lnerf_workspace_bytes.argtypes = [ctypes.POINTER(LnerfMLP), ctypes.c_int, ctypes.c_int]
    lib.lnerf_workspace_bytes.restype = ctypes.c_size_t
    lib.lnerf_train_step.argtypes = [ctypes.c_void_p, ctypes.POINTER(LnerfMLP), ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.POINTER(LnerfBatch), ctypes.c_float,
                                     ctypes.c_int, ctypes.POINTER(LnerfOutputs), ctypes.c_void_p]
    lib.lnerf_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(LnerfMLP), ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.POINTER(LnerfBatch), ctypes.c_int,
                                 ctypes.POINTER(LnerfOutputs), ctypes.c_void_p]
    lib.lnerf_scale_by_device_scalar.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                 ctypes.c_void_p]
    lib.lnerf_adam_update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
    lib.lnerf_ctx_timings.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int]
    lib.lnerf_ctx_last_path.argtypes = [ctypes.c_void_p]
    lib.lnerf_ctx_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.lnerf_ctx_relu_masks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    if hasattr(lib, "lnerf_ctx_exceptional_rows"):   # (older in-tree A/B builds lack it)
        lib.lnerf_ctx_exceptional_rows.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_longlong),
                                                   ctypes.POINTER(ctypes.c_longlong)]
    if hasattr(lib, "lnerf_ctx_guard_fired"):   # (round 6; older A/B builds lack it)
        lib.lnerf_ctx_guard_fired.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    lib.lnerf_get_rays.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_void_p]
    for name in ("lnerf_ctx_timings", "lnerf_ctx_last_path", "lnerf_ctx_set_option", "lnerf_ctx_relu_masks",
                 "lnerf_ctx_exceptional_rows", "lnerf_ctx_guard_fired",
                 "lnerf_ctx_create", "lnerf_train_step", "lnerf_render",
                 "lnerf_scale_by_device_scalar", "lnerf_adam_update", "lnerf_get_rays"):
        if hasattr(lib, name):
            getattr(lib, name).restype = ctypes.c_int


def build_knobs() -> int:
    """lnerf_build_knobs(): non-default compile-time knobs of the loaded library (0 = product)."""
    return int(load_library().lnerf_build_knobs())


def last_error() -> str:
    return load_library().lnerf_last_error().decode()


def make_mlp(shapes, w_k: int, w_n: int) -> LnerfMLP:
    m = LnerfMLP()
    m.num_layers = len(shapes)
    for l, (k, n) in enumerate(shapes):
        m.k[l], m.n[l] = int(k), int(n)
    m.w_k, m.w_n = int(w_k), int(w_n)
    return m


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


@dataclass
class StepResult:
    loss: object        # torch scalar tensor (device)
    acc_color: object   # (rays, 3)
    grads: object       # packed [d_ws (L*w_k*w_n), d_bs (L*w_n), loss] (device)
    d_ws: object
    d_bs: object
    d_dists: object = None
    d_target: object = None
    d_x: object = None


class Engine:
    """Native-API driver on one GPU. Inputs are torch tensors already resident on the device."""

    def __init__(self, device: int = 0):
        import torch
        self.torch = torch
        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        if self.lib.lnerf_ctx_create(ctypes.byref(h), device) != 0:
            raise RuntimeError(f"lnerf_ctx_create: {last_error()}")
        self.ctx = h

    def close(self):
        if self.ctx:
            self.lib.lnerf_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def alloc_grads(self, L: int, w_k: int, w_n: int):
        nW, nB = L * w_k * w_n, L * w_n
        g = self.torch.zeros(nW + nB + 1, dtype=self.torch.float32, device=f"cuda:{self.device}")
        return g, g[:nW].view(L, w_k, w_n), g[nW:nW + nB].view(L, w_n), g[nW + nB:]

    @staticmethod
    def _batch(rays, samples, input_mode, num_freqs, x, dists, target, near, far):
        return LnerfBatch(rays, samples, input_mode, num_freqs, x.data_ptr(),
                          None if dists is None else dists.data_ptr(), target.data_ptr(),
                          float(near), float(far))

    def train_step(self, mlp: LnerfMLP, ws, bs, x, dists, target, *, samples: int,
                   input_mode: int = INPUT_POINTS, num_freqs: int = 5, seed=None, flags: int = 0,
                   grads=None, want_per_ray: bool = False, want_dx: bool = False,
                   acc_color=None, near: float = 2.0, far: float = 6.0) -> StepResult:
        """One fwd+bwd over the batch. seed=None seeds with the batch loss (train_nerf.py:477);
        a float seeds with that constant. `grads` (from alloc_grads) is reused if given.
        INPUT_RAYS: x = (rays, 6) [o, d], dists=None, samples at linspace(near, far, S)."""
        torch = self.torch
        rays = target.shape[0]
        b = self._batch(rays, samples, input_mode, num_freqs, x, dists, target, near, far)
        if grads is None:
            grads = self.alloc_grads(mlp.num_layers, mlp.w_k, mlp.w_n)
        g, dws, dbs, loss = grads
        if acc_color is None:
            acc_color = torch.empty(rays, 3, dtype=torch.float32, device=target.device)
        d_dists = d_target = d_x = None
        if want_per_ray:
            d_dists = torch.empty(rays, samples, dtype=torch.float32, device=target.device)
            d_target = torch.empty(rays, 3, dtype=torch.float32, device=target.device)
        if want_dx:
            d_x = torch.zeros(rays * samples, mlp.k[0], dtype=torch.float32, device=target.device)
            flags |= WANT_DX
        o = LnerfOutputs(loss.data_ptr(), acc_color.data_ptr(), dws.data_ptr(), dbs.data_ptr(),
                         None if d_x is None else d_x.data_ptr(),
                         None if d_dists is None else d_dists.data_ptr(),
                         None if d_target is None else d_target.data_ptr())
        if seed is None:
            flags |= SEED_LOSS
            seed = 1.0
        rc = self.lib.lnerf_train_step(self.ctx, ctypes.byref(mlp), ws.data_ptr(), bs.data_ptr(),
                                       ctypes.byref(b), float(seed), flags, ctypes.byref(o),
                                       self._stream())
        if rc != 0:
            raise RuntimeError(f"lnerf_train_step: {last_error()}")
        return StepResult(loss[0], acc_color, g, dws, dbs, d_dists, d_target, d_x)

    def mlp_fit_step(self, mlp: LnerfMLP, ws, bs, x, target, *, seed=None, flags: int = 0, grads=None,
                     outputs=None, want_grad: bool = True):
        """fit_img.py's chunk step on the device (scripts/mlp_fit.py): the MLP on `x` (rows, k[0])
        ENCODED rows, sigmoid on every output, loss = sum (sigmoid(z) - target)^2 over
        (rows, n_out); with want_grad the reverse pass (grad_mlp_fit) into `grads`, seeded with
        `seed` (fit_img.py:515 passes the previous chunk loss) or, seed=None, with this loss.
        Returns (loss, outputs (rows, n_out), grads)."""
        torch = self.torch
        rows, nout = target.shape[0], mlp.n[mlp.num_layers - 1]
        if outputs is None:
            outputs = torch.empty(rows, nout, dtype=torch.float32, device=target.device)
        if not want_grad:
            loss, out = self.render(mlp, ws, bs, x, None, target, samples=1, input_mode=INPUT_ENCODED,
                                    flags=flags | HEAD_FIT, acc=outputs)
            return loss, out, None
        r = self.train_step(mlp, ws, bs, x, None, target, samples=1, input_mode=INPUT_ENCODED, seed=seed,
                            flags=flags | HEAD_FIT, grads=grads, acc_color=outputs)
        return r.loss, outputs, r.grads

    def render(self, mlp: LnerfMLP, ws, bs, x, dists, target, *, samples: int,
               input_mode: int = INPUT_POINTS, num_freqs: int = 5, near: float = 2.0,
               far: float = 6.0, flags: int = 0, acc=None, loss=None):
        """Forward only (train_nerf.py:616-661 eval render): (loss, acc_color). flags may select
        MFMA_BF16 (the config-5 inference precision), MFMA_BF16X6 or GENERIC."""
        torch = self.torch
        rays = target.shape[0]
        b = self._batch(rays, samples, input_mode, num_freqs, x, dists, target, near, far)
        if acc is None:
            acc = torch.empty(rays, 3, dtype=torch.float32, device=target.device)
        if loss is None:
            loss = torch.empty(1, dtype=torch.float32, device=target.device)
        o = LnerfOutputs(loss.data_ptr(), acc.data_ptr(), None, None, None, None, None)
        rc = self.lib.lnerf_render(self.ctx, ctypes.byref(mlp), ws.data_ptr(), bs.data_ptr(),
                                   ctypes.byref(b), flags, ctypes.byref(o), self._stream())
        if rc != 0:
            raise RuntimeError(f"lnerf_render: {last_error()}")
        return loss[0], acc

    def get_rays(self, width: int, K, c2w):
        """train_nerf.py:23-62 on the device: (width*width, 6) float32 rays [o, d]."""
        import numpy as np
        torch = self.torch
        Kd = np.ascontiguousarray(np.asarray(K, np.float64).reshape(3, 3))
        cd = np.ascontiguousarray(np.asarray(c2w, np.float64)[:3, :4])
        out = torch.empty(width * width, 6, dtype=torch.float32, device=f"cuda:{self.device}")
        dp = ctypes.POINTER(ctypes.c_double)
        rc = self.lib.lnerf_get_rays(width, Kd.ctypes.data_as(dp), cd.ctypes.data_as(dp),
                                     ctypes.c_void_p(out.data_ptr()), self._stream())
        if rc != 0:
            raise RuntimeError(f"lnerf_get_rays: {last_error()}")
        return out

    def timings(self):
        """Per-kernel ms of the last TIMING step: pack, fused, loss, dw, reduce, total."""
        out = (ctypes.c_float * 6)()
        n = self.lib.lnerf_ctx_timings(self.ctx, out, 6)
        if n < 0:
            raise RuntimeError(f"lnerf_ctx_timings: {last_error()}")
        keys = ("pack", "fused", "loss", "dw", "reduce", "total")
        return {keys[i]: out[i] for i in range(n)}

    def exceptional_rows(self, split=False):
        """Rows (summed over layers) the last fp16x3 training step multiplied on the bf16x6 split
        (lnerf_ctx_exceptional_rows; synchronises); split=True: (rows, of them rays' last samples)."""
        n, t = ctypes.c_longlong(0), ctypes.c_longlong(0)
        if self.lib.lnerf_ctx_exceptional_rows(self.ctx, ctypes.byref(n), ctypes.byref(t)) != 0:
            raise RuntimeError(f"lnerf_ctx_exceptional_rows: {last_error()}")
        return (int(n.value), int(t.value)) if split else int(n.value)

    def guard_fired(self):
        """The last training step's fp16x3 floor guard (lnerf_ctx_guard_fired; synchronises): 1 if k1
        found a hidden G element below fp16x3's floor and the step re-ran on the bf16x6 split, 0 if
        not, -1 if the step had no guard (an explicit precision flag, the generic path, ...)."""
        f = ctypes.c_int(0)
        if self.lib.lnerf_ctx_guard_fired(self.ctx, ctypes.byref(f)) != 0:
            raise RuntimeError(f"lnerf_ctx_guard_fired: {last_error()}")
        return int(f.value)

    def last_path(self) -> dict:
        """The kernels the last train_step/render ran (lnerf_ctx_last_path)."""
        v = self.lib.lnerf_ctx_last_path(self.ctx)
        if v < 0:
            raise RuntimeError(f"lnerf_ctx_last_path: {last_error()}")
        return dict(generic=bool(v & PATH_GENERIC), fused=bool(v & PATH_FUSED),
                    k16=bool(v & PATH_K16), dw16=bool(v & PATH_DW16), k16_w4=bool(v & PATH_K16_W4),
                    kr=bool(v & PATH_KR), a24=bool(v & PATH_A24),
                    planes=(v >> 8) & 3)

    def relu_masks(self, L: int, R: int):
        """The last training step's hidden ReLU decisions (k16 path): numpy bool (L-1, R, 256),
        [l, r, f] = feature f of hidden layer l at sample row r was positive."""
        import numpy as np
        torch = self.torch
        out = torch.empty((L - 1) * R * 32, dtype=torch.uint8, device=f"cuda:{self.device}")
        rc = self.lib.lnerf_ctx_relu_masks(self.ctx, ctypes.c_void_p(out.data_ptr()), out.numel(),
                                           self._stream())
        if rc != 0:
            raise RuntimeError(f"lnerf_ctx_relu_masks: {last_error()}")
        bits = out.cpu().numpy().reshape(L - 1, R, 32)
        return np.unpackbits(bits, axis=2, bitorder="little").astype(bool)

    def set_option(self, option: int, value: int):
        """lnerf_ctx_set_option (OPT_DW_GRID: the dW kernel's workgroup budget, 0 = default)."""
        if self.lib.lnerf_ctx_set_option(self.ctx, option, value) != 0:
            raise RuntimeError(f"lnerf_ctx_set_option: {last_error()}")

    def scale_by_device_scalar(self, buf, scale):
        rc = self.lib.lnerf_scale_by_device_scalar(ctypes.c_void_p(buf.data_ptr()), buf.numel(),
                                                   ctypes.c_void_p(scale.data_ptr()),
                                                   self._stream())
        if rc != 0:
            raise RuntimeError(f"lnerf_scale_by_device_scalar: {last_error()}")

    def adam_update(self, params, grads, m, v, t: int, lr: float, beta1=0.9, beta2=0.999,
                    eps=1e-8):
        rc = self.lib.lnerf_adam_update(params.data_ptr(), grads.data_ptr(), m.data_ptr(),
                                        v.data_ptr(), params.numel(), t, lr, beta1, beta2, eps,
                                        self._stream())
        if rc != 0:
            raise RuntimeError(f"lnerf_adam_update: {last_error()}")
