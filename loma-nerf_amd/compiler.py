"""Drop-in for loma's `compiler` module (loma_public/compiler.py:70-278) on MI355X.

The reference's drivers do `sys.path.append(loma_public)`, `import compiler` and then
`_, lib = compiler.compile(open("scripts/nerf.py").read(), target="c", output_filename=...)`
(train_nerf.py:4-12,209-213; fit_img.py:355-361). Put this directory *before* loma_public on
sys.path (or on PYTHONPATH) and the same call returns a CDLL of libloma_nerf.so whose
`nerf_evaluate_and_march`, `grad_nerf_evaluate_and_march`, `mlp_fit`, `grad_mlp_fit` and
`mult_a_b` carry the argtypes loma would have set (compiler.py:262-276), backed by HIP kernels.

No loma is compiled: the engine implements the NeRF programs natively. `compile` therefore checks
that the source defines exactly those programs (a fingerprint of each function's AST, so
formatting and comments do not matter) and raises for anything else -- set
LNERF_ALLOW_UNVERIFIED=1 to bind modified sources anyway (their semantics stay the reference's).
"""
from __future__ import annotations

import ast
import ctypes
import hashlib
import os
import sys
import warnings

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import lnerf  # noqa: E402


class UserError(Exception):
    """Mirrors loma's error.UserError for callers that catch it."""


# sha256(ast.dump(FunctionDef, include_attributes=False)) of the reference programs this engine
# implements (scripts/nerf.py:1-304, scripts/mlp_fit.py:1-147 and :150-172).
KNOWN_FUNCTIONS = {
    "nerf_evaluate_and_march": "e93e4a98564e4cf86b9e53f08b1d8438a4c0447c746f6bd106e1615512701675",
    "mlp_fit": "355b6b3323508d6c91f6602ec9a146681e55e355d5910c45ad80f12a085153b9",
    "mult_a_b": "547f3700098905eec9fc3bf11d3c5ec0f8ce3e34e4a590a93a5bb7535a19dc1a",
}
GRADIENTS = {"nerf_evaluate_and_march": "grad_nerf_evaluate_and_march", "mlp_fit": "grad_mlp_fit"}


def _fingerprint(fn: ast.FunctionDef) -> str:
    return hashlib.sha256(ast.dump(fn, include_attributes=False).encode()).hexdigest()


def _scan(loma_code: str):
    try:
        tree = ast.parse(loma_code)
    except SyntaxError as e:
        raise UserError(f"cannot parse loma source: {e}") from e
    funcs, grads = {}, {}
    for node in tree.body:
        if isinstance(node, ast.FunctionDef):
            funcs[node.name] = node
        elif isinstance(node, ast.Assign) and isinstance(node.value, ast.Call):
            call = node.value
            if isinstance(call.func, ast.Name) and call.func.id in ("rev_diff", "fwd_diff"):
                if call.func.id == "fwd_diff":
                    raise UserError("fwd_diff is not provided by the MI355X engine")
                tgt = node.targets[0].id
                src = call.args[0].id
                grads[tgt] = src
    return funcs, grads


def compile(loma_code: str, target: str = "c", output_filename: str | None = None,
            opencl_context=None, opencl_device=None, opencl_command_queue=None,
            print_error: bool = True):
    """compiler.py:70-278 contract: returns (ctypes_structs, lib). `target` and
    `output_filename` are accepted for source compatibility; every target runs on the GPU."""
    funcs, grads = _scan(loma_code)
    allow = os.environ.get("LNERF_ALLOW_UNVERIFIED") == "1"
    for name, fn in funcs.items():
        if name not in KNOWN_FUNCTIONS:
            raise UserError(f"loma function '{name}' is not implemented by the MI355X engine")
        if _fingerprint(fn) != KNOWN_FUNCTIONS[name]:
            msg = (f"loma function '{name}' differs from the reference program the engine "
                   f"implements (scripts/nerf.py / scripts/mlp_fit.py)")
            if not allow:
                raise UserError(msg + "; set LNERF_ALLOW_UNVERIFIED=1 to bind it anyway")
            warnings.warn(msg)
    for gname, src in grads.items():
        if GRADIENTS.get(src) != gname:
            raise UserError(f"gradient '{gname} = rev_diff({src})' is not provided "
                            f"(expected names: {GRADIENTS})")
    # a fresh CDLL object per compile (its own function-pointer cache, like loma's CDLL)
    lib = lnerf.load_library(lnerf.LIB_PATH)
    return {}, lib


__all__ = ["compile", "UserError"]
