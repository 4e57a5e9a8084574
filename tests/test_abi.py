"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol include/lnerf.h
declares, binds with the argtypes loma's compiler would set, and fails loudly (no CPU fallback)
when no GPU is present. No compute calls are made on the GPU here."""
import ast
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import lnerf
from conftest import REPO, gpu_available

HEADER = os.path.join(REPO, "include", "lnerf.h")
REF_SCRIPTS = "/root/reference/scripts"


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "while", "sizeof")))


def test_header_symbols_match_binding_list():
    assert header_functions() == sorted(lnerf.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol():
    lib = lnerf.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", lnerf.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    for name in header_functions():
        assert name in exported, name
    assert lib.lnerf_version().decode().startswith("loma-nerf-amd")


def test_shipped_library_is_knob_free():
    """The library the product path loads was built with every compile-time knob at its product
    default (lnerf_build_knobs() == 0): no A/B or phase-profiling variant is installed as
    lib/libloma_nerf.so (the wrong-result timing knobs no longer exist in the sources)."""
    if os.environ.get("LNERF_LIB"):
        pytest.skip("LNERF_LIB selects a variant library on purpose")
    assert lnerf.build_knobs() == 0
    csrc = os.path.join(REPO, "loma-nerf_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h", ".cpp")):
            src = open(os.path.join(csrc, f)).read()
            for knob in ("NOSTORE", "NODMA", "NOBAR", "NOPE", "NOCOMP", "HALFLDS", "NOSPLIT", "NOMMA"):
                assert f"LNERF_K16_{knob}" not in src and f"LNERF_DW16_{knob}" not in src, (f, knob)


def test_library_is_gfx950_code_object():
    # the fat binary embeds the offload target triple of its code object(s)
    blob = open(lnerf.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def _loma_ctypes(annotation):
    """compiler.py:25-51 loma_to_ctypes_type, restated for In[...] / Out[...] annotations."""
    def base(node):
        if isinstance(node, ast.Name):
            return {"float": ctypes.c_float, "int": ctypes.c_int}[node.id]
        assert isinstance(node, ast.Subscript) and node.value.id == "Array"
        return ctypes.POINTER(base(node.slice))
    inout = annotation.value.id
    t = base(annotation.slice)
    if inout == "Out" and not issubclass(t, ctypes._Pointer):
        t = ctypes.POINTER(t)
    return t


@pytest.mark.skipif(not os.path.isdir(REF_SCRIPTS), reason="reference sources not present")
@pytest.mark.parametrize("script,funcs", [
    ("nerf.py", ["nerf_evaluate_and_march", "grad_nerf_evaluate_and_march"]),
    ("mlp_fit.py", ["mlp_fit", "grad_mlp_fit", "mult_a_b"]),
])
def test_compiler_shim_binds_reference_programs_with_loma_argtypes(script, funcs):
    import compiler
    src = open(os.path.join(REF_SCRIPTS, script)).read()
    structs, lib = compiler.compile(src, target="c", output_filename="_code/x")
    assert structs == {}
    tree = ast.parse(src)
    defs = {n.name: n for n in tree.body if isinstance(n, ast.FunctionDef)}
    for f in funcs:
        fn = getattr(lib, f)
        if f.startswith("grad_"):
            fwd = defs[f[len("grad_"):]]
            expect = []
            for a in fwd.args.args:
                t = _loma_ctypes(a.annotation)
                expect += [t, t if issubclass(t, ctypes._Pointer) else ctypes.POINTER(t)]
            expect.append(ctypes.c_float)      # _dreturn (reverse_diff.py:515-517)
            assert fn.restype is None
        else:
            expect = [_loma_ctypes(a.annotation) for a in defs[f].args.args]
            ret = defs[f].returns
            assert fn.restype == (ctypes.c_float if ret is not None else None)
        got = fn.argtypes
        assert len(got) == len(expect), f
        for g, e in zip(got, expect):
            assert ctypes.sizeof(g) == ctypes.sizeof(e)
            assert g.__name__ == e.__name__, (f, g, e)


@pytest.mark.skipif(not os.path.isdir(REF_SCRIPTS), reason="reference sources not present")
def test_compiler_shim_rejects_other_programs(monkeypatch):
    import compiler
    src = open(os.path.join(REF_SCRIPTS, "nerf.py")).read()
    with pytest.raises(compiler.UserError):
        compiler.compile(src.replace("+ 1e-10", "+ 1e-9"))           # modified semantics
    with pytest.raises(compiler.UserError):
        compiler.compile("def foo(x: In[float]) -> float:\n    return x\n")
    with pytest.raises(compiler.UserError):
        compiler.compile(src.replace("rev_diff(", "fwd_diff("))
    monkeypatch.setenv("LNERF_ALLOW_UNVERIFIED", "1")
    with pytest.warns(UserWarning):
        compiler.compile(src.replace("+ 1e-10", "+ 1e-9"))


def test_compiler_shim_formatting_insensitive():
    """The fingerprint is over the AST, so comments and layout do not matter."""
    import compiler
    if not os.path.isdir(REF_SCRIPTS):
        pytest.skip("reference sources not present")
    src = open(os.path.join(REF_SCRIPTS, "mlp_fit.py")).read()
    src2 = "# leading comment\n\n" + src.replace("    i: int = 0", "    i: int = 0  # trailing")
    compiler.compile(src2)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure mode")
def test_compat_call_without_gpu_fails_loudly():
    """No CPU fallback: without a device the loma entry points return NaN and set the error."""
    from loma_marshal import to_ctypes
    lib = lnerf.load_library()
    a = np.ones((2, 2), np.float32)
    loss = lib.mlp_fit(to_ctypes(a), 2, 2, to_ctypes(a), to_ctypes(np.ones((1, 2, 2), np.float32)),
                       to_ctypes(np.ones((1, 2), np.float32)), to_ctypes(a), 2, 2, 1,
                       to_ctypes(np.array([[2, 2]], np.int32)), to_ctypes(np.array([[2, 1]], np.int32)),
                       to_ctypes(np.array([[2, 2]], np.int32)), to_ctypes(np.zeros((1, 2, 2), np.float32)))
    assert np.isnan(loss)
    assert lnerf.last_error() != ""
    h = ctypes.c_void_p()
    assert lib.lnerf_ctx_create(ctypes.byref(h), 0) != 0


def test_generic_and_fused_shape_support_flags():
    # flag values are part of the ABI
    assert (lnerf.SEED_LOSS, lnerf.ACCUMULATE, lnerf.WANT_DX, lnerf.GENERIC, lnerf.FAST,
            lnerf.TIMING, lnerf.MFMA_F32, lnerf.MFMA_BF16) == (1, 2, 4, 8, 16, 32, 64, 128)
    src = open(HEADER).read()
    for name, val in (("LNERF_SEED_LOSS", 1), ("LNERF_ACCUMULATE", 2), ("LNERF_WANT_DX", 4),
                      ("LNERF_GENERIC", 8), ("LNERF_FAST", 16), ("LNERF_TIMING", 32),
                      ("LNERF_MFMA_F32", 64), ("LNERF_MFMA_BF16", 128)):
        assert re.search(rf"{name}\s*=\s*{val}\b", src), name
