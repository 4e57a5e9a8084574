"""Host-only AddressSanitizer + UBSan run of the loma-ABI marshalling (SURVEY.md §5 sanitizers):
tests/native/marshal_check.cpp builds the product's gather/scatter (loma-nerf_amd/csrc/
lnerf_marshal.h) and the oracle's nested-pointer wrapper (oracle/nerf_oracle_abi.c + the C
restatement) with -fsanitize=address,undefined and runs them on ctypes-style row-allocated tables
of the train_nerf chunk (fake trace and real rows) and an mlp_fit chunk. No GPU, no HIP."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="no host toolchain")
def test_marshalling_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", NATIVE], check=True)
    env = dict(os.environ)
    # the harness may preload a library of its own ahead of the ASan runtime
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([os.path.join(NATIVE, "build", "marshal_check")], env=env, capture_output=True,
                       text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    assert "all marshalling checks passed" in out, out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out
