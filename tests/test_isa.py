"""The shipped code object's waits and wait states, read back from its disassembly (CPU only).

Why: round 3's k16 read its weight fragments and biases through inline-asm
`ds_read_b128` counted by hand, and split its operands in inline asm. hipcc neither counts an asm
load nor pads the MFMA wait states around an asm statement (cdna_hip_programming.md §5.7): the
k16 build under LLVM's max-ilp scheduler returned a 1.8 % wrong loss (gpurun_out/t19.log). The
audit of that build (scripts/isa_check.py) found the cause: the asm operand split wrote the next
k-step's B registers 1-2 wait states after an MFMA that still read the same registers as its C
operand (gfx950 needs 3 for a 4-pass XDL MFMA) -- 33 such writes in the default <16,2,8>
instantiation and 5-57 in every other fp16x3 one, in BOTH builds; which schedule the race
corrupted was luck. Round 4 keeps the LDS-DMA in asm (no register destination, counted by its
own vmcnt) and makes every VGPR-writing instruction compiler-visible or in-place, so:

  * every load's destination is waited for before any use, on every path of every kernel
    (pending-load audit, all product kernels);
  * the fp16x3 / bf16 k16 instantiations and dw16 satisfy the gfx950 MFMA wait-state rules
    (MFMA D -> reader/writer, C read -> VALU write, VALU write -> MFMA operand);
  * M0 is read only by the LDS-DMA right after the asm statement that wrote it;
  * no inline asm in the kernels writes a register except in place ("+v": its last writer was a
    compiler instruction the compiler already padded).
Test infrastructure; the product never imports scripts/.
"""
import os
import re
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "loma-nerf_amd", "lib", "libloma_nerf.so")
CSRC = os.path.join(ROOT, "loma-nerf_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "scripts"))

# the product instantiations: cfg3 fp16x3 training (<16,2,8>), cfg2 (<2,2,8>), the render
# (<16,1,8>), the 4-wave variant (<16,2,4>), bf16x6 (<16,3,8>), the deep-narrow <4,2,8>
K16 = r"k16_fwd_bwd_kernelILi(16|2|4)ELi[123]ELi[48]E"
K16_SPLIT_BF16 = r"k16_fwd_bwd_kernelILi(16|2|4)ELi[12]ELi[48]E"   # the MFMA rules: fp16x3 + bf16
DW16 = r"dw16_kernel"
KR = r"kr_fwd_kernel"   # the bf16 render kernel (lnerf_render.hip)
OTHER = r"(pack16|wmax16|k16_masks|k1_reduce|grad_reduce|loss_reduce|lg_|k_adam|adam|get_rays|positional|ray_)"


@pytest.fixture(scope="module")
def asm():
    if not os.path.exists(LIB):
        pytest.skip("libloma_nerf.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    import isa_check
    return isa_check.disassemble_all(LIB)


def _report(asm, rx):
    import isa_check
    rep = isa_check.check(LIB, rx, asm=asm)
    assert rep, f"no kernel matches {rx}"
    return rep


def _fmt(name, fs):
    return [f"{name[:60]}: {k} at {ins.addr:#x} {ins.mn} {ins.ops.strip()} <- {src:#x} {regs}"
            for k, ins, src, regs in fs[:5]]


def test_every_load_waited_for_before_use(asm):
    bad = []
    for rx in (K16, DW16, KR, OTHER):
        for name, fs in _report(asm, rx).items():
            bad += _fmt(name, [f for f in fs if f[0] == "pending-load"])
    assert not bad, "\n".join(bad)


def test_mfma_wait_states_product_kernels(asm):
    bad = []
    for rx in (K16_SPLIT_BF16, DW16, KR):
        for name, fs in _report(asm, rx).items():
            bad += _fmt(name, fs)
    assert not bad, "\n".join(bad)


def test_m0_read_only_by_lds_dma(asm):
    import isa_check
    kernels = isa_check.parse_kernels(asm, K16 + "|" + KR)
    assert kernels
    bad = []
    for name, insts in kernels.items():
        bad += _fmt(name, isa_check.m0_findings(insts))
        assert any("load_lds" in i.mn for i in insts), name   # the weight ring is LDS-DMA fed
    assert not bad, "\n".join(bad)


_ASM = re.compile(r"\basm\s*(?:volatile\s*)?\((.*?)\);", re.S)


def test_inline_asm_writes_registers_only_in_place():
    """Source rule behind the ISA checks: an asm statement may write a register only in place."""
    found = []
    for fn in sorted(os.listdir(CSRC)):
        if not fn.endswith((".hip", ".h", ".cpp")):
            continue
        src = open(os.path.join(CSRC, fn)).read()
        for m in _ASM.finditer(src):
            body = m.group(1)
            parts = body.split(":")
            outs = parts[1] if len(parts) > 1 else ""
            for c in re.findall(r'"([^"]*)"\s*\(', outs):
                if c.startswith("=") and ("v" in c or "a" in c):
                    line = src[:m.start()].count("\n") + 1
                    found.append(f"{fn}:{line}: output constraint {c!r}")
    assert not found, "\n".join(found)


def test_int24_activation_slabs_move_12_bytes_per_lane(asm):
    """fp16x3 training writes and reads the A slabs as int24 (lnerf_internal.h a24_slabs): k1
    stores 12 B per lane (global_store_dwordx3) and k2 loads 12 B per lane (global_load_dwordx3).
    Guards a round-4 miscompile: __builtin_bit_cast of an ext_vector element (raw[1]) yielded
    element 0, so k2's decode read one dword three times and the compiler narrowed the 12-B load
    to one global_load_dword (three quarters of A decoded from the wrong bytes)."""
    import isa_check
    k1 = isa_check.parse_kernels(asm, r"k16_fwd_bwd_kernelILi16ELi2ELi8E")
    k2 = isa_check.parse_kernels(asm, r"dw16_kernelILi2E")
    assert k1 and k2
    for name, insts in k1.items():
        assert any(i.mn == "global_store_dwordx3" for i in insts), name
        # the packed int24 data (v_perm_b32 results) leaves only through 12-B stores: a store
        # widened to 16 B would overwrite the neighbouring lane's 4 bytes (the 12-B runs
        # are only 4-B aligned), so no dwordx4 store may take a register v_perm_b32 wrote last
        last = {}
        for i in insts:
            if i.mn.startswith("global_store"):
                data = isa_check.regs_of(i.ops.split(",")[1]) if "," in i.ops else frozenset()
                perm = {r for r in data if last.get(r) == "v_perm_b32"}
                # (the 2-B store of a row's shift word, built by v_perm_b32 too, is not slab data)
                if perm and i.mn not in ("global_store_byte", "global_store_short"):
                    assert i.mn == "global_store_dwordx3", (name, hex(i.addr), i.mn, i.ops)
            for r in getattr(i, "vdst", ()):
                last[r] = i.mn
    for name, insts in k2.items():
        assert any(i.mn == "global_load_dwordx3" for i in insts), name
