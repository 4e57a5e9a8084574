#!/usr/bin/env python3
"""Wait-count and MFMA-hazard audit of a gfx950 code object, from the disassembly alone.

Why: the fused kernels issue some LDS reads from inline asm (lnerf_k16.hip ds_read_at, the bias
reads; lnerf_k32.hip) and wait for them with hand-counted `s_waitcnt lgkmcnt(N)`, and write some
operands from inline asm (the fp16x3 operand split, the ReLU mask chain). hipcc neither counts
an asm load (it may copy, spill or overwrite the destination before the data lands) nor pads
the wait states around an asm statement's instructions (cdna_hip_programming.md §5.7 items 1-2).
Round 3's k16 build under the max-ilp scheduler gave a 1.8 % wrong loss; this audit re-derives,
on every path of every kernel:

1. **Pending loads** (MI355X_MICROARCH.md: vector-memory ops -- loads, stores, LDS-DMA -- retire
   in issue order; LDS ops retire in order; SMEM in any order). After `lgkmcnt(N)` an LDS op may
   still be pending iff fewer than N LDS ops were issued after it; an SMEM op iff N > 0. After
   `vmcnt(N)` a VM op may still be pending iff fewer than N VM ops were issued after it.
   Finding: an instruction (other than s_waitcnt) naming a register whose load may be pending.
2. **MFMA wait states** (the gfx950 rules of LLVM's GCNHazardRecognizer; one state per
   instruction, N + 1 per `s_nop N`):
   * an XDL MFMA's D -> any non-MFMA reader or writer of it: passes + 4 states (passes + 3 for
     2-pass); the next MFMA may take it whole as C with no gap;
   * an MFMA reading C -> a VALU write of it (WAR): passes - 1 states;
   * a VALU write -> an MFMA reading it as A, B or C: 2 states.
Control flow: a may-analysis over basic blocks (union of pending ops / recent events at joins,
the minimum count of younger ops and of elapsed states), iterated to a fixpoint.

Usage: isa_check.py LIB.so|OBJ.o [--kernel REGEX] [-v]   (exit 1 on any finding)
Test infrastructure (tests/test_isa.py): the product never imports this.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
CAP = 64       # younger-op counts saturate here (the counters are 6-bit)
WINDOW = 24    # MFMA / VALU events older than this many wait states are dropped

_line_re = re.compile(r"^\s+(\S+)(.*?)\s*//\s*([0-9A-Fa-f]+):")
_fn_re = re.compile(r"^([0-9a-f]+) <([^>]+)>:")
_rng_re = re.compile(r"(?<![\w])([vsa])\[(\d+):(\d+)\]")
_one_re = re.compile(r"(?<![\w\[:])([vsa])(\d+)(?![\w:])")
_cnt_re = re.compile(r"(vmcnt|lgkmcnt|expcnt)\((\d+)\)")


def extract_code_objects(path: str, out_dir: str) -> list:
    """The gfx950 code objects of a hipcc-built .so or .o: its .hip_fatbin section holds one
    offload bundle per translation unit (a linked .so concatenates them)."""
    fb = os.path.join(out_dir, "fatbin.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--only-section=.hip_fatbin", f"--dump-section=.hip_fatbin={fb}",
                    path, os.path.join(out_dir, "junk")], check=True, capture_output=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    cos = []
    for i, st in enumerate(starts):
        part = os.path.join(out_dir, f"bundle{i}.bin")
        with open(part, "wb") as f:
            f.write(data[st:starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(out_dir, f"gfx950_{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            cos.append(co)
    return cos


def disassemble(co: str) -> str:
    r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True,
                       text=True)
    return r.stdout


def disassemble_all(path: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        return "\n".join(disassemble(co) for co in extract_code_objects(path, d))


def regs_of(ops: str) -> frozenset:
    out = set()
    for m in _rng_re.finditer(ops):
        k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
        out.update(f"{k}{i}" for i in range(a, b + 1))
    for m in _one_re.finditer(ops):
        out.add(f"{m.group(1)}{m.group(2)}")
    return frozenset(out)


def _operands(ops: str):
    ops = ops.strip()
    return [o.strip() for o in ops.split(",")] if ops else []


def mfma_passes(mn: str) -> int:
    m = re.search(r"_(\d+)x(\d+)x(\d+)", mn)
    if not m:
        return 8
    mm = int(m.group(1))
    return {4: 2, 16: 4, 32: 8}.get(mm, 8)   # gfx950: 16x16x32 16 cycles = 4 passes


class Inst:
    __slots__ = ("addr", "size", "mn", "ops", "regs", "kind", "dst", "wait", "states", "valu", "mfma",
                 "vdst", "srcab", "srcc", "passes", "vreads")

    def __init__(self, addr, mn, ops):
        self.addr, self.mn, self.ops = addr, mn, ops
        self.regs = regs_of(ops)
        self.kind = None     # "lds" | "smem" | "vm" | "vm+smem" (flat)
        self.dst = frozenset()
        self.wait = None     # (vm, lgkm) limits of an s_waitcnt
        self.states = 1
        self.mfma = mn.startswith(("v_mfma", "v_smfmac"))
        self.valu = mn.startswith("v_") and not self.mfma
        opl = _operands(ops)
        self.vdst = frozenset(r for r in regs_of(opl[0]) if r[0] in "va") if (opl and (self.valu or self.mfma)) \
            else frozenset()
        self.vreads = frozenset(r for r in self.regs if r[0] in "va")
        self.srcab = self.srcc = frozenset()
        self.passes = 0
        if self.mfma and len(opl) >= 4:
            self.srcab = regs_of(opl[1]) | regs_of(opl[2])
            self.srcc = regs_of(opl[3])
            self.passes = mfma_passes(mn)
        if mn == "s_nop":
            try:
                self.states = int(ops.strip(), 0) + 1
            except ValueError:
                self.states = 1
        if mn.startswith("ds_"):
            self.kind = "lds"
            if any(t in mn for t in ("read", "permute", "swizzle", "_rtn", "consume", "append")):
                self.dst = regs_of(opl[0]) if opl else frozenset()
        elif mn.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_memtime", "s_memrealtime",
                            "s_dcache", "s_sendmsg", "s_atc_probe", "s_get_waveid")):
            self.kind = "smem"
            if mn.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_memtime", "s_memrealtime")):
                self.dst = regs_of(opl[0]) if opl else frozenset()
        elif mn.startswith(("global_", "buffer_", "scratch_", "image_", "tbuffer_")):
            self.kind = "vm"
            if ("load" in mn and "load_lds" not in mn) or ("atomic" in mn and re.search(r"\b(sc0|glc)\b", ops)):
                self.dst = regs_of(opl[0]) if opl else frozenset()
        elif mn.startswith("flat_"):
            self.kind = "vm+smem"
            if "load" in mn or ("atomic" in mn and re.search(r"\b(sc0|glc)\b", ops)):
                self.dst = regs_of(opl[0]) if opl else frozenset()
        if mn == "s_waitcnt":
            lim = {"vmcnt": 63, "lgkmcnt": 15}
            found = False
            for m in _cnt_re.finditer(ops):
                found = True
                if m.group(1) in lim:
                    lim[m.group(1)] = int(m.group(2))
            if not found:
                try:   # raw immediate: the gfx9 encoding
                    v = int(ops.strip(), 0)
                    lim["vmcnt"] = (v & 0xF) | ((v >> 10) & 0x30)
                    lim["lgkmcnt"] = (v >> 8) & 0xF
                except ValueError:
                    pass
            self.wait = (lim["vmcnt"], lim["lgkmcnt"])


def parse_kernels(asm: str, kernel_re: str = ".") -> dict:
    kernels, cur = {}, None
    rx = re.compile(kernel_re)
    for line in asm.splitlines():
        m = _fn_re.match(line)
        if m:
            cur = kernels.setdefault(m.group(2), []) if rx.search(m.group(2)) else None
            continue
        if cur is None:
            continue
        m = _line_re.match(line)
        if m:
            cur.append(Inst(int(m.group(3), 16), m.group(1), m.group(2)))
    for insts in kernels.values():
        for i, ins in enumerate(insts):
            ins.size = (insts[i + 1].addr - ins.addr) if i + 1 < len(insts) else 4
    return kernels


def blocks_of(insts):
    """Basic blocks [(start, end)] and successor lists (block indices)."""
    idx = {ins.addr: i for i, ins in enumerate(insts)}
    leaders = {0}
    succ_i = {}
    for i, ins in enumerate(insts):
        mn = ins.mn
        if mn.startswith(("s_branch", "s_cbranch")):
            tgt = None
            try:
                imm = int(_operands(ins.ops)[0].split()[0], 0)
                if imm >= 0x8000:
                    imm -= 0x10000
                tgt = idx.get(ins.addr + ins.size + 4 * imm)
            except (ValueError, IndexError):
                pass
            s = [tgt] if tgt is not None else []
            if mn.startswith("s_cbranch") and i + 1 < len(insts):
                s.append(i + 1)
            succ_i[i] = s
            leaders.update(s)
            if i + 1 < len(insts):
                leaders.add(i + 1)
        elif mn in ("s_endpgm", "s_setpc_b64", "s_trap"):
            succ_i[i] = []
            if i + 1 < len(insts):
                leaders.add(i + 1)
    starts = sorted(leaders)
    bidx = {s: b for b, s in enumerate(starts)}
    blocks, succ = [], []
    for b, s in enumerate(starts):
        e = starts[b + 1] if b + 1 < len(starts) else len(insts)
        blocks.append((s, e))
        last = e - 1
        if last in succ_i:
            succ.append([bidx[t] for t in succ_i[last]])
        else:
            succ.append([b + 1] if b + 1 < len(starts) else [])
    return blocks, succ


# State: (pend, mf, vw)
#   pend: {op_addr: (kind, dst_regs, younger_lds, younger_vm)}  may-pending loads
#   mf:   {mfma_addr: (elapsed_states, vdst, srcc, passes)}      recent MFMAs
#   vw:   {valu_addr: (elapsed_states, vdst)}                    recent VALU writes

def step(ins, pend, mf, vw, findings):
    """Apply one instruction in place; append findings (kind, ins, src_addr, regs) if a list."""
    if ins.wait is not None:
        vm_lim, lg_lim = ins.wait
        for a in list(pend):
            k, d, yl, yv = pend[a]
            if (k == "lds" and yl >= lg_lim) or (k == "smem" and lg_lim == 0) or \
                    (k == "vm" and yv >= vm_lim) or (k == "vm+smem" and yv >= vm_lim and lg_lim == 0):
                del pend[a]
    else:
        if findings is not None and ins.regs:
            for a, (k, d, yl, yv) in pend.items():
                if d and not d.isdisjoint(ins.regs):
                    hit = d & ins.regs
                    if k == ins.kind and k in ("lds", "vm"):
                        # a younger load of the same in-order class may overwrite an older one's
                        # destination (it returns later); its address / data operands may not
                        hit = hit - ins.dst
                    if hit:
                        findings.append(("pending-load", ins, a, sorted(hit)))
        if findings is not None and (ins.valu or ins.kind or ins.mfma):
            for a, (el, dst, srcc, passes) in mf.items():
                if ins.mfma:
                    if dst and not dst.isdisjoint(ins.srcab):
                        need = passes + 3 + (passes != 2)
                        if el < need:
                            findings.append(("mfma-D->srcAB", ins, a, sorted(dst & ins.srcab) + [f"el={el}"]))
                    # D -> C of the next MFMA: exact overlap chains with no gap (not modelled further)
                    continue
                if dst and not dst.isdisjoint(ins.vreads):
                    need = passes + 3 + (passes != 2)
                    if el < need:
                        findings.append(("mfma-D->use", ins, a, sorted(dst & ins.vreads) + [f"el={el}"]))
                if ins.valu and srcc and not srcc.isdisjoint(ins.vdst):
                    if el < passes - 1:
                        findings.append(("mfma-C-WAR", ins, a, sorted(srcc & ins.vdst) + [f"el={el}"]))
        if findings is not None and ins.mfma:
            srcs = ins.srcab | ins.srcc
            for a, (el, dst) in vw.items():
                if el < 2 and not dst.isdisjoint(srcs):
                    findings.append(("valu->mfma", ins, a, sorted(dst & srcs)))
        if ins.kind is not None:
            for a in pend:
                k, d, yl, yv = pend[a]
                if ins.kind == "lds":
                    yl = min(CAP, yl + 1)
                if ins.kind.startswith("vm"):
                    yv = min(CAP, yv + 1)
                pend[a] = (k, d, yl, yv)
            if ins.dst:   # ops without a register destination only count as younger ops
                pend[ins.addr] = (ins.kind, ins.dst, 0, 0)
    # elapse wait states (the instruction itself is one state, s_nop N is N + 1)
    s = ins.states
    for a in list(mf):
        el, dst, srcc, p = mf[a]
        el += s
        if el > WINDOW:
            del mf[a]
        else:
            mf[a] = (el, dst, srcc, p)
    for a in list(vw):
        el, dst = vw[a]
        el += s
        if el > WINDOW:
            del vw[a]
        else:
            vw[a] = (el, dst)
    if ins.mfma:
        # an MFMA taking an older MFMA's D as its C has consumed it (the hardware orders the chain):
        # that D no longer needs the reader/writer gap, only this MFMA's C read (WAR) does
        for a in list(mf):
            el, dst, srcc, p = mf[a]
            if dst and not dst.isdisjoint(ins.srcc):
                mf[a] = (el, dst - ins.srcc, srcc, p)
        mf[ins.addr] = (0, ins.vdst, ins.srcc, ins.passes)
    elif ins.valu and ins.vdst:
        vw[ins.addr] = (0, ins.vdst)
    # a later write of a register ends an older MFMA's / VALU's claim on it only for RAW; keep it


def merge_into(dst, src, fn):
    changed = False
    for k, v in src.items():
        o = dst.get(k)
        if o is None:
            dst[k] = v
            changed = True
        else:
            m = fn(o, v)
            if m != o:
                dst[k] = m
                changed = True
    return changed


def _m_pend(o, v):
    return (o[0], o[1], min(o[2], v[2]), min(o[3], v[3]))


def _m_mf(o, v):
    return (min(o[0], v[0]),) + o[1:]


def analyse(insts):
    blocks, succ = blocks_of(insts)
    nb = len(blocks)
    sin = [None] * nb
    sin[0] = ({}, {}, {})
    import heapq
    heap = [0]
    queued = [False] * nb
    queued[0] = True
    while heap:
        b = heapq.heappop(heap)
        queued[b] = False
        pend, mf, vw = (dict(x) for x in sin[b])
        s, e = blocks[b]
        for i in range(s, e):
            step(insts[i], pend, mf, vw, None)
        for t in succ[b]:
            if sin[t] is None:
                sin[t] = (dict(pend), dict(mf), dict(vw))
                ch = True
            else:
                tp, tm, tv = sin[t]
                ch = merge_into(tp, pend, _m_pend) | merge_into(tm, mf, _m_mf) | merge_into(tv, vw, _m_mf)
            if ch and not queued[t]:
                queued[t] = True
                heapq.heappush(heap, t)
    findings = []
    for b in range(nb):
        if sin[b] is None:
            continue
        pend, mf, vw = (dict(x) for x in sin[b])
        s, e = blocks[b]
        for i in range(s, e):
            step(insts[i], pend, mf, vw, findings)
    return findings


# Instructions that read M0 on gfx950 besides s_mov / s_add writes to it: LDS-DMA (its LDS base),
# indexed register moves, messages, interpolation and GWS.
_M0_READERS = ("global_load_lds", "buffer_load", "s_movrel", "v_movrel", "s_sendmsg", "v_interp",
               "ds_gws", "s_set_gpr_idx", "ds_append", "ds_consume", "ds_ordered")


def m0_findings(insts):
    """M0 is written only right before an LDS-DMA that reads it (lnerf_k16.hip glds16 writes it in
    the same asm statement): every M0 reader must be an LDS-DMA whose M0 was written at most two
    instructions earlier in the same straight line, and nothing else may read M0."""
    out = []
    for i, ins in enumerate(insts):
        reads_m0 = "m0" in ins.ops.replace(" ", "").split(",")[1:] or ins.mn.startswith(_M0_READERS)
        if not reads_m0 or ins.mn.startswith("s_mov_b32") and ins.ops.strip().startswith("m0"):
            continue
        if ins.mn.startswith("buffer_load") and " lds" not in ins.ops:
            continue
        if "load_lds" in ins.mn or (ins.mn.startswith("buffer_load") and " lds" in ins.ops):
            prev = insts[max(0, i - 3):i]
            if any(p.mn in ("s_mov_b32", "s_add_i32", "s_add_u32") and p.ops.strip().startswith("m0")
                   for p in prev):
                continue
        out.append(("m0", ins, ins.addr, ["m0"]))
    return out


def check(path: str, kernel_re: str = ".", verbose: bool = False, asm: str | None = None):
    """{kernel name: [findings]} for the kernels matching kernel_re."""
    if asm is None:
        asm = disassemble_all(path)
    kernels = parse_kernels(asm, kernel_re)
    rx = re.compile(kernel_re)
    report = {}
    for name, insts in kernels.items():
        if not rx.search(name) or not insts:
            continue
        fs = analyse(insts)
        report[name] = fs
        if verbose and fs:
            by = {}
            for f in fs:
                by[f[0]] = by.get(f[0], 0) + 1
            print(f"== {name}: {by}")
            byaddr = {ins.addr: ins for ins in insts}
            for kind, ins, a, regs in fs[:12]:
                src = byaddr[a]
                print(f"   {kind}: {ins.addr:#x} {ins.mn} {ins.ops.strip()}  <- {src.mn} @ {src.addr:#x} "
                      f"{','.join(regs)}")
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--kernel", default=".")
    ap.add_argument("-v", action="store_true")
    args = ap.parse_args()
    rep = check(args.path, args.kernel, args.v)
    bad = sum(len(f) for f in rep.values())
    print(f"{len(rep)} kernels, {bad} findings")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
