#!/usr/bin/env python3
"""Turns a scripts/gpu_sq.sh run (gpurun_out/sq/p1..p3) into profiles/<tag>_sq.json: per kernel,
the per-dispatch average of every SQ / GRBM counter, and the derived figures DESIGN.md cites.

Derived (MI355X_MICROARCH.md, "rocprofv3 PMC slots", "DVFS give-back", "LDS"):
  * busy_cycles     = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs) = the dispatch's GPU cycles
  * mfma_busy       = SQ_VALU_MFMA_BUSY_CYCLES / (busy_cycles x 1024 SIMDs) -- rocprof's MfmaUtil
                      (counter_defs.yaml: sum(MFMA_BUSY) / (max(GUI_ACTIVE) x SIMD_NUM))
  * clock_ghz       = busy_cycles / kernel duration (kernel-trace average, when a stats CSV is given)
  * mfma_flops      = SQ_INSTS_VALU_MFMA_MOPS_F16 x 512 (fp16 MFMA FLOP actually issued)
  * lds_conflict    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles / all LDS-array cycles)
  * lds_busy        = SQ_LDS_IDX_ACTIVE / (busy_cycles x 256 CUs), the LDS arrays' duty cycle
                      (units of SQ_LDS_IDX_ACTIVE assumed to be LDS cycles summed over CUs)
  * wave-cycle split = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
                      (disjoint, they add up to ~1); SQ_WAIT_INST_LDS is the LDS-issue-stall share
  * per_wave        = SQ_INSTS_* / SQ_WAVES (instruction mix of one wave)

    python scripts/summarize_sq.py r04 [gpurun_out/sq] [profiles/r04_kernel_stats.csv]
        [--workload cfg3|cfg5] [--name r04_render]
The library hash comes from <src>/lib_sha16.txt (written by scripts/gpu_sq.sh on the box).
"""
import collections
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
KEEP = ("k16_fwd_bwd_kernel", "kr_fwd_kernel", "dw16_kernel", "grad_reduce_kernel", "k1_reduce_kernel", "pack16_kernel",
        "adam_kernel", "loss_reduce_kernel")


def short(name):
    name = name.replace("lnerf::(anonymous namespace)::", "").replace("lnerf::", "")
    return name.split("(")[0].replace("void ", "").strip()


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("src", nargs="?", default=os.path.join(REPO, "gpurun_out", "sq"))
    ap.add_argument("stats_csv", nargs="?", default=None)
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--name", default=None)
    a = ap.parse_args()
    tag, src, stats_csv = a.tag, a.src, a.stats_csv
    name = a.name or tag
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)   # (kernel, dispatch, counter) -> summed over dims
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if not k.startswith(KEEP):
                continue
            per[(k, r.get("Dispatch_Id", ""), r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
    dur = {}
    if stats_csv and os.path.exists(stats_csv):
        for r in csv.DictReader(open(stats_csv)):
            dur[short(r["Name"])] = float(r["AverageNs"]) * 1e-9
    shaf = os.path.join(src, "lib_sha16.txt")
    cmdf = os.path.join(src, "command.txt")
    out = {"tag": tag, "workload": a.workload,
           "lib_sha16": open(shaf).read().strip() if os.path.exists(shaf) else None,
           "source": "scripts/gpu_sq.sh (3 rocprofv3 --pmc passes of "
                     + (open(cmdf).read().strip() if os.path.exists(cmdf) else "bench.py") + "), per-dispatch averages",
           "kernels": {}}
    for k, cs in sorted(vals.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"dispatches": max(len(v) for v in cs.values()), "counters": avg}
        der = {}
        cyc = avg.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        if cyc > 0:
            der["busy_cycles"] = cyc
            if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
                der["mfma_busy"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)
            if "SQ_LDS_IDX_ACTIVE" in avg:
                der["lds_busy"] = avg["SQ_LDS_IDX_ACTIVE"] / (cyc * 256)
            if k in dur:
                der["clock_ghz"] = cyc / dur[k] / 1e9
                der["avg_ms"] = dur[k] * 1e3
        if avg.get("SQ_LDS_IDX_ACTIVE"):
            der["lds_conflict"] = avg.get("SQ_LDS_BANK_CONFLICT", 0.0) / avg["SQ_LDS_IDX_ACTIVE"]
        if "SQ_INSTS_VALU_MFMA_MOPS_F16" in avg:
            der["mfma_f16_flops"] = avg["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in avg:
            der["mfma_bf16_flops"] = avg["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_MISC",
                      "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_FLAT", "SQ_INST_CYCLES_VMEM"):
                if c in avg:
                    der[c.lower().replace("sq_", "") + "_frac"] = avg[c] / wc
        nw = avg.get("SQ_WAVES")
        if nw:
            der["per_wave"] = {c.lower().replace("sq_insts_", ""): avg[c] / nw
                               for c in avg if c.startswith("SQ_INSTS_")}
        d["derived"] = der
        out["kernels"][k] = d
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    path = os.path.join(REPO, "profiles", f"{name}_sq.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, d in out["kernels"].items():
        der = d["derived"]
        print(f"{k:28s} mfma_busy {der.get('mfma_busy', float('nan')):.3f}  lds_busy "
              f"{der.get('lds_busy', float('nan')):.3f}  lds_conflict {der.get('lds_conflict', float('nan')):.3f}  "
              f"wait_any {der.get('wait_any_frac', float('nan')):.3f}  wait_inst {der.get('wait_inst_any_frac', float('nan')):.3f}")
    print("wrote", path)


if __name__ == "__main__":
    main()
