#!/usr/bin/env python3
"""Turns a scripts/gpu_steps.sh trace + pmc run (gpurun_out/prof/ or rprof/) into the committed summaries under
profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied as is)
  profiles/<tag>_pmc.json           per-kernel HBM bytes per launch from the FETCH_SIZE and
                                    WRITE_SIZE passes, with the gfx950 correction of
                                    MI355X_MICROARCH.md ("HBM / rocprofv3"): FETCH_SIZE counts
                                    half the bytes of 16 B/lane streaming reads -> x2;
                                    WRITE_SIZE is exact for 16 B/lane stores. Both are in KiB.

bench.py reads <tag>_pmc.json (newest tag whose lib_sha16 is the loaded library's) to fill
roofline.traffic for the same workload. The library hash is the one the GPU step recorded next to
the traces (<src>/lib_sha16.txt, scripts/gpu_steps.sh).

    python scripts/summarize_profile.py r04 [gpurun_out/prof] [--workload cfg3|cfg5] [--name r04_render]
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def short(name):
    name = name.replace("lnerf::(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "").strip()


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("src", nargs="?", default=os.path.join(REPO, "gpurun_out", "prof"))
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--name", default=None, help="output file stem (default: the tag)")
    a = ap.parse_args()
    tag, src = a.tag, a.src
    name = a.name or tag
    dst = os.path.join(REPO, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{name}_kernel_stats.csv"))
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"))
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("k16", "kr_", "dw", "grad_reduce", "loss_reduce", "pack", "wmax16", "k1_reduce", "adam")):
            continue
        f = fetch.get(k, 0.0) * 1024
        w = write.get(k, 0.0) * 1024
        kernels[k] = {"fetch_size_kib": fetch.get(k), "write_size_kib": write.get(k),
                      "hbm_read_bytes": 2 * f, "hbm_write_bytes": w,
                      "hbm_bytes_per_launch": 2 * f + w, **stats.get(k, {})}
    cmdf = os.path.join(src, "command.txt")
    shaf = os.path.join(src, "lib_sha16.txt")
    out = {"tag": tag, "command": open(cmdf).read().strip() if os.path.exists(cmdf) else None,
           "workload": a.workload, "lib_sha16": open(shaf).read().strip() if os.path.exists(shaf) else None,
           "correction": "hbm_read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE",
           "kernels": kernels}
    with open(os.path.join(dst, f"{name}_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:32s} {v.get('avg_ms', 0):8.3f} ms  read {v['hbm_read_bytes'] / 1e9:7.3f} GB  "
              f"write {v['hbm_write_bytes'] / 1e9:7.3f} GB")


if __name__ == "__main__":
    main()
