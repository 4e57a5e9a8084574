#!/usr/bin/env python3
"""Per-step kernel time vs wall time from a rocprofv3 --kernel-trace CSV of bench.py: for each
training step (a k16/k32/fused fwd-bwd dispatch starts one), the sum of kernel durations, the
idle gaps between consecutive dispatches, and the largest gap with the kernels either side.

    python scripts/trace_gaps.py gpurun_out/prof/trace/run_kernel_trace.csv
"""
import csv
import sys


def short(n):
    n = n.replace("lnerf::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    starts = [i for i, k in enumerate(ks) if k[0].startswith(("k16_fwd_bwd", "k32_fwd_bwd", "fused_fwd_bwd"))]
    print(f"{'step':>4} {'wall_us':>9} {'kernels_us':>10} {'gaps_us':>8}  largest gap")
    for si in range(len(starts) - 1):
        a, b = starts[si], starts[si + 1]
        wall = (ks[b][1] - ks[a][1]) / 1e3
        kern = sum(e - s for _, s, e in ks[a:b]) / 1e3
        gaps = [(ks[i + 1][1] - ks[i][2], ks[i][0], ks[i + 1][0]) for i in range(a, b)]
        g = max(gaps)
        print(f"{si:4d} {wall:9.1f} {kern:10.1f} {wall - kern:8.1f}  {g[0] / 1e3:.1f} us {g[1]} -> {g[2]}")


if __name__ == "__main__":
    main()
