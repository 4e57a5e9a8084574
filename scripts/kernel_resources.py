#!/usr/bin/env python3
"""Per-kernel register, spill, scratch and LDS figures of an in-tree library, from the code
object's metadata notes (llvm-readelf --notes).  python scripts/kernel_resources.py [LIB] [REGEX]"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def resources(lib, rx="."):
    import isa_check
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for co in isa_check.extract_code_objects(lib, d):
            txt = subprocess.run([f"{isa_check.LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                                 text=True, check=True).stdout
            for blk in re.split(r"\n\s+- \.", txt):
                m = re.search(r"\.name:\s+(\S+)", blk)
                if not m or not re.search(rx, m.group(1)) or m.group(1).endswith(".kd"):
                    continue
                f = {}
                for key in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                            "private_segment_fixed_size", "group_segment_fixed_size"):
                    mm = re.search(r"\." + key + r":\s+(\d+)", blk)
                    if mm:
                        f[key] = int(mm.group(1))
                out[m.group(1)] = f
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(HERE), "loma-nerf_amd", "lib",
                                                             "libloma_nerf.so")
    rx = sys.argv[2] if len(sys.argv) > 2 else "."
    for k, f in resources(lib, rx).items():
        print(f"{k[:70]:70s} " + " ".join(f"{a.replace('_count', '').replace('_segment_fixed_size', '')}={b}"
                                           for a, b in f.items()))
