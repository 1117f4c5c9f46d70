#!/usr/bin/env python3
"""Per-kernel VGPR/SGPR/scratch/LDS from hipcc -save-temps assembly metadata.
Usage: python tools/kmeta.py file.s [substring]"""
import re
import sys


def kernels(path):
    text = open(path).read()
    meta = text[text.index(".amdgpu_metadata"):]
    out = []
    for blk in re.split(r"\n\s+- \.", meta):
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or ".kd" in name.group(1):
            continue
        get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1)) if re.search(rf"\.{k}:\s+(\d+)", blk) else -1
        out.append((name.group(1), get("vgpr_count"), get("sgpr_count"), get("private_segment_fixed_size"),
                    get("vgpr_spill_count")))
    return out


if __name__ == "__main__":
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for n, v, s, p, sp in kernels(sys.argv[1]):
        if sub in n:
            print(f"{v:4d} vgpr {s:4d} sgpr scratch {p:5d} spill {sp:3d}  {n}")
