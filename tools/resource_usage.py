#!/usr/bin/env python3
"""Compact per-kernel register/occupancy table of the gfx950 build.

    python tools/resource_usage.py [extra hipcc -D flags ...]

Compiles rv_kernels.hip and rv_wavefront.hip with -Rpass-analysis=
kernel-resource-usage (same flags as rvgrt_amd/csrc/Makefile) and prints one
line per kernel: VGPRs, SGPRs, occupancy (waves/SIMD), LDS bytes, scratch.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rvgrt_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
         "-fno-slp-vectorize", "-c", "-x", "hip", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    extra = sys.argv[1:]
    rows = []
    for src in ("rv_kernels.hip", "rv_wavefront.hip"):
        p = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, src], cwd=CSRC, capture_output=True, text=True)
        cur = None
        for line in p.stderr.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1)}
                rows.append(cur)
                continue
            for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                             ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                             ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)")):
                m = re.search(pat, line)
                if m and cur is not None:
                    cur[key] = int(m.group(1))
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*", "", n).replace("rv::", "")
        print(f"{n:60s} vgpr {r.get('vgpr', '?'):>3} sgpr {r.get('sgpr', '?'):>3} occ {r.get('occ', '?')} "
              f"lds {r.get('lds', 0):>5} scratch {r.get('scratch', 0)}")


if __name__ == "__main__":
    main()
