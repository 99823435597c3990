#!/usr/bin/env python3
"""Whole-grid world fixtures at BASELINE.json's full sizes, from the CPU oracle.

For every world the benchmark configurations render (C2 512^3, C3/C4 1024^3,
C5 2048^3) and the reference's native 4096 x 512 x 4096 world, the oracle
builds the world from scratch -- voxel bits from Evaluate (src/CArray.cu:8-30),
the 3-pass CSDF (src/CoarseArray.cu:37-152), GI init (:211-245) and the GI
updates the configurations render with (:273-355, deterministic per Appendix
R5) -- and this script records the sha256 of each grid in the reference
layouts, whole and per z-slab (16 contiguous slabs: z is the slowest axis of
every grid, so a failing slab names where the grids part).

    python tests/golden/make_world_hashes.py [name ...]   # -> world_hashes.json

Names: c2 (512^3), c4 (1024^3: C3 renders after sweep 1, C4 after sweep 2),
c5 (2048^3), native (4096x512x4096, GI after the first UpdateGIData window).
The 2048^3 and native builds take ~15 min each on 8 host threads (Evaluate on
8 G voxels).  The GPU suite compares the HIP build's exported grids with these
hashes (tests/test_gpu_world_full.py); the oracle build itself is pinned by the
small-world golden fixtures (tests/golden/golden.json, tests/test_golden.py).
Like every fixture here, it pins the restated semantics ("parity unpinned"
against CUDA itself).
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O                      # noqa: E402
from rvgrt_amd.atlas import load_atlas              # noqa: E402

OUT = os.path.join(HERE, "world_hashes.json")
NSLAB = 16
RAYPS = 262144          # src/CoarseArray.cu:376-395 (cells per UpdateGIData)

# name -> (log2 dims, GI stages after init: list of (label, frame, first, count or None = all cells))
WORLDS = {
    "c2": ((9, 9, 9), [("gi_sweep1", 0, 0, None)]),
    "c4": ((10, 10, 10), [("gi_sweep1", 0, 0, None), ("gi_sweep2", 1, 0, None)]),
    "c5": ((11, 11, 11), [("gi_sweep1", 0, 0, None), ("gi_sweep2", 1, 0, None)]),
    "native": ((12, 9, 12), [("gi_window0", 0, 0, RAYPS)]),
}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def grid_hashes(a: np.ndarray) -> dict:
    """Whole-array sha256 and NSLAB contiguous z-slab sha256s (z slowest)."""
    return {"sha256": sha(a), "slabs": [sha(s) for s in np.split(a.reshape(-1), NSLAB)], "bytes": int(a.nbytes)}


def build(name: str, atlas) -> dict:
    log2, stages = WORLDS[name]
    w = O.OracleWorld(*log2, atlas=atlas)
    rec = {"log2": list(log2), "nslab": NSLAB, "timing_s": {}}
    t = time.time(); w.fill(); rec["timing_s"]["fill"] = round(time.time() - t, 1)
    rec["bits"] = grid_hashes(w.bits)
    rec["solid_voxels"] = int(np.unpackbits(w.bits.view(np.uint8)).sum(dtype=np.int64))
    print(name, "fill", rec["timing_s"]["fill"], flush=True)
    t = time.time(); w.build_csdf(); rec["timing_s"]["csdf"] = round(time.time() - t, 1)
    rec["csdf"] = grid_hashes(w.csdf)
    rec["csdf_saturated_frac"] = float((w.csdf == 64).mean())
    print(name, "csdf", rec["timing_s"]["csdf"], flush=True)
    t = time.time(); w.gi_init(); rec["timing_s"]["gi_init"] = round(time.time() - t, 1)
    rec["gi_init"] = grid_hashes(w.gi)
    for label, frame, first, count in stages:
        t = time.time(); w.gi_update(frame, first=first, count=count)
        rec["timing_s"][label] = round(time.time() - t, 1)
        rec[label] = grid_hashes(w.gi)
        rec[label]["update"] = {"frame": frame, "first": first, "count": count}
        print(name, label, rec["timing_s"][label], flush=True)
    return rec


def main(names):
    atlas = load_atlas()
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    out["generator"] = "tests/golden/make_world_hashes.py (oracle/rv_oracle.c)"
    out.setdefault("worlds", {})
    out["threads"] = O.get_threads()
    for name in names:
        out["worlds"][name] = build(name, atlas)
        with open(OUT, "w") as f:                      # keep finished worlds if a later one is interrupted
            json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", OUT, sorted(out["worlds"]))


if __name__ == "__main__":
    main(sys.argv[1:] or list(WORLDS))
