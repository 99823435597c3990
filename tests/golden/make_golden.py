#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/ from the CPU oracle.

The reference ships no tests, golden images or fixtures
and may not be executed here, so these vectors come from the oracle
(oracle/rv_oracle.c), itself cross-checked against the independent numpy
restatement (tests/np_ref.py) and analytic KATs.  They pin the oracle and
the HIP path against regressions ("parity unpinned" against CUDA itself).

    python tests/golden/make_golden.py      # writes golden.json, traces.npz, *.png
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as O                      # noqa: E402
from rvgrt_amd.atlas import load_atlas, write_png   # noqa: E402

FRAME_W, FRAME_H = 160, 96
from rvgrt_amd.configs import TEST_POSES_128 as POSES   # noqa: E402
FLAGS = {"c1": 0, "c2": O.F_SHADOW, "ref": O.F_PREPASS | O.F_WATER | O.F_GI}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    atlas = load_atlas()
    out = {"generator": "tests/golden/make_golden.py (oracle/rv_oracle.c)", "worlds": {}, "frames": {}}
    for lg, sweeps in [(6, 1), (7, 1)]:
        w = O.OracleWorld(lg, lg, lg, atlas=atlas).build(gi_sweeps=sweeps)
        gi0 = O.OracleWorld(lg, lg, lg, atlas=atlas)
        gi0.bits[:] = w.bits; gi0.csdf[:] = w.csdf
        gi0.gi_init()
        out["worlds"][f"{1 << lg}^3"] = {"bits": sha(w.bits), "csdf": sha(w.csdf), "gi_init": sha(gi0.gi),
                                         f"gi_after_{sweeps}_sweep": sha(w.gi),
                                         "solid_voxels": int(np.unpackbits(w.bits.view(np.uint8)).sum())}
        if lg == 7:
            world = w
    for pname, (pos, yaw, pitch) in POSES.items():
        cam = O.camera_from_pose(pos, yaw, pitch, FRAME_W, FRAME_H)
        for fname, flags in FLAGS.items():
            r = O.render(world, O.make_frame(FRAME_W, FRAME_H, flags, cam))
            key = f"128^3_{FRAME_W}x{FRAME_H}_{fname}_{pname}"
            out["frames"][key] = {"rgba": sha(r["rgba"]), "mv": sha(r["mv"]), "depth": sha(r["depth"]),
                                  "flags": flags, "pose": [list(pos), yaw, pitch], "stats": r["stats"]}
            write_png(os.path.join(HERE, f"{key}.png"), r["rgba"])
    rng = np.random.default_rng(2025)
    n = 256
    org = (rng.uniform(-0.2, 1.2, (n, 3)) * 128).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    dist = rng.uniform(-5, 20, n).astype(np.float32)
    h = world.trace_batch(org, d, dist)
    np.savez_compressed(os.path.join(HERE, "traces_128.npz"), org=org, dir=d, dist=dist,
                        hit=h["hit"], undef=h["undef"], pos=h["pos"], normal=h["normal"], u=h["u"], v=h["v"],
                        n_sphere=h["n_sphere"], n_dda=h["n_dda"], n_check=h["n_check"])
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", len(out["frames"]), "frames,", len(out["worlds"]), "worlds, 256 traces")


if __name__ == "__main__":
    main()
