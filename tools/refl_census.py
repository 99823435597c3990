#!/usr/bin/env python3
"""Reflection-ray step census (C4 P1's water branch): per wave, the longest reflection
ray's steps (sphere + DDA) against the sum over its lanes -- how much of the branch's issue time is lanes
waiting for the wave's longest crawl, and what a step budget with the remainder compacted into full
waves would leave.  Needs a library built with -DRV_REFL_DIAG=1 (tools/build_variant.sh refldiag
"-DRV_REFL_DIAG=1"; RVGRT_LIB=rvgrt_amd/variants/refldiag/librvgrt_hip.so).  Not part of the product.

usage: python tools/refl_census.py [config] [pose] [frames]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32

    cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
    pose = sys.argv[2] if len(sys.argv) > 2 else "P1"
    nfr = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    torch.cuda.set_device(0)
    W, H = cfg.width, cfg.height
    r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=load_atlas())
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    lib = ctypes.CDLL(os.environ["RVGRT_LIB"])
    seq = camera_path(pose_f32(cfg, pose), W, H, nfr, pan=0.0005, ref_compat=True)
    r.sync()
    lib.rv_refl_diag_dump()   # clear
    for k in range(nfr):
        d = seq[k]
        r.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                jx=d.jitter_x, jy=d.jitter_y, flags=cfg.flags | rv.RV_F_STATS)
    r.sync()
    sys.stdout.flush()
    lib.rv_refl_diag_dump()
    r.close()


if __name__ == "__main__":
    main()
