#!/usr/bin/env python3
"""How much of the render's water branch runs in mixed waves.

computeColor's water branch (src/StateRender.cu:53-87: fBm normal, reflection
ray, reflection shadow ray) runs for the water lanes of a wave while its land
and sky lanes idle, then the land branch (texture, cones) with the water lanes
idle.  Compacting water pixels into full waves only saves the water-branch
passes of MIXED 8x8 waves.  This tool counts them on the real frames: the
world is built on the GPU and exported, the primary hits come from the CPU
oracle (oracle/rv_oracle.c, test infrastructure used here as an analysis
tool), and every 8x8 tile is classified.

    python tools/water_waves.py [c3 c4 ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import rvgrt_amd as rv
    from oracle import oracle as O
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, pose_f32
    O.set_threads(min(16, os.cpu_count() or 1))
    atlas = load_atlas()
    for name in sys.argv[1:] or ["c3", "c4"]:
        cfg = CONFIGS[name]
        W, H = cfg.width, cfg.height
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=atlas)
        r.world_build()
        r.sync()
        w = O.OracleWorld(cfg.log2_n, cfg.log2_n, cfg.log2_n, atlas=atlas)
        w.bits[:] = r.world_export(rv.RV_WORLD_BITS)
        w.csdf[:] = r.world_export(rv.RV_WORLD_CSDF)
        r.close()
        for pose in ("P0", "P1"):
            pos, yaw, pitch = pose_f32(cfg, pose)
            cam, vp = rv.camera_from_pose(pos, yaw, pitch, W, H)
            fr = O.make_frame(W, H, 0, rv.camera_dict(cam, vp))
            h = O.primary_hits(w, fr)
            hit = h["hit"] != 0
            water = hit & (h["pos"][..., 1] < 31.001)
            land = hit & ~water
            Ht, Wt = H // 8, W // 8
            t = lambda a: a[:Ht * 8, :Wt * 8].reshape(Ht, 8, Wt, 8).sum(axis=(1, 3))
            nw, nl = t(water), t(land)
            ns = 64 - nw - nl
            allw = int(((nw == 64)).sum())
            mixed = (nw > 0) & (nw < 64)
            nmixed = int(mixed.sum())
            wl_mixed = int(nw[mixed].sum())
            passes = allw + nmixed
            compact = allw + -(-wl_mixed // 64)
            print(f"{name} {pose}: water {water.mean():.4f} land {land.mean():.4f} sky {1 - hit.mean():.4f} of pixels;"
                  f" tiles {Ht * Wt}: all-water {allw}, mixed {nmixed} (with land {int((mixed & (nl > 0)).sum())},"
                  f" sky-only partner {int((mixed & (nl == 0)).sum())}), water lanes in mixed tiles {wl_mixed}"
                  f" (mean {wl_mixed / max(nmixed, 1):.1f}/64); water-branch wave passes {passes} -> {compact}"
                  f" compacted ({1 - compact / max(passes, 1):.3f} saved); land-branch passes skipped by all-water"
                  f" tiles only", flush=True)


if __name__ == "__main__":
    main()
