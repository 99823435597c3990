#!/usr/bin/env python3
"""Per-stage traversal step counts of one reference frame (RV_F_STATS census): where the sphere /
DDA / check steps go (pre-pass, render, GI update), and the world's highest solid row (the sky
exit's bound).  Diagnostics for DESIGN.md s5; not part of the product.

    python tools/step_census.py [c3 c4 c5] [--pose P0]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, pose_f32
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    pose = sys.argv[sys.argv.index("--pose") + 1] if "--pose" in sys.argv else "P0"
    args = [a for a in args if a != pose]
    for name in args or ["c4"]:
        cfg = CONFIGS[name]
        W, H = cfg.width, cfg.height
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=load_atlas())
        r.world_build()
        for s in range(max(cfg.gi_sweeps, 0)):
            r.gi_update(s)
        bits = r.world_export(rv.RV_WORLD_BITS).reshape(cfg.n, cfg.n, cfg.n // 32)   # [z, y, x words]
        rows = np.flatnonzero(bits.any(axis=(0, 2)))
        cam, vp = rv.camera_from_pose(*pose_f32(cfg, pose), W, H)
        r.stats_reset()
        r.frame(cam, vp, flags=cfg.flags | rv.RV_F_STATS)
        r.set_gi_stats(1)
        r.update_gi_data()
        r.sync()
        print(f"{name} {pose}: highest solid row {rows.max() if len(rows) else -1} (camera y {pose_f32(cfg, pose)[0][1]})")
        for k, st in enumerate(rv._lib.STAGES):
            s = r.stats(k)
            if s["traces"] or s.get("gi_traces"):
                print(f"  {st:11s} traces {s['traces']:>10d} gi {s.get('gi_traces', 0):>8d} sphere {s['sphere_steps']:>11d} "
                      f"dda {s['dda_steps']:>11d} check {s['csdf_checks']:>9d} cone_steps {s['cone_steps']:>10d}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
