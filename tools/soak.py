#!/usr/bin/env python3
"""Soak: many frames of renderLoop's calls on the full-size world, the product's launches against the
plain schedules, compared every `--check` frames -- long-run evidence that the flow launch's tagged
hand-off (epochs, the two-phase shadow, the GI window carried across calls) and the pipelined loop's
kept work never drift.  Not part of the product; its log is profiles/r06/soak_<config>.txt.

  drop-in: context A renders with the flow launch (one k_ref_flow per drawCUDA), context B with
           drawCUDA's two launches (rv_set_flow(0)); both take UpdateGIData + drawCUDA per frame.
  native:  context C runs rv_render_frame_seq on the pipelined loop in calls of --call frames,
           context D one UpdateGIData + frame at a time.
Every check compares the color / motion / depth / half-res images and the whole GI grid, bit for bit.

usage: python tools/soak.py [config c3] [frames 20000] [--check 2000] [--call 50]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="c3")
    ap.add_argument("frames", nargs="?", type=int, default=20000)
    ap.add_argument("--check", type=int, default=2000)
    ap.add_argument("--call", type=int, default=50)
    a = ap.parse_args()
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32
    cfg = CONFIGS[a.config]
    W, H, flags = cfg.width, cfg.height, rv.RV_FLAGS_REFERENCE
    atlas = load_atlas()
    kinds = (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH, rv.RV_IMAGE_HALF_DIST, rv.RV_IMAGE_HALF_SHADOW)

    def make():
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=flags, atlas=atlas)
        r.world_build()
        for s in range(max(cfg.gi_sweeps, 0)):
            r.gi_update(s)
        return r

    def same(x, y, tag, k):
        for kind in kinds:
            if not np.array_equal(x.readback(kind), y.readback(kind)):
                raise SystemExit(f"{tag}: image {kind} differs after frame {k}")
        if not np.array_equal(x.world_export(rv.RV_WORLD_GI), y.world_export(rv.RV_WORLD_GI)):
            raise SystemExit(f"{tag}: GI grid differs after frame {k}")

    pose = pose_f32(cfg, "P0")
    t0 = time.time()
    # -- drop-in: flow vs two launches
    A, B = make(), make()
    B.set_flow(0)
    done = 0
    while done < a.frames:
        n = min(a.check, a.frames - done)
        seq = camera_path(pose, W, H, n, start=done, pan=0.0005, ref_compat=True)
        for k in range(n):
            d = seq[k]
            c = d.cam
            for r in (A, B):
                r.update_gi_data()
                r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                            np.ctypeslib.as_array(d.prev_vp), 0.0, d.time)
        done += n
        same(A, B, "drop-in", done)
        active, launches, fallbacks = A.flow_info()
        print(f"drop-in {cfg.name}: {done} frames identical (flow active {active}, launches {launches}, "
              f"fallbacks {fallbacks}; {time.time() - t0:.0f} s)", flush=True)
        if fallbacks:
            raise SystemExit("a flow render wave fell back")
    A.close()
    B.close()
    # -- native: pipelined calls vs one frame at a time
    Cx, D = make(), make()
    D.set_pipeline(0)
    done = 0
    while done < a.frames:
        n = min(a.check, a.frames - done)
        seq = camera_path(pose, W, H, n, start=done, pan=0.0005, ref_compat=True)
        for s in range(0, n, a.call):
            e = min(n, s + a.call)
            Cx.render_frame_seq(seq[s:e], next_desc=seq[e], flags=flags, gi_per_frame=True)
            for d in seq[s:e]:
                D.update_gi_data()
                D.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                        jx=d.jitter_x, jy=d.jitter_y, flags=flags)
        done += n
        same(Cx, D, "native", done)
        print(f"native {cfg.name}: {done} frames identical ({time.time() - t0:.0f} s)", flush=True)
    Cx.close()
    D.close()
    print(f"SOAK OK {cfg.name} {a.frames} frames per loop, {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
