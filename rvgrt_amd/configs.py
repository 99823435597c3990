"""Benchmark / parity configurations C1-C5 (BASELINE.json `configs`,
SURVEY.md s8d).  World N^3, reference Evaluate with seed offset 0, cameras
from the reference defaults (src/Character.cpp:30,45-46)."""
from __future__ import annotations

import math
from dataclasses import dataclass

from ._lib import RV_F_GI, RV_F_PREPASS, RV_F_SHADOW, RV_F_WATER

FLAGS_PRIMARY = 0                                   # C1: primary rays, textured, no shadow/GI
FLAGS_SHADOW = RV_F_SHADOW                          # C2: primary + 1 sun-shadow ray per pixel
FLAGS_REFERENCE = RV_F_PREPASS | RV_F_WATER | RV_F_GI   # C3-C5: the reference frame


@dataclass(frozen=True)
class RenderConfig:
    name: str
    log2_n: int
    width: int
    height: int
    flags: int
    gi_sweeps: int          # deterministic full GI sweeps after GI init (-1: no GI grid needed)
    gi_per_frame: bool      # run UpdateGIData (RAYPS cells) every frame, as renderLoop does
    n_gpus: int
    describe: str

    @property
    def n(self):
        return 1 << self.log2_n

    def pose(self, which="P0"):
        """Camera pose P0 (reference defaults) or P1 (water/reflection heavy)."""
        n = self.n
        if which == "P0":
            return (0.1 * n, min(0.6 * n, 350.0), 0.1 * n), -0.7, -math.pi - 0.3
        return (0.1 * n, 60.0, 0.1 * n), -0.7, -math.pi - 0.6


CONFIGS = {
    "c1": RenderConfig("c1", 8, 640, 360, FLAGS_PRIMARY, -1, False, 0,
                       "256^3 world, 640x360, primary rays only, 1 spp (CPU scalar DDA case)"),
    "c2": RenderConfig("c2", 9, 1920, 1080, FLAGS_SHADOW, -1, False, 1,
                       "512^3 world, 1920x1080, primary + 1 shadow ray"),
    "c3": RenderConfig("c3", 10, 1920, 1080, FLAGS_REFERENCE, 1, True, 1,
                       "1024^3 world, 1920x1080, 1-bounce reflection + voxel-cone GI"),
    "c4": RenderConfig("c4", 10, 3840, 2160, FLAGS_REFERENCE, 2, True, 4,
                       "1024^3 world, 3840x2160, 2-bounce GI"),
    "c5": RenderConfig("c5", 11, 3840, 2160, FLAGS_REFERENCE, 2, True, 8,
                       "2048^3 world, 3840x2160, 2-bounce GI + reflections"),
}

# Poses for the small (128^3) parity worlds: the C1-C5 pose rule puts the
# camera inside the mountains at the world's low-x/low-z corner there, so the
# small-world tests look back at them from the open water side instead.
TEST_POSES_128 = {
    "P0": ((110.0, 70.0, 120.0), 2.44, -3.4415927),   # mountains, water, sky
    "P1": ((64.0, 45.0, 120.0), 3.14, -3.2),          # water/reflection heavy
}


# float32 yaw/pitch exactly as the reference stores them (float members)
def pose_f32(cfg: RenderConfig, which="P0"):
    import numpy as np
    pos, yaw, pitch = cfg.pose(which)
    return (tuple(float(np.float32(v)) for v in pos), float(np.float32(yaw)), float(np.float32(pitch)))


# src/Character.cpp:9-15: the TAA jitter table; Character::Update uses
# entry frameCount % 8, scaled by 0.5 (:101-102).
JITTER_SEQUENCE = ((-1 / 8, -1 / 8), (1 / 8, 3 / 8), (5 / 8, -3 / 8), (-3 / 8, 5 / 8),
                   (-7 / 8, -5 / 8), (3 / 8, 7 / 8), (7 / 8, -7 / 8), (-5 / 8, 1 / 8))


def camera_path(pose, width, height, frames, start=0, pan=0.0005, ref_compat=True):
    """The per-frame inputs renderLoop hands drawCUDA (src/main.cpp:119-132)
    for a camera panning `pan` rad of yaw per frame from `pose` ((pos, yaw,
    pitch) as RenderConfig.pose returns it): frame f's camera and unjittered
    VP from Character::Update, the previous frame's VP, and the jitter
    sequence -- with ref_compat, time and jitter mapped as drawCUDA maps them
    (time <- jitterY, jitter <- (0, 0)), or applied as
    ray jitter without.  Only time and jitter are mapped here: the other
    ref_compat quirk, minDist's normalized-coordinate texel fetch, is the frame
    flag RV_F_REF_FETCH, which rv_draw_cuda adds on a ref_compat context and
    a caller of rv_render_frame_seq / rv_frame passes in `flags` when it wants
    it (the bench renders the exact texel fetch).
    Returns frames + 1 rv_frame_desc: frames start..start+frames-1 and the
    one after them (rv_render_frame_seq's `next`)."""
    import numpy as np
    from .render import camera_from_pose, frame_desc
    pos, yaw, pitch = pose

    def cam(f):
        y = float(np.float32(np.float32(yaw) + np.float32(pan) * np.float32(f)))
        return camera_from_pose(pos, y, float(np.float32(pitch)), width, height)

    out = []
    _, prev = cam(start - 1)
    for f in range(start, start + frames + 1):
        c, vp = cam(f)
        jx, jy = (float(np.float32(v * 0.5)) for v in JITTER_SEQUENCE[f % 8])
        if ref_compat:
            out.append(frame_desc(c, vp, prev, time=jy, jx=0.0, jy=0.0))
        else:
            out.append(frame_desc(c, vp, prev, time=0.0, jx=jx, jy=jy))
        prev = vp
    return out
