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
                       "1024^3 world, 3840x2160, 2-bounce GI, screen-tile split (RCCL gather)"),
    "c5": RenderConfig("c5", 11, 3840, 2160, FLAGS_REFERENCE, 2, True, 8,
                       "2048^3 world, 3840x2160, 2-bounce GI + reflections, tile-parallel"),
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
