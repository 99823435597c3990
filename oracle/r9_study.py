"""R9 sensitivity study: how far the reference's compiled arithmetic can sit
from the no-contraction oracle (SURVEY.md Appendix R9, s8c tolerance).

TEST INFRASTRUCTURE ONLY (imported by tests/test_r9_numerics.py and
tools/r9_report.py; never by the product).

The reference is built by nvcc with its default --fmad=true
(/root/reference/CMakeLists.txt:59-62), so ptxas fuses the a*b+c of e.g.
`pos + dir*dist` (src/raytracing_functions.cu:79), the CSDF jump
`posOnRay + camDir*(dist*2)` (:137), the hit position
`currentPos + (tMax-delta)*camDir` (:155,160,164), the cone sample
`pos + dir*currentDist` (:229) and every dot/normalize into FFMAs, and its
tanf (:236) and powf (src/StateRender.cu:85,142) are CUDA's <= 2-ulp
versions.  The oracle and the HIP product are both uncontracted and use the
correctly rounded tan constant.  This module renders the same configuration
with study builds of the oracle (oracle/Makefile: gcc -ffp-contract=fast and
clang -ffp-contract=on, both with hardware FMA) and with tanf/powf moved by
whole ulps, and measures the divergence from the plain oracle:

* world: voxels of the bitfield that flip (the noise's 0.7 threshold),
* primary rays: hit/miss agreement and hit-voxel agreement (all rays, and
  non-grazing rays: |cos(dir, normal)| >= GRAZING_COS),
* RGBA8: the per-pixel max |delta| histogram, exact / <= 2 LSB fractions.

`end_to_end` variants build their own world and GI grid with the study
arithmetic too (everything the reference computes on the device is
contracted); `render_only` variants render on the plain oracle's world.
"""
from __future__ import annotations

import numpy as np

from . import oracle as O

GRAZING_COS = 0.1          # rays within ~5.7 deg of the surface plane count as grazing

# (name, build, tan_ulp, pow_ulp, end_to_end)
VARIANTS = [
    ("fma_gcc", "fma_gcc", 0, 0, True),
    ("fma_clang", "fma_clang", 0, 0, True),
    ("fma_gcc_render_only", "fma_gcc", 0, 0, False),
    ("tan+2", "plain", 2, 0, False),
    ("tan-2", "plain", -2, 0, False),
    ("pow+2", "plain", 0, 2, False),
    ("pow-2", "plain", 0, -2, False),
    ("fma_gcc_tan+2_pow+2", "fma_gcc", 2, 2, True),
    ("fma_gcc_tan-2_pow-2", "fma_gcc", -2, -2, True),
]


def build_world(build, lg, sweeps, atlas):
    with O.numerics(build):
        return O.OracleWorld(lg, lg, lg, atlas=atlas).build(gi_sweeps=sweeps)


def render(world, build, tan_ulp, pow_ulp, W, H, flags, cam):
    with O.numerics(build, tan_ulp, pow_ulp):
        fr = O.make_frame(W, H, flags, cam)
        r = O.render(world, fr)
        r["hits"] = O.primary_hits(world, fr, halfdist=r["halfdist"] if flags & O.F_PREPASS else None)
    return r


def pixel_dirs(cam, W, H):
    """Camera ray directions of the full-res pixels (src/StateRender.cu:44-45),
    in float64: only used to classify grazing rays."""
    x = np.arange(W, dtype=np.float64) / W
    y = np.arange(H, dtype=np.float64) / H
    nx, ny = np.meshgrid(x * 2 - 1, y * 2 - 1)
    d = (np.asarray(cam["fo"], np.float64)[None, None] + nx[..., None] * np.asarray(cam["ri"], np.float64)
         + ny[..., None] * np.asarray(cam["up"], np.float64))
    return d / np.linalg.norm(d, axis=-1, keepdims=True)


def hit_voxel(h):
    """The solid voxel a primary hit stopped in: the hit lies on the face whose
    outward normal is `normal`, so the voxel is half a voxel behind it."""
    return np.floor(h["pos"].astype(np.float64) - 0.5 * h["normal"].astype(np.float64)).astype(np.int64)


def compare(ref, var, dirs):
    a, b = ref["rgba"].astype(np.int32), var["rgba"].astype(np.int32)
    d = np.abs(a - b).max(axis=2)
    n = d.size
    hist = {str(k): int((d == k).sum()) for k in range(0, 4)}
    hist[">=4"] = int((d >= 4).sum())
    ha, hb = ref["hits"], var["hits"]
    hit_agree = float((ha["hit"] == hb["hit"]).mean())
    both = (ha["hit"] == 1) & (hb["hit"] == 1) & (ha["undef"] == 0) & (hb["undef"] == 0)
    same_vox = np.all(hit_voxel(ha) == hit_voxel(hb), axis=-1)
    cosn = np.abs((dirs * ha["normal"].astype(np.float64)).sum(-1))
    ng = both & (cosn >= GRAZING_COS)
    return {
        "pixels": n,
        "rgba_exact": float((d == 0).mean()),
        "rgba_le2": float((d <= 2).mean()),
        "rgba_max": int(d.max()),
        "rgba_hist": hist,
        "hit_agree": hit_agree,
        "hit_voxel_agree": float(same_vox[both].mean()) if both.any() else 1.0,
        "hit_voxel_agree_nongrazing": float(same_vox[ng].mean()) if ng.any() else 1.0,
        "hits": int(both.sum()),
        "nongrazing_hits": int(ng.sum()),
        "mv_exact": float(np.all(ref["mv"] == var["mv"], axis=-1).mean()),
        "depth_exact": float((ref["depth"] == var["depth"]).mean()),
    }


def world_diff(wa, wb):
    ba = np.unpackbits(wa.bits.view(np.uint8))
    bb = np.unpackbits(wb.bits.view(np.uint8))
    return {"voxels": int(ba.size), "voxels_flipped": int((ba != bb).sum()),
            "csdf_cells_diff": int((wa.csdf != wb.csdf).sum()),
            "gi_cells_diff": int((wa.gi.reshape(-1, 4) != wb.gi.reshape(-1, 4)).any(axis=1).sum())}


def tolerance_ok(m):
    """RGBA8 |d| <= 2 LSB on >= 99.5 % of pixels, hit/miss
    agreement >= 99.9 %, hit-voxel agreement >= 99.5 % on non-grazing rays."""
    return m["rgba_le2"] >= 0.995 and m["hit_agree"] >= 0.999 and m["hit_voxel_agree_nongrazing"] >= 0.995


def study(lg, sweeps, W, H, flags, pose, atlas, variants=VARIANTS):
    """Runs every variant on one configuration; returns (world diffs, metrics)."""
    pos, yaw, pitch = pose
    cam = O.camera_from_pose(pos, yaw, pitch, W, H)
    base_world = build_world("plain", lg, sweeps, atlas)
    ref = render(base_world, "plain", 0, 0, W, H, flags, cam)
    dirs = pixel_dirs(cam, W, H)
    worlds, out = {}, {}
    for name, build, tu, pu, e2e in variants:
        if e2e:
            if build not in worlds:
                worlds[build] = build_world(build, lg, sweeps, atlas)
            w = worlds[build]
        else:
            w = base_world
        out[name] = compare(ref, render(w, build, tu, pu, W, H, flags, cam), dirs)
    wd = {b: world_diff(base_world, w) for b, w in worlds.items()}
    return wd, out


def gi_cells_diff(wa, wb):
    return int((wa.gi.reshape(-1, 4) != wb.gi.reshape(-1, 4)).any(axis=1).sum())


def long_gi_sequence(lg, sweeps, frames, W, H, flags, pose, atlas, builds=("fma_gcc", "fma_clang"),
                     render_at=None, rays=262144):
    """The GI feedback loop under the reference's arithmetic: the reference
    runs UpdateGIData before every drawCUDA, forever (src/main.cpp:119-132),
    and every update reads the grid the previous ones wrote -- the bounce hit's
    GI texel and the cell's own old value (src/CoarseArray.cu:315-354) -- so a
    cell that a contracted build computes differently can spread.  Each build
    (plain, and the contraction emulations) builds its own world and runs
    `frames` rolling RAYPS windows (frame numbers 0.., the offset of
    src/CoarseArray.cu:392-394) on it; after every update the GI cells that
    differ from the plain build's grid are counted, and at the frames in
    `render_at` (default: the last) each build renders the same camera on its
    own grid and is compared with the plain render (compare()).  Returns one
    record per frame."""
    pos, yaw, pitch = pose
    cam = O.camera_from_pose(pos, yaw, pitch, W, H)
    worlds = {"plain": build_world("plain", lg, sweeps, atlas)}
    for b in builds:
        worlds[b] = build_world(b, lg, sweeps, atlas)
    n = len(worlds["plain"].gi) // 4
    render_at = set(render_at) if render_at else {frames}
    dirs = pixel_dirs(cam, W, H)
    off, curve = 0, []
    for k in range(1, frames + 1):
        cnt = min(rays, n - off)
        for b, w in worlds.items():
            with O.numerics(b):
                w.gi_update(k - 1, first=off, count=cnt)
        off = 0 if off + rays >= n else off + rays
        rec = {"frame": k, "gi_cells": n, "gi_cells_diff": {b: gi_cells_diff(worlds["plain"], worlds[b]) for b in builds}}
        if k in render_at:
            ref = render(worlds["plain"], "plain", 0, 0, W, H, flags, cam)
            rec["render"] = {b: compare(ref, render(worlds[b], b, 0, 0, W, H, flags, cam), dirs) for b in builds}
        curve.append(rec)
    return curve
