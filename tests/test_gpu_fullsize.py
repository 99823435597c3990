"""GPU parity at BASELINE.json's full sizes (C2 512^3, C3/C4
1024^3, C5 2048^3), where rebuilding the whole world on the CPU oracle is too
slow for a test.  The GPU world is exported and checked with properties and
samples the oracle can answer at any size:

* voxel bits: 200k sampled voxels against the oracle's Evaluate (> 0.7);
* CSDF: zero exactly where a coarse 2x2x2 cell holds a solid voxel, over the
  whole grid (catches any addressing error of the brick layout);
* traversal: 20k random rays traced on the GPU and by the oracle on the
  exported world, bit-exact (32-bit brick offsets up to 2 GiB of records);
* GI: a RAYPS-style partial update window, GPU vs oracle on the same grid;
* frames: sampled rows of the config's frame (its resolution and flags),
  GPU vs oracle render of the same rows on the exported world.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import random_rays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


@pytest.mark.parametrize("cfgname", ["c2", "c3", "c5"])
def test_fullsize_world_traversal_gi_frame_rows(rv, atlas, oracle, cfgname):
    from rvgrt_amd.configs import CONFIGS, pose_f32
    cfg = CONFIGS[cfgname]
    lg, n = cfg.log2_n, cfg.n
    W, H = cfg.width, cfg.height
    r = rv.StateRender((lg,) * 3, W, H, flags=cfg.flags, atlas=atlas)
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    r.sync()
    ow = oracle.OracleWorld(lg, lg, lg, atlas=atlas)
    ow.bits[:] = r.world_export(rv.RV_WORLD_BITS)
    ow.csdf[:] = r.world_export(rv.RV_WORLD_CSDF)
    ow.gi[:] = r.world_export(rv.RV_WORLD_GI)
    rng = np.random.default_rng(lg)

    # voxel bits vs Evaluate at sampled voxels
    m = 200_000
    xyz = rng.integers(0, n, size=(m, 3))
    p = np.ascontiguousarray(xyz.astype(np.float32))
    val = np.zeros(m, np.float32)
    oracle.lib().or_evaluate_batch(p.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p), m)
    idx = xyz[:, 0].astype(np.int64) | (xyz[:, 1].astype(np.int64) << lg) | (xyz[:, 2].astype(np.int64) << (2 * lg))
    got = (ow.bits[idx >> 5] >> (idx & 31).astype(np.uint32)) & 1
    assert np.array_equal(got.astype(bool), val > 0.7)

    # CSDF zero <=> coarse cell solid, whole grid (done in z slabs to bound memory)
    cs = ow.csdf.reshape(n // 2, n // 2, n // 2)
    v = ow.bits.view(np.uint8)
    slab = 64
    for z0 in range(0, n, slab):
        b = np.unpackbits(v[(z0 * n * n) // 8:((z0 + slab) * n * n) // 8], bitorder="little")
        solid = b.reshape(slab // 2, 2, n // 2, 2, n // 2, 2).any(axis=(1, 3, 5))
        assert np.array_equal(cs[z0 // 2:(z0 + slab) // 2] == 0, solid), f"z slab {z0}"

    # traversal bit-exact on the exported world
    org, dirs, dist = random_rays(rng, 20_000, (n, n, n))
    g = r.trace_rays(org, dirs, dist)
    o = ow.trace_batch(org, dirs, dist)
    assert np.array_equal(g["hit"], o["hit"]) and np.array_equal(g["undef"], o["undef"])
    assert np.array_equal(g["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(g["normal"], o["normal"])
    assert np.array_equal(g["u"], o["u"]) and np.array_equal(g["v"], o["v"])
    assert np.array_equal(g["sphere_steps"], o["n_sphere"]) and np.array_equal(g["dda_steps"], o["n_dda"])

    # GI: one RAYPS window at a rolling offset, same grid on both sides
    if cfg.gi_sweeps >= 0:
        ncell = (n // 4) ** 3
        first, count = ncell // 3, 4096
        r.gi_update(7, first=first, count=count)
        ow.gi_update(7, first=first, count=count)
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi)

    # sampled rows of the config's frame
    pos, yaw, pitch = pose_f32(cfg)
    cam, vp = rv.camera_from_pose(pos, yaw, pitch, W, H)
    r.frame(cam, vp)
    img = r.readback(rv.RV_IMAGE_COLOR)
    mv = r.readback(rv.RV_IMAGE_MOTION)
    dep = r.readback(rv.RV_IMAGE_DEPTH)
    fr = oracle.make_frame(W, H, cfg.flags, rv.camera_dict(cam, vp))
    rows = sorted(set(rng.integers(0, H, 6).tolist()) | {0, H // 2, H - 1})
    for y in rows:
        ref = oracle.render(ow, fr, y, y + 1, want_stats=False)
        assert np.array_equal(img[y], ref["rgba"][y]), f"{cfgname} row {y}"
        assert np.array_equal(mv[y], ref["mv"][y]) and np.array_equal(dep[y], ref["depth"][y])
    r.close()


@pytest.mark.parametrize("cfgname", ["c3", "c4"])
def test_fullsize_pipelined_frames(rv, atlas, cfgname):
    """The C3/C4 frame loop as bench.py runs it (pipelined launches: render
    k | GI update k+1 | pre-pass k+1) against UpdateGIData + drawCUDA one
    frame at a time on the same full-size world: colour, depth and the GI
    grid bit-identical after 6 frames (the one-at-a-time frames are checked
    against the oracle by the test above)."""
    from rvgrt_amd.configs import CONFIGS, pose_f32
    cfg = CONFIGS[cfgname]
    W, H = cfg.width, cfg.height
    cam, vp = rv.camera_from_pose(*pose_f32(cfg), W, H)
    rs = []
    for pipe in (1, 0):
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=atlas)
        r.world_build()
        for s in range(max(cfg.gi_sweeps, 0)):
            r.gi_update(s)
        r.set_pipeline(pipe)
        if pipe:
            r.render_frames(6, cam, vp, gi_per_frame=True)
        else:
            for _ in range(6):
                r.update_gi_data()
                r.frame(cam, vp)
        r.sync()
        rs.append(r)
    a, b = rs
    assert np.array_equal(a.readback(rv.RV_IMAGE_COLOR), b.readback(rv.RV_IMAGE_COLOR))
    assert np.array_equal(a.readback(rv.RV_IMAGE_DEPTH), b.readback(rv.RV_IMAGE_DEPTH))
    assert np.array_equal(a.world_export(rv.RV_WORLD_GI), b.world_export(rv.RV_WORLD_GI))
    for r in rs:
        r.close()
