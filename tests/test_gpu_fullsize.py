"""GPU parity at BASELINE.json's full sizes and at the reference's own native
configuration (C1 256^3 @ 640x360, C2 512^3 @ 1080p, C3 1024^3 @
1080p, C4 1024^3 @ 2160p with 2 GI sweeps, C5 2048^3 @ 2160p; the reference's
4096 x 512 x 4096 world at 1280 x 800 through drawCUDA with ref_compat,
include/cumath.cuh:19-31, include/State.hpp:28-29).

C1 is small enough for the oracle to build the whole world and render the
whole frame.  Above it, where an oracle world build is too slow for a test,
the GPU world is exported and checked with what the oracle answers at any
size:

* the whole world first: bits, CSDF and the GI grid the config renders with
  hash equal to the oracle's own whole-grid build (tests/world_golden.py,
  tests/test_gpu_full_world.py), so the oracle never renders on a world it
  did not compute itself;
* voxel bits: 200k sampled voxels against the oracle's Evaluate (> 0.7);
* CSDF: zero exactly where a coarse 2x2x2 cell holds a solid voxel, over the
  whole grid (catches any addressing error of the brick layout);
* traversal: 20k random rays traced on the GPU and by the oracle on the
  exported world, bit-exact (32-bit brick offsets up to 2 GiB of records);
* GI: a RAYPS-style partial update window, GPU vs oracle on the same grid;
* frames: the config's whole frame (its resolution, flags and pose), GPU vs
  oracle render on the exported world (RGBA8, MV and depth of every pixel;
  the oracle renders a 4K reference frame in about a second on the box's
  host threads).
"""
import ctypes as C

import numpy as np
import pytest

import world_golden as WG
from conftest import random_rays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def coarse_solid(bits, dims, z0, z1):
    """Coarse 2x2x2 cells of voxel slices [z0, z1) holding a solid voxel, from
    the canonical bit words (x fastest, little bit order), as bool (z, y, x)."""
    X, Y, Z = dims
    v = bits.view(np.uint8).reshape(Z, Y, X // 8)[z0:z1]
    v = np.bitwise_or.reduce(v.reshape(-1, 2, Y, X // 8), axis=1)
    v = np.bitwise_or.reduce(v.reshape(v.shape[0], Y // 2, 2, X // 8), axis=2)
    v = v | (v >> 1)                                       # x pairs inside a byte -> even bits
    b = np.unpackbits(v, axis=-1, bitorder="little").reshape(v.shape[0], Y // 2, X // 8, 8)[..., ::2]
    return b.reshape(v.shape[0], Y // 2, X // 2).astype(bool)


def check_world_rays_gi(r, rv, oracle, atlas, log2, seed, golden, gi_window=True, stage=None):
    """The exported GPU world against the oracle's answers; returns the oracle
    world holding it.  golden: the config (or world fixture) whose whole-grid
    oracle hashes the world must match first."""
    WG.assert_world(r, rv, golden, stage=stage)
    lx, ly, lz = log2
    X, Y, Z = 1 << lx, 1 << ly, 1 << lz
    ow = oracle.OracleWorld(lx, ly, lz, atlas=atlas)
    ow.bits[:] = r.world_export(rv.RV_WORLD_BITS)
    ow.csdf[:] = r.world_export(rv.RV_WORLD_CSDF)
    ow.gi[:] = r.world_export(rv.RV_WORLD_GI)
    rng = np.random.default_rng(seed)

    # voxel bits vs Evaluate at sampled voxels
    m = 200_000
    xyz = rng.integers(0, [X, Y, Z], size=(m, 3))
    p = np.ascontiguousarray(xyz.astype(np.float32))
    val = np.zeros(m, np.float32)
    oracle.lib().or_evaluate_batch(p.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p), m)
    idx = xyz[:, 0].astype(np.int64) | (xyz[:, 1].astype(np.int64) << lx) | (xyz[:, 2].astype(np.int64) << (lx + ly))
    got = (ow.bits[idx >> 5] >> (idx & 31).astype(np.uint32)) & 1
    assert np.array_equal(got.astype(bool), val > 0.7)

    # CSDF zero <=> coarse cell solid, whole grid, in z slabs
    cs = ow.csdf.reshape(Z // 2, Y // 2, X // 2)
    slab = 64
    for z0 in range(0, Z, slab):
        assert np.array_equal(cs[z0 // 2:(z0 + slab) // 2] == 0, coarse_solid(ow.bits, (X, Y, Z), z0, z0 + slab)), \
            f"z slab {z0}"

    # traversal bit-exact on the exported world
    org, dirs, dist = random_rays(rng, 20_000, (X, Y, Z))
    g = r.trace_rays(org, dirs, dist)
    o = ow.trace_batch(org, dirs, dist)
    assert np.array_equal(g["hit"], o["hit"]) and np.array_equal(g["undef"], o["undef"])
    assert np.array_equal(g["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(g["normal"], o["normal"])
    assert np.array_equal(g["u"], o["u"]) and np.array_equal(g["v"], o["v"])
    assert np.array_equal(g["sphere_steps"], o["n_sphere"]) and np.array_equal(g["dda_steps"], o["n_dda"])

    # GI: one RAYPS window at a rolling offset, same grid on both sides
    if gi_window:
        ncell = (X // 4) * (Y // 4) * (Z // 4)
        first, count = ncell // 3, 4096
        r.gi_update(7, first=first, count=count)
        ow.gi_update(7, first=first, count=count)
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi)
    return ow


def spread_rows(H, n, rng):
    """n rows spread evenly over the frame (jittered inside their bands), plus
    the first, middle and last rows."""
    band = H / n
    rows = (np.arange(n) * band + rng.uniform(0, band, n)).astype(int)
    return sorted(set(np.clip(rows, 0, H - 1).tolist()) | {0, H // 2, H - 1})


def check_rows(r, rv, oracle, ow, W, H, flags, cam_d, rng, time=0.0, nrows=64, pvp=None):
    """Rows of the GPU frame (nrows spread rows; None: every row) against the oracle: RGBA8, MV and depth
    bit-exact (the HIP path computes the oracle's arithmetic: no contraction,
    correctly rounded division/sqrt; ocml's powf has matched glibc's on every
    pixel so far).  The tolerance of SURVEY s8c is for the reference's own
    compiled arithmetic, priced separately (tests/test_r9_numerics.py)."""
    img = r.readback(rv.RV_IMAGE_COLOR)
    mv = r.readback(rv.RV_IMAGE_MOTION)
    dep = r.readback(rv.RV_IMAGE_DEPTH)
    fr = oracle.make_frame(W, H, flags, cam_d, time=time, pvp=pvp)
    rows = list(range(H)) if nrows is None else spread_rows(H, nrows, rng)
    ref = oracle.render_rows(ow, fr, rows, want_stats=False)
    d = np.abs(img[rows].astype(np.int32) - ref["rgba"][rows].astype(np.int32)).max(axis=-1)
    print(f"{len(rows)} rows: {int((d > 0).sum())} of {d.size} pixels differ, max |d| {int(d.max())}")
    assert d.max() == 0
    assert np.array_equal(mv[rows], ref["mv"][rows]) and np.array_equal(dep[rows], ref["depth"][rows])
    return rows, ref


def test_c1_full_world_full_frame(rv, atlas, oracle):
    """C1 (BASELINE configs[0]: 256^3, 640x360, primary rays only) at its
    size: the oracle builds the whole world and renders the whole frame."""
    from rvgrt_amd.configs import CONFIGS, pose_f32
    cfg = CONFIGS["c1"]
    lg, W, H = cfg.log2_n, cfg.width, cfg.height
    ow = oracle.OracleWorld(lg, lg, lg, atlas=atlas).build(gi_sweeps=0)
    r = rv.StateRender((lg,) * 3, W, H, flags=cfg.flags, atlas=atlas)
    r.world_build()
    assert np.array_equal(r.world_export(rv.RV_WORLD_BITS), ow.bits)
    assert np.array_equal(r.world_export(rv.RV_WORLD_CSDF), ow.csdf)
    assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi)
    for pose in ("P0", "P1"):
        cam, vp = rv.camera_from_pose(*pose_f32(cfg, pose), W, H)
        r.stats_reset()
        r.frame(cam, vp, flags=cfg.flags | rv.RV_F_STATS)
        img = r.readback(rv.RV_IMAGE_COLOR)
        ref = oracle.render(ow, oracle.make_frame(W, H, cfg.flags, rv.camera_dict(cam, vp)))
        assert np.array_equal(img, ref["rgba"]), pose
        assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref["mv"])
        assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref["depth"])
        st = r.stats()
        for k in ("traces", "primary", "tex_samples", "undef_hits"):
            assert st[k] == ref["stats"][k], (pose, k)
        # the frame traversal's sky exit (World::ytop) ends upward rays above the terrain early: the
        # same hits from fewer steps (the step counts themselves: rv_trace_rays, test_trace_bit_exact)
        for k in ("sphere_steps", "dda_steps", "csdf_checks"):
            assert st[k] <= ref["stats"][k], (pose, k)
    r.close()


@pytest.mark.parametrize("cfgname,pose", [("c2", "P0"), ("c3", "P0"), ("c3", "P1"), ("c4", "P0"), ("c4", "P1"),
                                         ("c5", "P0"), ("c5", "P1")])
def test_fullsize_world_traversal_gi_frame_rows(rv, atlas, oracle, cfgname, pose):
    from rvgrt_amd.configs import CONFIGS, pose_f32
    cfg = CONFIGS[cfgname]
    lg = cfg.log2_n
    W, H = cfg.width, cfg.height
    r = rv.StateRender((lg,) * 3, W, H, flags=cfg.flags, atlas=atlas)
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    r.sync()
    ow = check_world_rays_gi(r, rv, oracle, atlas, (lg,) * 3, lg, cfgname, gi_window=cfg.gi_sweeps >= 0)
    cam, vp = rv.camera_from_pose(*pose_f32(cfg, pose), W, H)
    r.frame(cam, vp)
    # the whole frame: every pixel's RGBA8, MV and depth
    check_rows(r, rv, oracle, ow, W, H, cfg.flags, rv.camera_dict(cam, vp), None, nrows=None)
    r.close()


def test_reference_native_config_draw_cuda(rv, atlas, oracle):
    """The reference as it ships: 4096 x 512 x 4096 world (include/cumath.cuh:
    19-21), 1280 x 800 (include/State.hpp:28-29), GI initialised then one
    UpdateGIData before each drawCUDA (src/main.cpp:119-132), drawCUDA with
    the c_cam off-by-one (time <- jitterY, jitter <- (0, 0); Appendix R1) and
    minDist's normalized-coordinate fetch (RV_F_REF_FETCH), camera at the
    reference defaults (src/Character.cpp:30,45-46)."""
    import math
    log2 = (12, 9, 12)
    W, H = 1280, 800
    flags = rv.RV_FLAGS_REFERENCE
    r = rv.StateRender(log2, W, H, flags=flags, atlas=atlas, ref_compat=True)
    r.world_build()
    r.update_gi_data()              # frame 0: cells [0, 262144)
    r.sync()
    ow = check_world_rays_gi(r, rv, oracle, atlas, log2, 12, "native", stage="gi_window0")
    f32 = lambda v: float(np.float32(v))
    cam, vp = rv.camera_from_pose((128.0, 350.0, 128.0), f32(-0.7), f32(-math.pi - 0.3), W, H)
    d = rv.camera_dict(cam, vp)
    r.draw_cuda(d["pos"], d["fo"], d["up"], d["ri"], vp, vp, 0.3, 0.7)   # jitterX ignored, time = 0.7
    rows, ref = check_rows(r, rv, oracle, ow, W, H, flags | rv.RV_F_REF_FETCH, d, np.random.default_rng(7),
                           time=0.7)
    assert len(rows) >= 64
    # R9 on the reference's own configuration: the same rows with the arithmetic
    # nvcc compiles the reference to (FMA contraction, oracle/r9_study.py) stay
    # within the SURVEY s8c tolerance of the uncontracted ones
    with oracle.numerics("fma_gcc"):
        var = oracle.render_rows(ow, oracle.make_frame(W, H, flags | rv.RV_F_REF_FETCH, d, time=0.7), rows,
                                 want_stats=False)
    dv = np.abs(var["rgba"][rows].astype(np.int32) - ref["rgba"][rows].astype(np.int32)).max(axis=-1)
    print(f"native rows under FMA contraction: {(dv == 0).mean():.5f} exact, {(dv <= 2).mean():.5f} within 2 LSB")
    assert (dv <= 2).mean() >= 0.995
    # how much the R6 fetch matters on this frame: the same rows with exact texel indices (informational)
    fr = oracle.make_frame(W, H, flags, d, time=0.7)
    img = r.readback(rv.RV_IMAGE_COLOR)
    plain = oracle.render_rows(ow, fr, rows, want_stats=False)["rgba"][rows]
    ndiff = int(np.any(plain != img[rows], axis=-1).sum())
    print(f"native frame: {ndiff} pixels of {len(rows)} rows differ between the reference fetch and exact texels")
    r.close()


@pytest.mark.parametrize("cfgname,grp,pose", [("c3", 0, "P0"), ("c4", 0, "P0"), ("c3", 8, "P0"), ("c4", 8, "P0"),
                                              ("c4", 0, "P1"), ("c3", 8, "P1")])
def test_fullsize_pipelined_frames(rv, atlas, cfgname, grp, pose):
    """The C3/C4 frame loop as bench.py runs it (pipelined launches: render
    k | GI update k+1 | pre-pass k+1; or grouped: 8 frames per launch) against UpdateGIData + drawCUDA one
    frame at a time (drawCUDA's two launches, rv_set_flow(0)) on the same full-size world: colour, depth
    and the GI grid bit-identical after 6 frames (the one-at-a-time frames are checked against the oracle
    by the tests above).  P1 (water-heavy): the water reflection's empty-column skip of the pipelined and
    grouped launches (rv_device.h trace COL) on most of the frame; the one-at-a-time frames' two launches
    equal the flow launch, which does not take the skip, and the oracle (test_fullsize_drop_in_flow_frames)."""
    from rvgrt_amd.configs import CONFIGS, pose_f32
    cfg = CONFIGS[cfgname]
    W, H = cfg.width, cfg.height
    cam, vp = rv.camera_from_pose(*pose_f32(cfg, pose), W, H)
    rs = []
    for pipe in (1, 0):
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=atlas)
        r.world_build()
        for s in range(max(cfg.gi_sweeps, 0)):
            r.gi_update(s)
        r.set_pipeline(pipe)
        r.set_flow(0)
        nf = 12 if grp else 6    # grouped: 8 frames per launch, the call ends mid-group
        if pipe:
            r.set_frame_group(grp)
            r.render_frames(nf, cam, vp, gi_per_frame=True)
        else:
            for _ in range(nf):
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


@pytest.mark.parametrize("cfgname,pose", [("c3", "P0"), ("c4", "P0"), ("c4", "P1"), ("c5", "P0")])
def test_fullsize_drop_in_flow_frames(rv, atlas, oracle, cfgname, pose):
    """renderLoop's own calls at full size (UpdateGIData, then drawCUDA with a
    moving camera, one frame per call, ref_compat): the flow launch (pre-pass k
    | next window's GI cells | render k, render waves waiting per pre-pass tile)
    against drawCUDA's two launches -- colour, motion, depth, half-res images
    and the GI grid bit-identical after every frame, no render wave fell back
    -- and the last frame whole against the oracle on the exported world."""
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32
    cfg = CONFIGS[cfgname]
    W, H = cfg.width, cfg.height
    seq = camera_path(pose_f32(cfg, pose), W, H, 6, pan=0.002, ref_compat=True)
    rs = []
    for flow in (1, 0):
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=atlas, ref_compat=True)
        r.world_build()
        for s in range(max(cfg.gi_sweeps, 0)):
            r.gi_update(s)
        r.set_flow(flow)
        rs.append(r)
    WG.assert_world(rs[0], rv, cfgname)   # bits, CSDF and the swept GI grid: the oracle's own whole builds
    lg = cfg.log2_n
    ow = oracle.OracleWorld(lg, lg, lg, atlas=atlas)
    ow.bits[:] = rs[0].world_export(rv.RV_WORLD_BITS)
    ow.csdf[:] = rs[0].world_export(rv.RV_WORLD_CSDF)
    ow.gi[:] = rs[0].world_export(rv.RV_WORLD_GI)
    kinds = (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH, rv.RV_IMAGE_HALF_DIST, rv.RV_IMAGE_HALF_SHADOW)
    for k in range(5):
        d = seq[k]
        c = d.cam
        for r in rs:
            r.update_gi_data()
            r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                        np.ctypeslib.as_array(d.prev_vp), 0.0, d.time)
        for kind in kinds:
            assert np.array_equal(rs[0].readback(kind), rs[1].readback(kind)), (k, kind)
        assert np.array_equal(rs[0].world_export(rv.RV_WORLD_GI), rs[1].world_export(rv.RV_WORLD_GI)), k
    assert rs[0].flow_info()[1:] == (5, 0)
    # the 5 UpdateGIData windows (frames 0-4, rolling offset from 0; src/CoarseArray.cu:376-395) by the
    # oracle on its own swept grid: the grid the last frame renders with
    for fno in range(5):
        ow.gi_update(fno, first=fno * WG.RAYPS, count=WG.RAYPS)
    assert np.array_equal(rs[0].world_export(rv.RV_WORLD_GI), ow.gi)
    d = seq[4]
    check_rows(rs[0], rv, oracle, ow, W, H, cfg.flags | rv.RV_F_REF_FETCH,
               rv.camera_dict(d.cam, np.ctypeslib.as_array(d.vp)), None, time=d.time, nrows=None,
               pvp=np.ctypeslib.as_array(d.prev_vp))
    for r in rs:
        r.close()
