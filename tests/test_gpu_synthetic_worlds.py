"""GPU parity on worlds the terrain generator never makes: imported voxel bits
(rv_world_import) with the CSDF and the GI grid built on the GPU from them, against
the oracle building the same from the same bits.

The procedural worlds of the other tests are smooth height fields with a solid
floor; these reach the traversal's remaining paths: rays that start inside solid
voxels (the reference's mask = -128 hit, Appendix R2) on every pixel of a full
world, an empty world (every ray leaves the grid; no sky row, no sun horizon),
1 to 40 % random occupancy (DDA stops at every distance, CSDF values 0-64 in every
cell), one-voxel pillars (grazing rays along faces, the column skip between them)
and ragged power-of-two dims.  Bar: bit-exact -- CSDF, GI init, a GI update window,
20,000 traced rays with the reference's step counts, and whole frames (RGBA8,
motion, depth, half-res distance) at the reference's flags and the C2 flags.
"""
import numpy as np
import pytest

from conftest import random_rays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def _voxels(kind, X, Y, Z, rng):
    """Dense [z, y, x] occupancy of one synthetic world."""
    if kind == "empty":
        return np.zeros((Z, Y, X), bool)
    if kind == "full":
        return np.ones((Z, Y, X), bool)
    if kind == "sparse":
        return rng.uniform(size=(Z, Y, X)) < 0.01
    if kind == "dense":
        return rng.uniform(size=(Z, Y, X)) < 0.40
    if kind == "pillars":            # a floor and 1-voxel pillars of mixed heights every 6 voxels
        v = np.zeros((Z, Y, X), bool)
        v[:, :8, :] = True
        h = rng.integers(10, Y - 10, (Z // 6 + 1, X // 6 + 1))
        for k in range(0, Z, 6):
            for i in range(0, X, 6):
                v[k, :h[k // 6, i // 6], i] = True
        return v
    if kind == "blocks":             # 4^3 blocks at 10 %, with a floor (ragged dims)
        b = rng.uniform(size=(Z // 4, Y // 4, X // 4)) < 0.10
        v = b.repeat(4, 0).repeat(4, 1).repeat(4, 2)
        v[:, :2, :] = True
        return v
    raise ValueError(kind)


WORLDS = [("empty", (7, 7, 7)), ("full", (6, 6, 6)), ("sparse", (7, 7, 7)), ("dense", (6, 6, 6)),
          ("pillars", (7, 7, 7)), ("blocks", (6, 5, 7))]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind,dims", WORLDS, ids=[w[0] for w in WORLDS])
def test_synthetic_world_bit_exact(rv, atlas, oracle, kind, dims):
    lx, ly, lz = dims
    ow = oracle.OracleWorld(lx, ly, lz, atlas=atlas)
    X, Y, Z = ow.X, ow.Y, ow.Z
    rng = np.random.default_rng(sum(map(ord, kind)))
    vox = _voxels(kind, X, Y, Z, rng)
    ow.bits[:] = np.packbits(vox.ravel(), bitorder="little").view(np.uint32)
    ow.build_csdf()
    ow.gi_init()

    W, H = 160, 96
    r = rv.StateRender(dims, W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
    try:
        r.world_import(rv.RV_WORLD_BITS, ow.bits)
        r.csdf_build()
        assert np.array_equal(r.world_export(rv.RV_WORLD_CSDF), ow.csdf), "CSDF built from the imported bits"
        r.gi_init()
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi), "GI init"
        n = len(ow.gi) // 4
        first, count = n // 5, min(n - n // 5, 9000)
        r.gi_update(2, first=first, count=count)
        ow.gi_update(2, first=first, count=count)
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi), "GI update window"

        org, d, dist = random_rays(np.random.default_rng(7), 20000, (X, Y, Z))
        g = r.trace_rays(org, d, dist)
        o = ow.trace_batch(org, d, dist)
        assert (g["hit"] == o["hit"]).all() and (g["undef"] == o["undef"]).all()
        assert np.array_equal(g["pos"].view(np.uint32), o["pos"].view(np.uint32))
        assert np.array_equal(g["normal"], o["normal"])
        assert np.array_equal(g["u"].view(np.uint32), o["u"].view(np.uint32))
        assert np.array_equal(g["v"].view(np.uint32), o["v"].view(np.uint32))
        for a, b in (("sphere_steps", "n_sphere"), ("dda_steps", "n_dda"), ("csdf_checks", "n_check")):
            assert np.array_equal(g[a], o[b]), a
        if kind == "empty":
            assert not o["hit"].any()
        if kind == "full":   # every ray that starts in the grid starts in a solid voxel (R2)
            p0 = org + d * dist[:, None]
            inside = ((p0 >= 0) & (p0 < np.array([X, Y, Z], np.float32))).all(axis=1)
            assert o["undef"][inside].mean() > 0.99 and inside.mean() > 0.5

        cam, vp = rv.camera_from_pose((0.1 * X, 0.7 * Y, 0.1 * Z), -0.7, -np.pi - 0.3, W, H)
        for flags in (rv.RV_FLAGS_REFERENCE, rv.RV_F_SHADOW):
            r.frame(cam, vp, flags=flags)
            ref = oracle.render(ow, oracle.make_frame(W, H, flags, rv.camera_dict(cam, vp)), want_stats=False)
            assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref["rgba"]), flags
            assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref["mv"]), flags
            assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref["depth"]), flags
            if flags & rv.RV_F_PREPASS:
                assert np.array_equal(r.readback(rv.RV_IMAGE_HALF_DIST).view(np.uint32),
                                      ref["halfdist"].view(np.uint32))
    finally:
        r.close()


FLOW_WORLDS = [("pillars", (7, 7, 7)), ("sparse", (7, 7, 7)), ("full", (6, 6, 6)), ("blocks", (6, 5, 7))]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind,dims", FLOW_WORLDS, ids=[w[0] for w in FLOW_WORLDS])
def test_synthetic_world_drop_in_flow(rv, atlas, oracle, kind, dims):
    """renderLoop's calls (UpdateGIData, drawCUDA with ref_compat, a moving camera) on the same
    worlds: the one-launch flow frames equal drawCUDA's two launches image for image and GI grid
    for grid, with no render wave falling back; the last frame and the grid equal the oracle."""
    from rvgrt_amd.configs import camera_path
    lx, ly, lz = dims
    ow = oracle.OracleWorld(lx, ly, lz, atlas=atlas)
    X, Y, Z = ow.X, ow.Y, ow.Z
    vox = _voxels(kind, X, Y, Z, np.random.default_rng(sum(map(ord, kind))))
    ow.bits[:] = np.packbits(vox.ravel(), bitorder="little").view(np.uint32)
    ow.build_csdf()
    ow.gi_init()
    W, H, rays, nfr = 192, 128, 3000, 6
    ngi = len(ow.gi) // 4
    seq = camera_path(((0.1 * X, 0.7 * Y, 0.1 * Z), -0.7, -np.pi - 0.3), W, H, nfr, pan=0.03, ref_compat=True)
    ctx = []
    try:
        for flow in (1, 0):
            r = rv.StateRender(dims, W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas, gi_rays_per_frame=rays)
            ctx.append(r)
            r.world_import(rv.RV_WORLD_BITS, ow.bits)
            r.csdf_build()
            r.gi_init()
            r.set_flow(flow)
        a, b = ctx
        for k in range(nfr):
            for r in (a, b):
                r.update_gi_data()
                c = seq[k].cam
                r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(seq[k].vp),
                            np.ctypeslib.as_array(seq[k].prev_vp), 0.0, seq[k].time)
            for kind_img in (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH, rv.RV_IMAGE_HALF_DIST,
                             rv.RV_IMAGE_HALF_SHADOW):
                assert np.array_equal(a.readback(kind_img), b.readback(kind_img)), (k, kind_img)
        assert np.array_equal(a.world_export(rv.RV_WORLD_GI), b.world_export(rv.RV_WORLD_GI))
        active, launches, fallbacks = a.flow_info()
        assert active and launches == nfr and fallbacks == 0
        off = 0
        for fno in range(nfr):
            ow.gi_update(fno, first=off, count=min(rays, ngi - off))
            off = 0 if off + rays >= ngi else off + rays
        assert np.array_equal(a.world_export(rv.RV_WORLD_GI), ow.gi)
        d = seq[nfr - 1]
        fr = oracle.make_frame(W, H, rv.RV_FLAGS_REFERENCE | rv.RV_F_REF_FETCH,
                               rv.camera_dict(d.cam, np.ctypeslib.as_array(d.vp)), time=d.time,
                               pvp=np.ctypeslib.as_array(d.prev_vp))
        ref = oracle.render(ow, fr, want_stats=False)
        assert np.array_equal(a.readback(rv.RV_IMAGE_COLOR), ref["rgba"])
        assert np.array_equal(a.readback(rv.RV_IMAGE_MOTION), ref["mv"])
        assert np.array_equal(a.readback(rv.RV_IMAGE_DEPTH), ref["depth"])
    finally:
        for r in ctx:
            r.close()


def _basis(fo, up_hint):
    fo = np.asarray(fo, np.float64)
    fo /= np.linalg.norm(fo)
    ri = np.cross(fo, up_hint)
    ri /= np.linalg.norm(ri)
    up = np.cross(fo, ri)
    return [np.asarray(v, np.float32) for v in (fo, up, ri)]


# (name, camera position, forward, up, right): exact axis-aligned bases put the centre column's rays on
# zero direction components (the 1e10 deltaDist path) and integer positions on voxel faces
CAMERAS = [
    ("axis_z", (64.0, 40.0, 64.0), (0, 0, 1), (0, -1, 0), (1, 0, 0)),
    ("down", (64.5, 120.0, 64.5), (0, -1, 0), (0, 0, 1), (1, 0, 0)),
    ("axis_x_face", (0.0, 48.0, 64.0), (1, 0, 0), (0, -1, 0), (0, 0, -1)),
    ("outside", (-40.0, 90.0, -40.0)) + tuple(_basis((1.0, -0.45, 1.0), (0, 1, 0))),
    ("in_floor", (64.25, 5.0, 64.75)) + tuple(_basis((0.3, -0.2, 1.0), (0, 1, 0))),
    ("corner", (0.0, 0.0, 0.0)) + tuple(_basis((1.0, 1.0, 1.0), (0, 1, 0))),
]


@pytest.mark.parametrize("name,pos,fo,up,ri", CAMERAS, ids=[c[0] for c in CAMERAS])
def test_camera_edge_cases(rv, atlas, oracle, oracle_world, name, pos, fo, up, ri):
    """Frames from cameras no pose of the bench takes -- looking exactly along an axis from an
    integer position, straight down, from a voxel face at the grid's edge, from outside the grid,
    from inside the solid floor (every primary ray the R2 undefined hit) and from the grid's
    corner -- equal the oracle bit for bit (reference and C2 flags) on the procedural 128^3 world."""
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    W, H = 160, 96
    r = rv.StateRender((7, 7, 7), W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
    try:
        r.world_import(rv.RV_WORLD_BITS, ow.bits)
        r.world_import(rv.RV_WORLD_CSDF, ow.csdf)
        r.world_import(rv.RV_WORLD_GI, ow.gi)
        _, vp = rv.camera_from_pose((12.8, 76.8, 12.8), -0.7, -np.pi - 0.3, W, H)
        cam = rv._lib.rv_camera()
        for k, v in (("pos", pos), ("forward", fo), ("up", up), ("right", ri)):
            getattr(cam, k)[:] = [float(x) for x in np.asarray(v, np.float32)]
        for flags in (rv.RV_FLAGS_REFERENCE, rv.RV_F_SHADOW):
            r.frame(cam, vp, flags=flags)
            ref = oracle.render(ow, oracle.make_frame(W, H, flags, rv.camera_dict(cam, vp)), want_stats=False)
            assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref["rgba"]), flags
            assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref["mv"]), flags
            assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref["depth"]), flags
    finally:
        r.close()


ODD_SIZES = [(161, 97), (67, 33), (1000, 7), (2, 2), (130, 258), (1707, 961)]


@pytest.mark.parametrize("W,H", ODD_SIZES)
def test_odd_resolutions(rv, atlas, oracle, oracle_world, W, H):
    """Frame sizes off every tile grid -- odd (a DLSS render size such as 1707 x 961 for a 2560 x
    1441 window), tiny, one-texel-high half-res images, taller than wide: the two-launch frame and
    the drop-in flow frame (renderLoop's calls) equal the oracle.  The half-res images are
    floor(W / 2) x floor(H / 2) as the reference's (src/StateRender.cu:150-151,318-325)."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    seq = camera_path(TEST_POSES_128["P0"], W, H, 2, pan=0.01, ref_compat=True)
    d = seq[1]
    for flow in (0, 1):
        r = rv.StateRender((7, 7, 7), W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
        try:
            r.world_import(rv.RV_WORLD_BITS, ow.bits)
            r.world_import(rv.RV_WORLD_CSDF, ow.csdf)
            r.world_import(rv.RV_WORLD_GI, ow.gi)
            r.set_flow(flow)
            c = d.cam
            r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                        np.ctypeslib.as_array(d.prev_vp), 0.0, d.time)
            fr = oracle.make_frame(W, H, rv.RV_FLAGS_REFERENCE | rv.RV_F_REF_FETCH,
                                   rv.camera_dict(c, np.ctypeslib.as_array(d.vp)), time=d.time,
                                   pvp=np.ctypeslib.as_array(d.prev_vp))
            ref = oracle.render(ow, fr, want_stats=False)
            assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref["rgba"]), flow
            assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref["mv"]), flow
            assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref["depth"]), flow
        finally:
            r.close()


@pytest.mark.parametrize("W,H", ODD_SIZES)
def test_odd_resolutions_wavefront_and_tiles(rv, atlas, oracle_world, W, H):
    """The same sizes through the wavefront stages and through screen tiles (three "ranks" of
    interleaved 16-px tiles with their own half-res halos, scattered back by rv_untile): both equal
    the per-pixel frame."""
    from rvgrt_amd.configs import TEST_POSES_128
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P1"], W, H)

    def ctx():
        r = rv.StateRender((7, 7, 7), W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
        r.world_import(rv.RV_WORLD_BITS, ow.bits)
        r.world_import(rv.RV_WORLD_CSDF, ow.csdf)
        r.world_import(rv.RV_WORLD_GI, ow.gi)
        return r

    full = ctx()
    wf = ctx()
    sink = ctx()
    try:
        full.frame(cam, vp)
        want = [full.readback(k).copy() for k in (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH)]
        wf.set_frame_path("wavefront")
        wf.frame(cam, vp)
        for k, img in zip((rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH), want):
            assert np.array_equal(wf.readback(k), img), k
        T = 16
        ids_all = np.arange(((W + T - 1) // T) * ((H + T - 1) // T), dtype=np.int32)
        for rank in range(3):
            ids = ids_all[rank::3]
            if not len(ids):
                continue
            rr = ctx()
            try:
                rr.frame_tiles(cam, vp, ids, tile_px=T)
                rr.sync()
                p, nbytes = rr.tile_buffer()
                assert nbytes >= len(ids) * T * T * 4
                sink.untile(p, ids, tile_px=T)
                sink.sync()
            finally:
                rr.close()
        assert np.array_equal(sink.readback(rv.RV_IMAGE_COLOR), want[0])
    finally:
        for r in (full, wf, sink):
            r.close()


@pytest.mark.parametrize("W,H", [(161, 97), (1707, 961)])
@pytest.mark.parametrize("loop", ["pipelined", "grouped"])
def test_odd_resolutions_frame_loops(rv, atlas, W, H, loop):
    """The native loops at odd sizes: rv_render_frame_seq pipelined (k_ref_pipe) and in groups of 4
    (k_ref_group) on a moving camera equal UpdateGIData + one frame at a time, images and GI grid."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    flags, rays = rv.RV_FLAGS_REFERENCE, 3000
    seq = camera_path(TEST_POSES_128["P0"], W, H, 7, pan=0.01, ref_compat=True)

    def make():
        r = rv.StateRender((7, 7, 7), W, H, flags=flags, atlas=atlas, gi_rays_per_frame=rays)
        r.world_build()
        r.gi_update(0)
        return r

    ref, r = make(), make()
    try:
        ref.set_pipeline(0)
        if loop == "grouped":
            r.set_frame_group(4)
        for a, b in ((0, 3), (3, 6)):
            r.render_frame_seq(seq[a:b], next_desc=seq[b], flags=flags, gi_per_frame=True)
            for d in seq[a:b]:
                ref.update_gi_data()
                ref.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                          jx=d.jitter_x, jy=d.jitter_y, flags=flags)
            for k in (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH, rv.RV_IMAGE_HALF_DIST):
                assert np.array_equal(r.readback(k), ref.readback(k)), (a, k)
            assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ref.world_export(rv.RV_WORLD_GI)), a
    finally:
        r.close()
        ref.close()


@pytest.mark.parametrize("flags,T,N,grp", [(8, 16, 3, 0), (7, 16, 3, 0), (7, 32, 2, 3)])
def test_odd_resolution_loopback_ranks(rv, atlas, flags, T, N, grp):
    """The N-rank loop (loopback communicator, one host thread per rank; see test_gpu_multirank.py) at
    161 x 97: partial tiles on the right and bottom edges, the gather and rank 0's assembly -- rank 0's
    frames and every rank's GI grid equal one context rendering whole frames one at a time."""
    import threading
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    W, H, rays = 161, 97, 3000
    gi = bool(flags & rv.RV_F_GI)
    seq = camera_path(TEST_POSES_128["P0"], W, H, 7, pan=0.02, ref_compat=True)

    def make():
        r = rv.StateRender((7, 7, 7), W, H, flags=flags, atlas=atlas, gi_rays_per_frame=rays)
        r.world_build()
        r.gi_update(0)
        return r

    ref = make()
    ref.set_pipeline(0)
    group = rv.LoopbackGroup(N, timeout_ms=60000)
    rs = [make() for _ in range(N)]
    comms = []
    try:
        for q, r in enumerate(rs):
            if not gi:
                r.set_frames_in_flight(4)
            r.set_tile_shard(T, q, N)
            r.set_frame_group(grp)
            comms.append(rv.Comm.loopback(r, group, q))
        errs = [None] * N

        def body(q):
            try:
                rs[q].render_frame_seq(seq[0:6], next_desc=seq[6], flags=flags, gi_per_frame=gi, comm=comms[q])
            except BaseException as e:   # noqa: BLE001 -- re-raised below
                errs[q] = e
        ts = [threading.Thread(target=body, args=(q,)) for q in range(N)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
            assert not t.is_alive(), "a rank thread hung"
        for e in errs:
            if e is not None:
                raise e
        for c in comms:
            c.wait(60000)
        for d in seq[0:6]:
            if gi:
                ref.update_gi_data()
            ref.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                      jx=d.jitter_x, jy=d.jitter_y, flags=flags)
        assert np.array_equal(rs[0].readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR))
        if gi:
            want = ref.world_export(rv.RV_WORLD_GI)
            for q, r in enumerate(rs):
                assert np.array_equal(r.world_export(rv.RV_WORLD_GI), want), q
    finally:
        for c in comms:
            c.close()
        for r in rs:
            r.close()
        group.close()
        ref.close()


@pytest.mark.parametrize("flags", list(range(16)) + [33, 39, 41])
def test_every_feature_combination(rv, atlas, oracle, oracle_world, flags):
    """Every combination of the frame's feature bits (pre-pass 1, water 2, GI 4, full-res shadow 8;
    plus the reference texel fetch 32 where a pre-pass exists), not only the bench's sets: the library's
    dispatch (compiled feature sets or the dynamic-feature kernel) equals the oracle on both poses."""
    from rvgrt_amd.configs import TEST_POSES_128
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    W, H = 160, 96
    r = rv.StateRender((7, 7, 7), W, H, flags=flags, atlas=atlas)
    try:
        r.world_import(rv.RV_WORLD_BITS, ow.bits)
        r.world_import(rv.RV_WORLD_CSDF, ow.csdf)
        r.world_import(rv.RV_WORLD_GI, ow.gi)
        for pose in ("P0", "P1"):
            cam, vp = rv.camera_from_pose(*TEST_POSES_128[pose], W, H)
            r.frame(cam, vp, flags=flags, time=0.25)
            ref = oracle.render(ow, oracle.make_frame(W, H, flags, rv.camera_dict(cam, vp), time=0.25),
                                want_stats=False)
            assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref["rgba"]), pose
            assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref["mv"]), pose
            assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref["depth"]), pose
    finally:
        r.close()
