"""Flow frames (rv_set_flow): the drop-in drawCUDA as one k_ref_flow launch.

renderLoop calls UpdateGIData, then drawCUDA, one frame per call with no
knowledge of the next camera (/root/reference/src/main.cpp:119-132,
src/StateRender.cu:289-346).  The flow launch runs that frame's pre-pass and
render together -- the render waves wait inside the launch for the pre-pass
tiles they read -- and the NEXT UpdateGIData's cells, which the next
rv_update_gi_data then only copies in.  Everything here must equal drawCUDA's
two launches (rv_set_flow(0)) bit for bit, and the oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def _make(rv, atlas, lg, W, H, rays, flow, flags=None):
    r = rv.StateRender((lg,) * 3, W, H, flags=rv.RV_FLAGS_REFERENCE if flags is None else flags, atlas=atlas,
                       gi_rays_per_frame=rays)
    r.world_build()
    r.gi_update(0)
    r.set_flow(flow)
    return r


def _draw(r, d):
    """drawCUDA with ref_compat: the jitterY argument is the frame time (Appendix R1)."""
    c = d.cam
    r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                np.ctypeslib.as_array(d.prev_vp), 0.0, d.time)


def _images(r, rv):
    return [r.readback(k).copy() for k in (rv.RV_IMAGE_COLOR, rv.RV_IMAGE_MOTION, rv.RV_IMAGE_DEPTH,
                                           rv.RV_IMAGE_HALF_DIST, rv.RV_IMAGE_HALF_SHADOW)]


@pytest.mark.parametrize("pose,rays,readback_every,pairs", [("P0", 5000, 1, 0), ("P1", 5000, 4, 0), ("P0", 4096, 3, 0),
                                                            ("P1", 5000, 2, 1)])
def test_flow_frames_equal_two_launches_and_oracle(rv, atlas, oracle, monkeypatch, pose, rays, readback_every, pairs):
    """renderLoop's calls with a moving camera (yaw pan, the jitter sequence as
    the frame time, previous VP per frame), over a rolling GI window that wraps
    the 32^3 grid: every image and the GI grid equal the two-launch path after
    every frame read back (reading back rarely leaves several frames queued
    behind each other); the grid equals the oracle's rolling updates and the
    last frame the oracle's render (RGBA8, MV, depth); no render wave had to
    fall back to evaluating its own window.  pairs: the GI cells of these (latency-variant) launches on
    lane pairs (RV_OPT_GI_PAIRS)."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    lg, W, H = 7, 320, 192
    nfr = 11
    seq = camera_path(TEST_POSES_128[pose], W, H, nfr + 1, pan=0.02, ref_compat=True)
    a, b = _make(rv, atlas, lg, W, H, rays, 1), _make(rv, atlas, lg, W, H, rays, 0)
    for r in (a, b):
        r.set_option(rv.RV_OPT_GI_PAIRS, pairs)
        assert r.get_option(rv.RV_OPT_GI_PAIRS) == pairs
    for k in range(nfr):
        for r in (a, b):
            r.update_gi_data()
            _draw(r, seq[k])
        if k % readback_every == 0 or k == nfr - 1:
            for x, y in zip(_images(a, rv), _images(b, rv)):
                assert np.array_equal(x, y), k
            assert np.array_equal(a.world_export(rv.RV_WORLD_GI), b.world_export(rv.RV_WORLD_GI)), k
    active, launches, fallbacks = a.flow_info()
    assert active and launches == nfr and fallbacks == 0
    assert b.flow_info()[1] == 0
    ow = oracle.OracleWorld(lg, lg, lg, atlas=atlas).build(gi_sweeps=1)
    ngi, off = (1 << (lg - 2)) ** 3, 0
    for fno in range(nfr):
        ow.gi_update(fno, first=off, count=min(rays, ngi - off))
        off = 0 if off + rays >= ngi else off + rays
    assert np.array_equal(a.world_export(rv.RV_WORLD_GI), ow.gi)
    d = seq[nfr - 1]
    fr = oracle.make_frame(W, H, rv.RV_FLAGS_REFERENCE | rv.RV_F_REF_FETCH, rv.camera_dict(d.cam, np.ctypeslib.as_array(d.vp)),
                           time=d.time, pvp=np.ctypeslib.as_array(d.prev_vp))
    ref = oracle.render(ow, fr)
    assert np.array_equal(a.readback(rv.RV_IMAGE_COLOR), ref["rgba"])
    assert np.array_equal(a.readback(rv.RV_IMAGE_MOTION), ref["mv"])
    assert np.array_equal(a.readback(rv.RV_IMAGE_DEPTH), ref["depth"])
    a.close()
    b.close()


def test_flow_gi_computed_ahead_is_dropped_when_stale(rv, atlas):
    """The cells a flow launch computes for the next UpdateGIData are used only
    when nothing changed in between: call sequences that skip, repeat or
    interleave calls (two updates in a row, two frames in a row, an explicit
    GI window, a GI import, a frame without an update before it) give the same
    grid and frames as the two-launch path doing the same calls."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    lg, W, H, rays = 7, 320, 192, 5000
    seq = camera_path(TEST_POSES_128["P0"], W, H, 16, pan=0.02, ref_compat=True)
    a, b = _make(rv, atlas, lg, W, H, rays, 1), _make(rv, atlas, lg, W, H, rays, 0)
    gi_host = a.world_export(rv.RV_WORLD_GI)
    script = ["u", "d", "u", "d", "u", "u", "d", "d", "u", "d", "g", "u", "d", "i", "u", "d", "d", "u", "d",
              "u", "d", "u", "d"]
    k = 0
    for op in script:
        for r in (a, b):
            if op == "u":
                r.update_gi_data()
            elif op == "d":
                _draw(r, seq[k % len(seq)])
            elif op == "g":   # an explicit window in between (rv_gi_update): the kept cells are stale
                r.gi_update(40, first=777, count=3000)
            elif op == "i":   # a GI import in between
                r.world_import(rv.RV_WORLD_GI, gi_host)
        if op == "d":
            k += 1
            for x, y in zip(_images(a, rv), _images(b, rv)):
                assert np.array_equal(x, y), (k, op)
        assert np.array_equal(a.world_export(rv.RV_WORLD_GI), b.world_export(rv.RV_WORLD_GI)), (k, op)
    assert a.flow_info()[2] == 0
    a.close()
    b.close()


def test_flow_fallback_evaluates_the_same_texels(rv, atlas, monkeypatch):
    """The bounded wait's way out: with RV_OPT_FLOW_FORCE_FALLBACK every render
    wave waits for a value no pre-pass wave publishes, gives up after
    RV_OPT_FLOW_SPIN polls and evaluates its half-res window itself (distance
    and shadow) -- the frames must not change (and every render wave is counted)."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    lg, W, H, rays = 7, 160, 96, 5000
    seq = camera_path(TEST_POSES_128["P1"], W, H, 4, pan=0.02, ref_compat=True)
    b = _make(rv, atlas, lg, W, H, rays, 0)
    a = _make(rv, atlas, lg, W, H, rays, 1)
    a.set_option(rv.RV_OPT_FLOW_FORCE_FALLBACK, 1)
    a.set_option(rv.RV_OPT_FLOW_SPIN, 4)
    for k in range(3):
        for r in (a, b):
            r.update_gi_data()
            _draw(r, seq[k])
        for x, y in zip(_images(a, rv), _images(b, rv)):
            assert np.array_equal(x, y), k
    assert np.array_equal(a.world_export(rv.RV_WORLD_GI), b.world_export(rv.RV_WORLD_GI))
    waves = (W // 8) * (H // 8)
    assert a.flow_info()[2] == 3 * waves
    a.close()
    b.close()


def test_flow_stats_frame_counts(rv, atlas):
    """An RV_F_STATS flow frame counts its pre-pass and render into their own
    stage blocks exactly as the two-launch frame does (the GI part is not run
    for a stats frame)."""
    from rvgrt_amd.configs import TEST_POSES_128
    lg, W, H = 7, 160, 96
    flags = rv.RV_FLAGS_REFERENCE | rv.RV_F_STATS
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P0"], W, H)
    out = []
    for flow in (1, 0):
        r = _make(rv, atlas, lg, W, H, 0, flow)
        r.stats_reset()
        r.update_gi_data()
        r.frame(cam, vp, flags=flags)
        out.append({k: r.stats(k) for k in range(8)})
        r.close()
    for k in (0, 2):
        assert out[0][k] == out[1][k], k


def test_flow_fallback_throughput_variant_4k(rv, atlas, monkeypatch):
    """The forced fallback on a 3840x2160 frame: 129,600 render waves, so the
    flow launch is the throughput instantiation (render look-ahead RV_G_REF, the
    variant C4/C5 frames run) -- its fallback (prepass_eval at that look-ahead)
    must give the two-launch frame's texels too, and every render wave counts."""
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32
    lg, W, H, rays = 8, 3840, 2160, 5000
    seq = camera_path(pose_f32(CONFIGS["c1"], "P0"), W, H, 3, pan=0.01, ref_compat=True)
    b = _make(rv, atlas, lg, W, H, rays, 0)
    a = _make(rv, atlas, lg, W, H, rays, 1)
    a.set_option(rv.RV_OPT_FLOW_FORCE_FALLBACK, 1)
    a.set_option(rv.RV_OPT_FLOW_SPIN, 2)
    for k in range(2):
        for r in (a, b):
            r.update_gi_data()
            _draw(r, seq[k])
        for x, y in zip(_images(a, rv), _images(b, rv)):
            assert np.array_equal(x, y), k
    assert np.array_equal(a.world_export(rv.RV_WORLD_GI), b.world_export(rv.RV_WORLD_GI))
    waves = (W // 8) * (H // 8)
    assert waves > 49152
    assert a.flow_info() == (True, 2, 2 * waves)
    a.close()
    b.close()
