"""Grouped reference frames (rv_set_frame_group): n frames per launch with
the GI update split into phase A (traces into records) and phase B (the
combine with the grid, read through the overlay of not-yet-applied
updates).  Frames, depth, half-res images and the GI grid must be
bit-identical to UpdateGIData + drawCUDA one frame at a time, for every
group size, over calls of any length, with rolling GI windows that wrap
(src/main.cpp:119-132, src/CoarseArray.cu:273-395)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def _make(rv, atlas, lg, W, H, rays, sweeps=1):
    r = rv.StateRender((lg,) * 3, W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas, gi_rays_per_frame=rays)
    r.world_build()
    for s in range(sweeps):
        r.gi_update(s)
    return r


def _ref_step(rv, ref, d, flags):
    ref.update_gi_data()
    ref.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
              jx=d.jitter_x, jy=d.jitter_y, flags=flags)


@pytest.mark.parametrize("F,rays,order", [(2, 5000, "102"), (3, 5000, "012"), (4, 2048, "102"), (8, 2048, "210"),
                                          (8, 1000, "102"), (32, 500, "102")])
def test_grouped_frames_equal_one_at_a_time(rv, atlas, oracle, monkeypatch, F, rays, order):
    """128^3 world (32768 GI cells): windows of 5000 (partial last window,
    linear cell order), 2048 (whole planes, blocked order) and 1000 cells;
    calls of 1, 2, 5, 7 and 3 frames on a moving camera, so groups end
    mid-call and calls end mid-group."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    lg, W, H = 7, 320, 192
    flags = rv.RV_FLAGS_REFERENCE
    seq = camera_path(TEST_POSES_128["P0"], W, H, 18, pan=0.01, ref_compat=True)
    ref, r = _make(rv, atlas, lg, W, H, rays), _make(rv, atlas, lg, W, H, rays)
    r.set_option(rv.RV_OPT_PIPE_ORDER, int(order, 16))
    ref.set_pipeline(0)
    r.set_frame_group(F)
    k = 0
    for n in (1, 2, 5, 7, 3):
        r.render_frame_seq(seq[k:k + n], next_desc=seq[k + n], flags=flags, gi_per_frame=True)
        for d in seq[k:k + n]:
            _ref_step(rv, ref, d, flags)
        k += n
        assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR)), n
        assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref.readback(rv.RV_IMAGE_DEPTH)), n
        assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref.readback(rv.RV_IMAGE_MOTION)), n
        assert np.array_equal(r.readback(rv.RV_IMAGE_HALF_DIST), ref.readback(rv.RV_IMAGE_HALF_DIST)), n
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ref.world_export(rv.RV_WORLD_GI)), n
    # the oracle agrees on the grid after the 18 updates
    ow = oracle.OracleWorld(lg, lg, lg, atlas=atlas).build(gi_sweeps=1)
    ngi, off = (1 << (lg - 2)) ** 3, 0
    for fno in range(18):
        ow.gi_update(fno, first=off, count=min(rays, ngi - off))
        off = 0 if off + rays >= ngi else off + rays
    assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi)
    r.close()
    ref.close()


def test_grouped_frames_mixed_with_pipe_and_single_frames(rv, atlas):
    """Grouped calls, per-frame pipelined calls and single frames interleave
    on one context: the GI window sequence continues across all of them."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    lg, W, H, rays = 7, 256, 160, 2048
    flags = rv.RV_FLAGS_REFERENCE
    seq = camera_path(TEST_POSES_128["P1"], W, H, 20, pan=0.02, ref_compat=True)
    ref, r = _make(rv, atlas, lg, W, H, rays), _make(rv, atlas, lg, W, H, rays)
    ref.set_pipeline(0)
    k = 0
    for mode, n in (("group", 6), ("pipe", 3), ("single", 1), ("group", 5), ("pipe", 2), ("group", 3)):
        if mode == "single":
            _ref_step(rv, r, seq[k], flags)
        else:
            r.set_frame_group(4 if mode == "group" else 0)
            r.render_frame_seq(seq[k:k + n], next_desc=seq[k + n], flags=flags, gi_per_frame=True)
        for d in seq[k:k + n]:
            _ref_step(rv, ref, d, flags)
        k += n
        assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR)), (mode, k)
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ref.world_export(rv.RV_WORLD_GI)), (mode, k)
    r.close()
    ref.close()


def test_grouped_frames_512_world_default_window(rv, atlas):
    """512^3 world with the reference's RAYPS = 64^3 cells per update (8
    windows per sweep: the group cap is 4), a 640x360 frame, 13 frames."""
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32
    cfg = CONFIGS["c2"]
    lg, W, H = 9, 640, 360
    flags = rv.RV_FLAGS_REFERENCE
    seq = camera_path(pose_f32(cfg), W, H, 13, pan=0.002, ref_compat=True)
    ref, r = _make(rv, atlas, lg, W, H, 0), _make(rv, atlas, lg, W, H, 0)
    ref.set_pipeline(0)
    r.set_frame_group(16)          # capped to 4 by the 2M-cell grid
    r.render_frame_seq(seq[:13], next_desc=seq[13], flags=flags, gi_per_frame=True)
    for d in seq[:13]:
        _ref_step(rv, ref, d, flags)
    assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR))
    assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ref.world_export(rv.RV_WORLD_GI))
    r.close()
    ref.close()


def test_grouped_frames_one_rank_rccl(rv, atlas):
    """Grouped reference frames through a one-rank RCCL communicator (the
    transport bench.py uses at N >= 4: sharded phase A, the record all-gather
    per group, the tile gather to rank 0 and its assembly) equal one context
    rendering whole frames one at a time."""
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    lg, W, H, rays = 7, 320, 192, 2048
    flags = rv.RV_FLAGS_REFERENCE
    seq = camera_path(TEST_POSES_128["P0"], W, H, 16, pan=0.01, ref_compat=True)
    ref, r = _make(rv, atlas, lg, W, H, rays), _make(rv, atlas, lg, W, H, rays)
    ref.set_pipeline(0)
    r.set_tile_shard(64, 0, 1)
    r.set_gather_bpp(3)
    r.set_frame_group(8)
    comm = rv.Comm(r, rv.Comm.unique_id(), 1, 0)
    k = 0
    for n in (9, 6):
        r.render_frame_seq(seq[k:k + n], next_desc=seq[k + n], flags=flags, gi_per_frame=True, comm=comm)
        for d in seq[k:k + n]:
            _ref_step(rv, ref, d, flags)
        k += n
        assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR)), n
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ref.world_export(rv.RV_WORLD_GI)), n
    comm.close()
    r.close()
    ref.close()
