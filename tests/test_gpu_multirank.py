"""The N-rank frame loop without N GPUs: N contexts on one GPU are the
ranks of an in-process loopback communicator (rv_comm_create_loopback), each
rank's rv_render_frame_seq driven by its own host thread.  This executes the
code paths one rank never reaches (DESIGN s7): the weighted
interleaved tile deal with padded slices, RGB24 / RGBA8 packing, the grouped
send/recv of packed tiles to rank 0 and its assembly, the sharded GI update
with its all-gather, the kept next-frame work across calls, and the check
that the ranks agree on the exchange's configuration.  Rank 0's frames and
every rank's GI grid must be bit-identical to one context rendering whole
frames one at a time; a rank that never arrives is an error after the
timeout, not a hang."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


LG, W, H, RAYS = 7, 320, 192, 5000


def _make(rv, atlas, flags):
    r = rv.StateRender((LG,) * 3, W, H, flags=flags, atlas=atlas, gi_rays_per_frame=RAYS)
    r.world_build()
    r.gi_update(0)
    return r


def _run_ranks(fns):
    """Runs fns[q]() on N threads; re-raises the first failure."""
    errs = [None] * len(fns)

    def body(q):
        try:
            fns[q]()
        except BaseException as e:   # noqa: BLE001 -- reported below
            errs[q] = e
    ts = [threading.Thread(target=body, args=(q,)) for q in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
        assert not t.is_alive(), "a rank thread hung"
    for e in errs:
        if e is not None:
            raise e


@pytest.mark.parametrize("flags,T,N,w0,bpp,grp", [
    (8, 16, 2, 1.0, 3, 0), (8, 16, 3, 0.9, 4, 0), (8, 32, 8, 0.87, 3, 0),       # batched groups (C1/C2 loop)
    (7, 32, 2, 1.0, 3, 0), (7, 32, 3, 0.94, 4, 0), (7, 16, 8, 0.87, 3, 0),      # pipelined reference frames
    (7, 64, 2, 0.98, 3, 0), (7, 64, 4, 0.94, 4, 0),                         # the bench's reference-frame tile size
    (7, 64, 2, 0.98, 3, 3), (7, 32, 3, 0.94, 4, 2), (7, 64, 4, 0.94, 3, 3),    # grouped reference frames: sharded
    (7, 16, 8, 0.87, 3, 3),                                                 # phase A, record all-gather per group
])
def test_loopback_ranks_equal_one_context(rv, atlas, flags, T, N, w0, bpp, grp):
    from rvgrt_amd.configs import TEST_POSES_128, camera_path
    gi = bool(flags & rv.RV_F_GI)
    seq = camera_path(TEST_POSES_128["P0"], W, H, 11, pan=0.02, ref_compat=True)
    ref = _make(rv, atlas, flags)
    ref.set_pipeline(0)
    group = rv.LoopbackGroup(N, timeout_ms=60000)
    rs = [_make(rv, atlas, flags) for _ in range(N)]
    comms = []
    for q, r in enumerate(rs):
        if not gi:
            r.set_frames_in_flight(4)
        r.set_tile_shard(T, q, N, root_weight=w0)
        r.set_gather_bpp(bpp)
        r.set_frame_group(grp)
        comms.append(rv.Comm.loopback(r, group, q))
    done = 0
    for a, b, nxt in ((0, 4, 4), (4, 11, None)):   # two calls: the second starts from the kept work
        _run_ranks([lambda q=q: rs[q].render_frame_seq(seq[a:b], next_desc=seq[nxt] if nxt else None, flags=flags,
                                                       gi_per_frame=gi, comm=comms[q]) for q in range(N)])
        for c in comms:
            c.wait(60000)
        for k in range(done, b):
            if gi:
                ref.update_gi_data()
            d = seq[k]
            ref.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                      jx=d.jitter_x, jy=d.jitter_y, flags=flags)
        done = b
        assert np.array_equal(rs[0].readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR)), (a, b)
        if gi:
            want = ref.world_export(rv.RV_WORLD_GI)
            for q, r in enumerate(rs):
                assert np.array_equal(r.world_export(rv.RV_WORLD_GI), want), (q, a, b)
    for c in comms:
        c.close()
    for r in rs:
        r.close()
    group.close()
    ref.close()


def test_loopback_rank_disagreement_is_rejected(rv, atlas):
    """Two ranks with different deal weights: every rank's first loop call
    fails (the configuration all-gather differs) instead of mis-slicing."""
    group = rv.LoopbackGroup(2, timeout_ms=30000)
    rs = [_make(rv, atlas, 8) for _ in range(2)]
    comms = []
    for q, r in enumerate(rs):
        r.set_tile_shard(16, q, 2, root_weight=1.0 if q == 0 else 0.8)
        comms.append(rv.Comm.loopback(r, group, q))
    from rvgrt_amd.configs import TEST_POSES_128
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P0"], W, H)
    errs = []

    def body(q):
        try:
            rs[q].render_frames(2, cam, vp, comm=comms[q])
        except rv.RvError as e:
            errs.append(str(e))
    ts = [threading.Thread(target=body, args=(q,)) for q in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert len(errs) == 2 and all("disagree" in e for e in errs), errs
    for c in comms:
        c.close()
    for r in rs:
        r.close()
    group.close()


def test_loopback_disagreement_after_agreed_call_is_rejected(rv, atlas):
    """An agreed first call, then rank 1 alone changes its deal weight: the
    next call fails on both ranks (the configuration exchange runs on every
    call, so both enter it) instead of desynchronising the collectives."""
    group = rv.LoopbackGroup(2, timeout_ms=30000)
    rs = [_make(rv, atlas, 8) for _ in range(2)]
    comms = []
    for q, r in enumerate(rs):
        r.set_tile_shard(16, q, 2, root_weight=1.0)
        comms.append(rv.Comm.loopback(r, group, q))
    from rvgrt_amd.configs import TEST_POSES_128
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P0"], W, H)
    _run_ranks([lambda q=q: rs[q].render_frames(2, cam, vp, comm=comms[q]) for q in range(2)])
    for c in comms:
        c.wait(60000)
    rs[1].set_tile_shard(16, 1, 2, root_weight=0.8)
    errs = []

    def body(q):
        try:
            rs[q].render_frames(2, cam, vp, comm=comms[q])
        except rv.RvError as e:
            errs.append(str(e))
    ts = [threading.Thread(target=body, args=(q,)) for q in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
        assert not t.is_alive(), "a rank thread hung"
    assert len(errs) == 2 and all("disagree" in e for e in errs), errs
    # a communicator used with a context other than its own is rejected
    other = _make(rv, atlas, 8)
    other.set_tile_shard(16, 0, 2)
    with pytest.raises(rv.RvError, match="another context"):
        other.render_frames(1, cam, vp, comm=comms[0])
    other.close()
    for c in comms:
        c.close()
    for r in rs:
        r.close()
    group.close()


def test_loopback_missing_rank_times_out(rv, atlas):
    """A peer that never arrives: the loop call returns an error after the
    group's timeout (2 s here), and the communicator can still be closed."""
    import time
    group = rv.LoopbackGroup(2, timeout_ms=2000)
    r = _make(rv, atlas, 8)
    r.set_tile_shard(16, 0, 2)
    comm = rv.Comm.loopback(r, group, 0)
    from rvgrt_amd.configs import TEST_POSES_128
    cam, vp = rv.camera_from_pose(*TEST_POSES_128["P0"], W, H)
    t0 = time.perf_counter()
    with pytest.raises(rv.RvError, match="did not arrive"):
        r.render_frames(3, cam, vp, comm=comm)
    assert time.perf_counter() - t0 < 30
    comm.close()
    r.close()
    group.close()


@pytest.mark.parametrize("cfgname,N,w0,grp", [("c4", 4, 0.94, 0), ("c4", 4, 0.94, 16), ("c5", 8, 0.87, 16)])
def test_loopback_ranks_full_size(rv, atlas, monkeypatch, cfgname, N, w0, grp):
    """The N-rank loop at BASELINE's full sizes: C4 (1024^3, 3840x2160, 2 GI sweeps)
    on 4 ranks and C5 (2048^3) on 8, 64-px tiles dealt by weight, RGB24 packing, per-frame pipelined
    (group 0: the sharded GI update's all-gather every frame) or grouped (16 frames per launch: sharded
    phase A, one record all-gather per group).  20 frames in two calls -- a whole group and a partial
    one, the second call starting from the kept work -- and rank 0's assembled frame and every rank's GI
    grid equal to one context rendering UpdateGIData + drawCUDA one frame at a time.  Full-size shares
    exercise what the 128^3 cases cannot: 2,040 tiles with padded weighted slices, 16-frame groups
    carrying whole-size GI windows, 33 MB RGB24 gather buffers.  C5's ranks run without the texture
    tile table (7.25 GB each at 2048^3, nine contexts on one GPU; the tiles are the same either way)."""
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32
    cfg = CONFIGS[cfgname]
    W, H = cfg.width, cfg.height
    seq = camera_path(pose_f32(cfg, "P0"), W, H, 21, pan=0.0005, ref_compat=True)

    def make():
        r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=atlas,
                           tex_table=-1 if cfgname == "c5" else 0)
        r.world_build()
        for s in range(cfg.gi_sweeps):
            r.gi_update(s)
        return r

    ref = make()
    ref.set_pipeline(0)
    group = rv.LoopbackGroup(N, timeout_ms=120000)
    rs = [make() for _ in range(N)]
    comms = []
    for q, r in enumerate(rs):
        r.set_tile_shard(64, q, N, root_weight=w0)
        r.set_gather_bpp(3)
        r.set_frame_group(grp)
        comms.append(rv.Comm.loopback(r, group, q))
    if grp:
        assert rs[0].frame_group_effective() == grp
    done = 0
    for a, b, nxt in ((0, 17, 17), (17, 20, None)):
        _run_ranks([lambda q=q: rs[q].render_frame_seq(seq[a:b], next_desc=seq[nxt] if nxt else None,
                                                       flags=cfg.flags, gi_per_frame=True, comm=comms[q])
                    for q in range(N)])
        for c in comms:
            c.wait(120000)
        for k in range(done, b):
            ref.update_gi_data()
            d = seq[k]
            ref.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                      jx=d.jitter_x, jy=d.jitter_y, flags=cfg.flags)
        done = b
        assert np.array_equal(rs[0].readback(rv.RV_IMAGE_COLOR), ref.readback(rv.RV_IMAGE_COLOR)), (a, b)
        want = ref.world_export(rv.RV_WORLD_GI)
        for q, r in enumerate(rs):
            assert np.array_equal(r.world_export(rv.RV_WORLD_GI), want), (q, a, b)
    for c in comms:
        c.close()
    for r in rs:
        r.close()
    group.close()
    ref.close()
