"""The shading and GI half restated twice: tests/np_shade.py (numpy, written from the
reference text) against the C oracle (oracle/rv_oracle.c) -- whole golden frames
(128^3, 160x96, poses P0 / P1, the C1 / C2 / reference flag sets and the
drop-in's minDist fetch) and GI update windows, bit for bit.  The ray cast
itself is the oracle's in both (pinned by tests/np_ref.py's scalar DDA), so
these tests check everything around it: texture, sky, cones, water, fog,
half-res taps, MV / depth and the GI blend."""
import numpy as np
import pytest

import np_shade as S

FLAGSETS = {"c1": 0, "c2": S.F_SHADOW, "ref": S.F_PREPASS | S.F_WATER | S.F_GI,
            "ref_fetch": S.F_PREPASS | S.F_WATER | S.F_GI | S.F_REF_FETCH}


def _world(ow):
    return {"dims": (ow.X, ow.Y, ow.Z), "csdf": ow.csdf, "gi": ow.gi.reshape(-1, 4), "solid": ow.voxels()}


def _trace(ow):
    return lambda org, d, dist: ow.trace_batch(np.ascontiguousarray(org, np.float32),
                                               np.ascontiguousarray(d, np.float32),
                                               np.ascontiguousarray(dist, np.float32))


def test_sun_direction_matches_oracle(oracle):
    assert np.array_equal(S.sun_dir().view(np.uint32), oracle.sun_dir().view(np.uint32))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("flagset", list(FLAGSETS))
@pytest.mark.parametrize("pose", ["P0", "P1"])
def test_frames_bit_exact_with_oracle(oracle, oracle_world, atlas, flagset, pose):
    from rvgrt_amd.configs import TEST_POSES_128
    W, H = 160, 96
    flags = FLAGSETS[flagset]
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    cam = oracle.camera_from_pose(*TEST_POSES_128[pose], W, H)
    time = 0.37 if pose == "P1" else 0.0                 # a moving water surface on the water pose
    ref = oracle.render(ow, oracle.make_frame(W, H, flags, cam, time=time))
    cam = dict(cam, pvp=cam["vp"])
    got = S.render(_trace(ow), _world(ow), cam, W, H, flags, time=time, atlas=atlas)
    hits = got["hits"]["hit"] != 0
    assert 0.2 < hits.mean() < 1.0                       # frames with sky and terrain
    if flags & S.F_WATER:
        assert ((got["hits"]["pos"][:, 1] < 31.001) & hits).any()   # the water branch ran
    bad = np.any(got["rgba"] != ref["rgba"], axis=-1)
    assert not bad.any(), f"{bad.sum()} pixels differ, first at {np.argwhere(bad)[:5].tolist()}"
    assert np.array_equal(got["mv"], ref["mv"])
    assert np.array_equal(got["depth"], ref["depth"])


def test_moving_camera_motion_vectors(oracle, oracle_world, atlas):
    """Previous VP != current VP: the motion vectors are non-zero and equal."""
    from rvgrt_amd.configs import TEST_POSES_128
    W, H = 96, 64
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    pos, yaw, pitch = TEST_POSES_128["P0"]
    cam = oracle.camera_from_pose(pos, yaw, pitch, W, H)
    prev = oracle.camera_from_pose((pos[0] + 1.5, pos[1], pos[2] - 1.0), yaw + 0.03, pitch, W, H)["vp"]
    flags = FLAGSETS["ref"]
    ref = oracle.render(ow, oracle.make_frame(W, H, flags, cam, pvp=prev, jx=0.01, jy=-0.02))
    got = S.render(_trace(ow), _world(ow), dict(cam, pvp=prev), W, H, flags, jx=0.01, jy=-0.02, atlas=atlas)
    assert np.array_equal(got["rgba"], ref["rgba"])
    assert np.array_equal(got["mv"], ref["mv"]) and (ref["mv"] != 0).any()
    assert np.array_equal(got["depth"], ref["depth"])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("lg,frame,first,count", [(6, 0, 0, None), (6, 5, 1000, 3000), (7, 3, 4096, 20000),
                                                  (7, 4732006, 3040, 8)])
def test_gi_update_window_bit_exact(oracle, oracle_world, atlas, lg, frame, first, count):
    """GlobalIlluminate over a window (whole grid; partial; a 128^3 plane-aligned window; the cell whose
    xorshift state is 0 at frame 4732006) equals the oracle's update of the same cells."""
    base = oracle_world(lg, lg, lg, gi_sweeps=1)
    n = len(base.gi) // 4
    count = n - first if count is None else count
    got = S.gi_update(_trace(base), _world(base), frame, first, count, atlas)
    w = oracle.OracleWorld(lg, lg, lg, atlas=atlas)
    w.bits[:] = base.bits
    w.csdf[:] = base.csdf
    w.gi[:] = base.gi
    w.gi_update(frame, first=first, count=count)
    want = w.gi.reshape(-1, 4)[first:first + count]
    bad = np.any(got != want, axis=1)
    assert not bad.any(), f"{bad.sum()} cells differ, first {np.flatnonzero(bad)[:5] + first}"
    if count > 100:
        assert (got != base.gi.reshape(-1, 4)[first:first + count]).any()   # the update changed cells


def test_cone_march_steps_and_occlusion(oracle, oracle_world):
    """traceCone alone: the numpy march against the oracle's single-cone entry point."""
    ow = oracle_world(7, 7, 7, gi_sweeps=1)
    rng = np.random.default_rng(5)
    pos = rng.uniform(0, 128, (400, 3)).astype(np.float32)
    d = rng.normal(size=(400, 3)).astype(np.float32)
    got, steps = S.trace_cone(pos, d, ow.gi.reshape(-1, 4), ow.csdf, (ow.X, ow.Y, ow.Z))
    import ctypes as C
    L, w = oracle.lib(), ow.c
    for i in range(len(pos)):
        n = C.c_int(0)
        r = L.or_trace_cone(C.byref(w), oracle.F3(*pos[i]), oracle.F3(*d[i]), C.byref(n))
        ref = np.array([r.x, r.y, r.z], np.float32)
        assert np.array_equal(ref.view(np.uint32), got[i].view(np.uint32)), i
        assert n.value == steps[i], i
