"""Known-answer tests of the DDA / sphere-march traversal (oracle trace(),
src/raytracing_functions.cu:65-202) on hand-built scenes, and a bit-exact
cross-check against the independent scalar restatement in np_ref.trace_py."""
import numpy as np
import pytest

import np_ref as R


def _world(oracle, atlas, lg=5):
    return oracle.OracleWorld(lg, lg, lg, atlas=atlas)


def _trace(w, o, d, dist=0.0):
    return w.trace_batch(np.array([o], np.float32), np.array([d], np.float32), np.array([dist], np.float32))[0]


def test_empty_world_misses(oracle, atlas):
    w = _world(oracle, atlas)
    w.build_csdf()
    for d in [(1, 0, 0), (0, -1, 0), (0.3, 0.4, -0.866)]:
        h = _trace(w, (16.5, 16.5, 16.5), d)
        assert h["hit"] == 0 and not h["undef"]
        assert list(h["pos"]) == [-500.0, -500.0, -500.0]


def test_single_voxel_axis_rays(oracle, atlas):
    w = _world(oracle, atlas)
    w.set_solid(20, 10, 10)
    w.build_csdf()
    # +x ray through the voxel's centre line from x = 4.25
    h = _trace(w, (4.25, 10.5, 10.5), (1, 0, 0))
    assert h["hit"] == 1 and not h["undef"]
    assert list(h["normal"]) == [-1.0, 0.0, 0.0]
    assert list(h["pos"]) == [20.0, 10.5, 10.5]          # enters the x = 20 face
    assert (h["u"], h["v"]) == (0.5, 0.5)
    # -y ray from above lands on the top face y = 11
    h = _trace(w, (20.25, 28.75, 10.5), (0, -1, 0))
    assert h["hit"] == 1 and list(h["normal"]) == [0.0, 1.0, 0.0]
    assert h["pos"][1] == 11.0
    # -z ray: normal +z, uv.x flipped only for step.z == +1
    h = _trace(w, (20.75, 10.25, 30.5), (0, 0, -1))
    assert h["hit"] == 1 and list(h["normal"]) == [0.0, 0.0, 1.0]
    assert h["pos"][2] == 11.0
    assert h["u"] == np.float32(0.75) and h["v"] == np.float32(0.25)
    h = _trace(w, (20.75, 10.25, 1.5), (0, 0, 1))
    assert h["hit"] == 1 and list(h["normal"]) == [0.0, 0.0, -1.0]
    assert h["u"] == np.float32(0.25)                    # 1 - 0.75
    # a ray that passes beside the voxel misses
    h = _trace(w, (4.25, 12.5, 10.5), (1, 0, 0))
    assert h["hit"] == 0


def test_start_inside_solid_is_reference_undefined_hit(oracle, atlas):
    """mask == -128 hit (Appendix R2): hit=true, pos stays (-500)^3."""
    w = _world(oracle, atlas)
    w.set_solid(8, 8, 8)
    w.build_csdf()
    h = _trace(w, (8.5, 8.5, 8.5), (0.6, 0.0, 0.8))
    assert h["hit"] == 1 and h["undef"] == 1
    assert list(h["pos"]) == [-500.0, -500.0, -500.0]
    assert list(h["normal"]) == [0.0, 0.0, 0.0]


def test_out_of_bounds_origin_misses(oracle, atlas):
    w = _world(oracle, atlas)
    w.set_solid(3, 3, 3)
    w.build_csdf()
    h = _trace(w, (-1.0, 3.5, 3.5), (1, 0, 0))
    assert h["hit"] == 0                                   # sphere march returns (-100)^3
    h = _trace(w, (3.5, 3.5, 40.0), (0, 0, -1))
    assert h["hit"] == 0


def test_negative_start_distance_moves_origin_back(oracle, atlas):
    w = _world(oracle, atlas)
    w.set_solid(10, 5, 5)
    w.build_csdf()
    h = _trace(w, (12.5, 5.5, 5.5), (1, 0, 0), dist=-3.0)   # starts at x = 9.5, just before the voxel
    assert h["hit"] == 1 and list(h["pos"]) == [10.0, 5.5, 5.5]


def test_dda_gives_up_after_200_steps(oracle, atlas):
    """A wall at the end of a corridor next to a rail: the CSDF reads 1 along
    the corridor, so the sphere march stops at once and the DDA never jumps;
    the 200-step DDA limit then turns a reachable wall into a miss."""
    lg = 8
    w = oracle.OracleWorld(lg, 5, 5, atlas=atlas)
    for x in range(0, 256):
        w.set_solid(x, 15, 16)                         # a solid rail next to the corridor
    w.set_solid(250, 16, 16)                           # the target
    w.build_csdf()
    near = _trace(w, (200.5, 16.5, 16.5), (1, 0, 0))
    assert near["hit"] == 1 and near["pos"][0] == 250.0
    far = _trace(w, (20.5, 16.5, 16.5), (1, 0, 0))
    assert far["hit"] == 0 and far["n_dda"] == 200


def test_trace_matches_scalar_restatement(oracle, oracle_world):
    w = oracle_world(6, 6, 6, gi_sweeps=-1)
    vox = w.voxels()
    cs = w.csdf.reshape(w.Z // 2, w.Y // 2, w.X // 2)
    rng = np.random.default_rng(5)
    from conftest import random_rays
    org, d, dist = random_rays(rng, 300, (w.X, w.Y, w.Z))
    o = w.trace_batch(org, d, dist)
    for k in range(len(dist)):
        ref = R.trace_py(lambda x, y, z: vox[z, y, x], lambda cx, cy, cz: int(cs[cz, cy, cx]),
                         (w.X, w.Y, w.Z), org[k], d[k], R.hround(dist[k]))
        hit, undef, pos, nrm, u, v = ref
        assert bool(o[k]["hit"]) == hit, k
        assert bool(o[k]["undef"]) == undef, k
        if hit:
            assert np.array_equal(np.array(pos, np.float32).view(np.uint32), o[k]["pos"].view(np.uint32)), k
            assert np.array_equal(np.array(nrm, np.float32), o[k]["normal"]), k
            assert np.float32(u) == o[k]["u"] and np.float32(v) == o[k]["v"], k
    assert o["hit"].mean() > 0.2
