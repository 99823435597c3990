"""The GPU's world build at BASELINE.json's full sizes against the oracle's
own computation, whole grids.

Every full-size frame test renders with the oracle on the world the GPU
built (tests/test_gpu_fullsize.py); these tests make that world the oracle's
own first, and run before them (file order):

* whole-grid fixtures (tests/golden/world_hashes.json, made by
  tests/golden/make_world_hashes.py): the oracle builds each world from
  scratch -- bits from Evaluate (src/CArray.cu:8-30), the 3-pass CSDF
  (src/CoarseArray.cu:37-152), GI init (:211-245) and the GI sweeps the
  configurations render with (:273-355, deterministic per Appendix R5) -- for
  512^3 (C2), 1024^3 (C3 after 1 sweep, C4 after 2), 2048^3 (C5, 2 sweeps) and
  the reference's native 4096 x 512 x 4096 world (GI after the first
  UpdateGIData window); the GPU's exported grids must hash the same, whole;
* live oracle runs on this box, array_equal:
  - 512^3: the whole world (bits, CSDF, GI init, a sweep);
  - 1024^3: the whole CSDF from the GPU's bits, then GI init and C4's two
    sweeps over the whole grid, each stage from the oracle's previous one
    (never from the GPU's grid); bits in 8 spread 16-plane slabs;
  - 2048^3: CSDF z-slabs (a slab of coarse planes [z0, z1) depends only on the
    bits of coarse planes [z0 - 64, z1 + 64): or_csdf_build_slab), bit slabs,
    and GI init / both sweeps over whole cell planes.
"""
import numpy as np
import pytest

import world_golden as WG

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def _gpu_world(rv, atlas, log2, stages):
    """Build on the GPU; yield (label, exported array) for bits, csdf, gi_init
    and each GI stage (label, frame) after it (frame None: one UpdateGIData)."""
    r = rv.StateRender(log2, 64, 64, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
    r.world_build()
    r.sync()
    out = {"bits": r.world_export(rv.RV_WORLD_BITS), "csdf": r.world_export(rv.RV_WORLD_CSDF),
           "gi_init": r.world_export(rv.RV_WORLD_GI)}
    for label, frame in stages:
        if frame is None:
            r.update_gi_data()
        else:
            r.gi_update(frame)
        r.sync()
        out[label] = r.world_export(rv.RV_WORLD_GI)
    r.close()
    return out


STAGES = {"c2": [("gi_sweep1", 0)], "c4": [("gi_sweep1", 0), ("gi_sweep2", 1)],
          "c5": [("gi_sweep1", 0), ("gi_sweep2", 1)], "native": [("gi_window0", None)]}


@pytest.mark.parametrize("name", ["c2", "c4", "c5", "native"])
def test_world_grids_equal_oracle_whole_builds(rv, atlas, name):
    rec = WG.load()[name]
    g = _gpu_world(rv, atlas, tuple(rec["log2"]), STAGES[name])
    for label, a in g.items():
        WG.assert_grid(a, rec[label], f"{name} {label}")
    # the fixture's own record: what fraction of the CSDF is saturated air (SDF_MAX_DIST = 64)
    print(f"{name}: whole-grid hashes equal ({', '.join(g)}), csdf saturated {rec['csdf_saturated_frac']:.3f}")


def test_world_512_live_oracle_whole(rv, atlas, oracle):
    """512^3 (C2): the oracle builds the whole world here from scratch."""
    g = _gpu_world(rv, atlas, (9, 9, 9), STAGES["c2"])
    ow = oracle.OracleWorld(9, 9, 9, atlas=atlas).fill()
    assert np.array_equal(g["bits"], ow.bits)
    ow.build_csdf()
    assert np.array_equal(g["csdf"], ow.csdf)
    ow.gi_init()
    assert np.array_equal(g["gi_init"], ow.gi)
    ow.gi_update(0)
    assert np.array_equal(g["gi_sweep1"], ow.gi)


def test_world_1024_live_oracle_whole_csdf_gi(rv, atlas, oracle):
    """1024^3 (C3/C4): whole CSDF, GI init and C4's two sweeps by the oracle,
    each from its own previous stage; bits in spread slabs (a whole-world
    Evaluate is ~1 min of host time here; the fixture test covers it whole)."""
    g = _gpu_world(rv, atlas, (10, 10, 10), STAGES["c4"])
    ow = oracle.OracleWorld(10, 10, 10, atlas=atlas)
    for z0 in (0, 136, 272, 408, 544, 680, 816, 1008):
        ow.fill(z0, z0 + 16)
    planes = (1 << 20) // 32          # words per voxel plane
    for z0 in (0, 136, 272, 408, 544, 680, 816, 1008):
        sl = slice(z0 * planes, (z0 + 16) * planes)
        assert np.array_equal(g["bits"][sl], ow.bits[sl]), z0
    ow.bits[:] = g["bits"]
    ow.build_csdf()
    assert np.array_equal(g["csdf"], ow.csdf)
    ow.gi_init()
    assert np.array_equal(g["gi_init"], ow.gi)
    ow.gi_update(0)
    assert np.array_equal(g["gi_sweep1"], ow.gi)      # the grid C3 renders with
    ow.gi_update(1)
    assert np.array_equal(g["gi_sweep2"], ow.gi)      # the grid C4 renders with


def test_world_2048_live_oracle_slabs(rv, atlas, oracle):
    """2048^3 (C5): CSDF z-slabs from the GPU's bits with their 64-plane halo,
    voxel slabs, and GI init / both sweeps over whole cell planes (each sweep's
    cells from the GPU's previous grid, which the fixture test pins whole)."""
    g = _gpu_world(rv, atlas, (11, 11, 11), STAGES["c5"])
    ow = oracle.OracleWorld(11, 11, 11, atlas=atlas)
    planes = (1 << 22) // 32
    for z0 in (0, 1000, 2040):
        ow.fill(z0, z0 + 8)
        sl = slice(z0 * planes, (z0 + 8) * planes)
        assert np.array_equal(g["bits"][sl], ow.bits[sl]), z0
    ow.bits[:] = g["bits"]
    cplane = 1024 * 1024
    for cz0, cz1 in ((0, 24), (600, 624)):        # the z = 0 face (Appendix R3) and an interior slab
        ow.build_csdf(cz0, cz1)
        sl = slice(cz0 * cplane, cz1 * cplane)
        assert np.array_equal(g["csdf"][sl], ow.csdf[sl]), (cz0, cz1)
    ow.csdf[:] = g["csdf"]
    gplane = 512 * 512
    cells = [(0, 2), (300, 302), (510, 512)]       # GI cell z-planes
    for stage, frame in (("gi_init", None), ("gi_sweep1", 0), ("gi_sweep2", 1)):
        if frame is not None:
            ow.gi[:] = g["gi_init" if frame == 0 else "gi_sweep1"]
        for z0, z1 in cells:
            if frame is None:
                ow.gi_init(first=z0 * gplane, count=(z1 - z0) * gplane)
            else:
                ow.gi_update(frame, first=z0 * gplane, count=(z1 - z0) * gplane)
            sl = slice(4 * z0 * gplane, 4 * z1 * gplane)
            assert np.array_equal(g[stage][sl], ow.gi[sl]), (stage, z0)
