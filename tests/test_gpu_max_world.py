"""The largest world rv_create accepts: 2^34 voxels (4096 x 1024 x 4096), whose brick records fill
the 32-bit gather offsets exactly (bits 2 GiB + CSDF 2 GiB; the sun horizon and column tops lie past
4 GiB in the same allocation), twice the reference's native 4096 x 512 x 4096.

The GPU builds the world and renders a reference frame; the oracle checks it without building the
whole world itself (minutes of CPU): voxel planes at the bottom, middle and top against its own
Evaluate, a CSDF slab and a range of GI-init cells recomputed from the GPU's exported bits, and frame
rows rendered on the GPU's exported world -- all bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dims", [(12, 10, 12), (13, 8, 13)], ids=["4096x1024x4096", "8192x256x8192"])
def test_max_world_build_and_frame(rv, atlas, oracle, dims):
    lx, ly, lz = dims
    W, H = 1920, 1080
    r = rv.StateRender(dims, W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
    try:
        r.world_build()
        bits = r.world_export(rv.RV_WORLD_BITS)
        X, Y, Z = 1 << lx, 1 << ly, 1 << lz
        assert bits.size == X * Y * Z // 32
        wpz = X * Y // 32                                   # bit words per z plane
        ow = oracle.OracleWorld(lx, ly, lz, atlas=atlas)
        for z0 in (0, Z // 2 - 4, Z - 8):
            ow.fill(z0, z0 + 8)
            sl = slice(z0 * wpz, (z0 + 8) * wpz)
            assert np.array_equal(bits[sl], ow.bits[sl]), f"voxel planes {z0}..{z0 + 8}"
        assert bits[(Z // 2) * wpz:(Z // 2 + 1) * wpz].any()

        # CSDF slab and GI init from the GPU's own bits
        ow.bits[:] = bits
        del bits
        csdf = r.world_export(rv.RV_WORLD_CSDF)
        cz0, cz1 = Z // 4 - 4, Z // 4 + 4                    # coarse planes
        ow.build_csdf(cz0, cz1)
        cpz = (X // 2) * (Y // 2)
        sl = slice(cz0 * cpz, cz1 * cpz)
        assert np.array_equal(csdf[sl], ow.csdf[sl]), "CSDF slab"
        ow.csdf[:] = csdf
        del csdf
        gi = r.world_export(rv.RV_WORLD_GI)
        ncell = len(gi) // 4
        first, count = ncell // 2, 60000
        ow.gi_init(first=first, count=count)
        g = gi.reshape(-1, 4)[first:first + count]
        assert np.array_equal(g, ow.gi.reshape(-1, 4)[first:first + count]), "GI init cells"
        assert (g[:, 0] != 0).any()
        ow.gi[:] = gi
        del gi

        # a reference frame: rows against the oracle on the same world
        pos = (0.1 * X, min(350.0, 0.9 * Y), 0.1 * Z)
        cam, vp = rv.camera_from_pose(pos, -0.7, -np.pi - 0.3, W, H)
        r.frame(cam, vp, flags=rv.RV_FLAGS_REFERENCE)
        img = r.readback(rv.RV_IMAGE_COLOR)
        rows = np.arange(3, H, 97)
        ref = oracle.render_rows(ow, oracle.make_frame(W, H, rv.RV_FLAGS_REFERENCE, rv.camera_dict(cam, vp)), rows,
                                 want_stats=False)
        assert np.array_equal(img[rows], ref["rgba"][rows])
        assert len(np.unique(img[rows].reshape(-1, 4), axis=0)) > 50       # terrain, water and sky
    finally:
        r.close()


@pytest.mark.parametrize("dims", [(4, 4, 4), (4, 11, 4), (9, 4, 5)], ids=["16^3", "16x2048x16", "512x16x32"])
def test_smallest_and_thinnest_worlds(rv, atlas, oracle, dims):
    """The smallest world (16^3: two bricks a side, GI grid 4^3) and one-brick-thin ones: the whole
    world (bits, CSDF, GI init and a sweep) and whole reference frames equal the oracle's own build."""
    lx, ly, lz = dims
    W, H = 96, 64
    ow = oracle.OracleWorld(lx, ly, lz, atlas=atlas).build(gi_sweeps=1)
    r = rv.StateRender(dims, W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas)
    try:
        r.world_build()
        r.gi_update(0)
        assert np.array_equal(r.world_export(rv.RV_WORLD_BITS), ow.bits)
        assert np.array_equal(r.world_export(rv.RV_WORLD_CSDF), ow.csdf)
        assert np.array_equal(r.world_export(rv.RV_WORLD_GI), ow.gi)
        X, Y, Z = ow.X, ow.Y, ow.Z
        for pos in ((0.5 * X, min(0.9 * Y, 60.0), 0.5 * Z), (-3.0, 0.5 * Y, -3.0)):
            cam, vp = rv.camera_from_pose(pos, -0.7, -np.pi - 0.3, W, H)
            r.frame(cam, vp, flags=rv.RV_FLAGS_REFERENCE)
            ref = oracle.render(ow, oracle.make_frame(W, H, rv.RV_FLAGS_REFERENCE, rv.camera_dict(cam, vp)),
                                want_stats=False)
            assert np.array_equal(r.readback(rv.RV_IMAGE_COLOR), ref["rgba"]), pos
            assert np.array_equal(r.readback(rv.RV_IMAGE_MOTION), ref["mv"]), pos
            assert np.array_equal(r.readback(rv.RV_IMAGE_DEPTH), ref["depth"]), pos
    finally:
        r.close()
