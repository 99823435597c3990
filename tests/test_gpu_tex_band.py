"""The texture tile table over the rows below the sky exit (rv_device.h tex_index, World::tex_ny).

The table is built once per context, for the world of its first build or bits import, and covers the
rows below that world's sky exit; it is kept through later world writes.  A later world that rises
above those rows must still render exactly: its hits above the table's rows take sampleTexture's noise
(src/raytracing_functions.cu:41-54), as hits outside the world do.  Checked against a context without
the table (rv_config.tex_table = -1), which evaluates the noise for every hit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rv():
    import rvgrt_amd
    rvgrt_amd._lib.load()
    return rvgrt_amd


def _bits(vox):
    return np.packbits(vox.ravel(), bitorder="little").view(np.uint32)


def test_rows_above_the_table_take_the_noise(rv, atlas, oracle_world, monkeypatch):
    from rvgrt_amd.configs import TEST_POSES_128
    ow = oracle_world(7, 7, 7, gi_sweeps=0)
    low = ow.voxels().copy()            # (z, y, x)
    low[:, 41:, :] = False              # solid rows 0..40: sky exit 42, table rows 0..47
    tall = low.copy()
    tall[:, 40:100, 20:28] = True       # walls up to row 99 on two sides of the world
    tall[20:28, 40:100, :] = True
    W, H = 192, 128

    def context(table):
        r = rv.StateRender((7, 7, 7), W, H, flags=rv.RV_FLAGS_REFERENCE, atlas=atlas, tex_table=0 if table else -1)
        r.world_import(rv.RV_WORLD_BITS, _bits(low))   # the table's world
        return r

    def frames(r, vox):
        r.world_import(rv.RV_WORLD_BITS, _bits(vox))
        r.csdf_build()
        r.gi_init()
        out = []
        for pose in ("P0", "P1"):
            cam, vp = rv.camera_from_pose(*TEST_POSES_128[pose], W, H)
            r.frame(cam, vp)
            out.append(r.readback(rv.RV_IMAGE_COLOR).copy())
        return out

    with_table, without = context(True), context(False)
    assert with_table.tex_table_info() == (True, 128 * 48 * 128 * 4)
    assert without.tex_table_info() == (False, 0)
    low_frames = frames(with_table, low)
    tall_frames = frames(with_table, tall)
    assert all(not np.array_equal(a, b) for a, b in zip(low_frames, tall_frames))   # the walls are in view
    assert with_table.tex_table_info() == (True, 128 * 48 * 128 * 4)              # kept through the rebuild
    for a, b in zip(tall_frames, frames(without, tall)):
        assert np.array_equal(a, b)
    with_table.close()
    without.close()
