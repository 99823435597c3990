"""R9: the SURVEY.md s8c tolerance holds between the no-contraction oracle
and emulations of the arithmetic the reference actually compiles to (nvcc
--fmad=true FMA contraction, CUDA's <= 2-ulp tanf/powf); see
oracle/r9_study.py and DESIGN.md s3.  The full report over C1 and the
128^3/256^3 reference frames is tools/r9_report.py ->
profiles/r03/r9_numerics.json."""
import pytest

from rvgrt_amd.configs import CONFIGS, TEST_POSES_128, pose_f32

REF = 1 | 2 | 4   # prepass, water, GI


@pytest.fixture(scope="module")
def study(oracle, atlas):
    from oracle import r9_study as S
    return S


def _cases():
    yield "c1_whole", 8, 0, 640, 360, 0, pose_f32(CONFIGS["c1"], "P0")
    for p in ("P0", "P1"):
        yield f"128_ref_{p}", 7, 1, 320, 180, REF, TEST_POSES_128[p]
    pos, yaw, pitch = TEST_POSES_128["P1"]
    yield "256_ref_P1", 8, 1, 640, 360, REF, (tuple(2 * v for v in pos), yaw, pitch)


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_tolerance_holds_under_reference_arithmetic(study, atlas, case):
    name, lg, sweeps, W, H, flags, pose = case
    wd, res = study.study(lg, sweeps, W, H, flags, pose, atlas)
    for build, d in wd.items():
        # the noise never crosses the 0.7 solidity threshold under contraction here
        assert d["voxels_flipped"] == 0 and d["csdf_cells_diff"] == 0, (build, d)
    for v, m in res.items():
        assert study.tolerance_ok(m), (name, v, m)
    # the contraction builds really compute something else (the study is not vacuous)
    assert res["fma_gcc"]["rgba_exact"] < 1.0 and res["fma_clang"]["rgba_exact"] < 1.0
    if flags & 4:
        assert wd["fma_gcc"]["gi_cells_diff"] > 0


def test_study_builds_contract(oracle):
    assert oracle.lib().or_numerics_contracted() == 0
    for v in ("fma_gcc", "fma_clang"):
        with oracle.numerics(v) as L:
            assert L.or_numerics_contracted() == 1


@pytest.mark.parametrize("pose", ["P0", "P1"])
def test_tolerance_holds_after_64_gi_updates(study, atlas, pose):
    """R9 over the GI feedback loop: 64 UpdateGIData frames (each a whole sweep
    of the 32^3 grid: RAYPS 262144 >= its 32768 cells), every update reading
    the grid the previous ones wrote, on worlds built and updated with the
    contracted arithmetic; the reference frame rendered on each build's grid
    after frame 64 stays within the SURVEY s8c tolerance of the plain oracle's
    (profiles/r04/r9_long_gi.json has the per-frame curve at 128^3 and
    256^3)."""
    curve = study.long_gi_sequence(7, 1, 64, 320, 180, REF, TEST_POSES_128[pose], atlas, render_at=[1, 64])
    assert len(curve) == 64
    for b, m in curve[-1]["render"].items():
        assert study.tolerance_ok(m), (pose, b, m)
    # the contracted grids really differ (the loop is not vacuous) and the difference stays a small
    # fraction of the grid
    for b, nd in curve[-1]["gi_cells_diff"].items():
        assert 0 < nd <= 0.05 * curve[-1]["gi_cells"], (b, nd)
