"""The product's traversal source (include/rvgrt/rv_device.h) compiled for
the CPU (tests/host/rv_host_trace.cpp) against the oracle: hit, position,
normal, uv and sphere/DDA/check step counts bit-exact on random rays, for
every traversal variant the GPU kernels can select (DDA look-ahead group
1/2/4/8 by stop search + re-walk, word reuse, the step-by-step replay).
Runs without a GPU; the GPU build of the same source is checked by
tests/test_gpu_parity.py::test_trace_bit_exact."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import random_rays

HERE = os.path.dirname(os.path.abspath(__file__))
HOST = os.path.join(HERE, "host")
HIT = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("u", "<f4"), ("v", "<f4"), ("hit", "<i4"),
                ("undef", "<i4"), ("sphere", "<i4"), ("dda", "<i4"), ("check", "<i4"), ("pad", "<i4")])


VARIANTS = {"g1": 0, "g2": 1, "g4": 2, "g8": 3, "g1_reuse": 4, "g4_replay": 5, "g8_replay": 6}


SAN = os.environ.get("RVGRT_SANITIZE") == "1"   # tests/test_sanitizers.py: the ASan + UBSan build


@pytest.fixture(scope="module")
def host_lib():
    subprocess.run(["make", "-s", "-C", HOST] + (["san"] if SAN else []), check=True)
    L = C.CDLL(os.path.join(HOST, "build", "librvhost_san.so" if SAN else "librvhost.so"))
    L.rvh_trace_rays.restype = C.c_int
    L.rvh_trace_rays.argtypes = [C.c_int] * 4 + [C.c_void_p] * 5 + [C.c_int64, C.c_void_p]
    assert L.rvh_variants() == len(VARIANTS)
    return L


def _trace(L, variant, ow, org, d, dist):
    out = np.zeros(len(dist), HIT)
    p = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    assert L.rvh_trace_rays(variant, ow.lx, ow.ly, ow.lz, p(ow.bits), p(ow.csdf), p(org), p(d), p(dist),
                            len(dist), p(out)) == 0
    return out


@pytest.mark.parametrize("dims", [(7, 7, 7), (8, 6, 7)])
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_host_trace_bit_exact(host_lib, oracle_world, dims, variant):
    ow = oracle_world(*dims, gi_sweeps=0)
    rng = np.random.default_rng(4321)
    org, d, dist = random_rays(rng, 20000, (ow.X, ow.Y, ow.Z))
    g = _trace(host_lib, VARIANTS[variant], ow, org, d, dist)
    o = ow.trace_batch(org, d, dist)
    assert (g["hit"] == o["hit"]).all()
    assert (g["undef"] == o["undef"]).all()
    assert np.array_equal(g["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(g["normal"], o["normal"])
    assert np.array_equal(g["u"].view(np.uint32), o["u"].view(np.uint32))
    assert np.array_equal(g["v"].view(np.uint32), o["v"].view(np.uint32))
    assert np.array_equal(g["sphere"], o["n_sphere"])
    assert np.array_equal(g["dda"], o["n_dda"])
    assert np.array_equal(g["check"], o["n_check"])
    assert g["hit"].mean() > 0.2 and (g["dda"] > 100).any()


def test_u8f_equals_ieee_division(host_lib):
    """rv::u8f (mul by RN(1/255) + one fma residual step), which the kernels
    use for every RGBA8 -> float conversion, equals the correctly rounded
    float32 division b / 255 of the reference (src/raytracing_functions.cu:59,
    :256-262, src/CoarseArray.cu:324-351) for all 256 bytes."""
    host_lib.rvh_u8f.restype = C.c_float
    host_lib.rvh_u8f.argtypes = [C.c_uint32]
    got = np.array([host_lib.rvh_u8f(b) for b in range(256)], np.float32)
    want = np.arange(256, dtype=np.float32) / np.float32(255.0)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_simplex3d_equals_oracle(host_lib):
    """rv::simplex3D (the corners' hash products strength-reduced from the
    base corner's) equals the oracle's simplex3D (include/TerrainGeneration.cuh:
    178-254) bit for bit on 200k points: texture-noise scale, water scale,
    world scale, negative and lattice-aligned coordinates."""
    from oracle import oracle as O
    rng = np.random.default_rng(77)
    pts = np.concatenate([rng.uniform(-3000, 3000, (100000, 3)) * 0.05 * 0.3,
                          rng.uniform(-2000, 2000, (50000, 3)) * 0.06,
                          rng.uniform(-4096, 4096, (40000, 3)) * 0.002,
                          rng.integers(-500, 500, (10000, 3)).astype(np.float64)]).astype(np.float32)
    got = np.empty(len(pts), np.float32)
    host_lib.rvh_simplex3D.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    host_lib.rvh_simplex3D(pts.ctypes.data, got.ctypes.data, len(pts))
    want = np.empty(len(pts), np.float32)
    O.lib().or_simplex3D_batch(np.ascontiguousarray(pts).ctypes.data, want.ctypes.data, len(pts))
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_texture_tile_table_equals_noise(host_lib):
    """World::tex (rv_device.h tex_index / tex_table_entry, built once per context by k_tex_table over
    the rows below the sky exit) gives the atlas tile sampleTexture's noise picks (src/raytracing_functions.cu:41-54) for every
    hit position: lattice points, faces (integral coordinates), the carry boundaries of the +121.3 /
    +1321.3 / +721.5 offsets (fractions near 0.7 and 0.5), the world's far faces and outside
    positions (the kernels then evaluate the noise)."""
    rng = np.random.default_rng(5)
    lx, ly, lz = 5, 4, 6
    dims = np.array([32, 16, 64], np.float64)
    n = 60000
    p = rng.uniform(0, 1, (n, 3)) * dims
    k = n // 6
    p[:k] = np.floor(p[:k])                                          # lattice points
    p[k:2 * k, 0] = np.floor(p[k:2 * k, 0])                          # face hits
    fr = np.array([0.7, 0.7, 0.5])
    for j in range(3):                                               # carry boundaries +- a few ulp
        s = slice((2 + j) * k, (3 + j) * k)
        base = np.floor(p[s]) + fr
        p[s] = np.nextafter(base.astype(np.float32), rng.choice([-np.inf, np.inf], base.shape)).astype(np.float64)
    p[5 * k:5 * k + 500] = dims - rng.uniform(0, 1e-4, (500, 3))     # the far faces
    p[5 * k + 500:5 * k + 1000] = dims + rng.uniform(0, 3, (500, 3))  # outside: noise path
    p[5 * k + 1000:5 * k + 1500] = -rng.uniform(0, 3, (500, 3))
    pts = np.ascontiguousarray(p.astype(np.float32))
    host_lib.rvh_texture_tiles.argtypes = [C.c_int] * 4 + [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    for ny in (0, 8):   # the whole world; a band of the lowest 8 rows (the rest: noise)
        tab = np.full(n, -1, np.int32)
        noi = np.full(n, -2, np.int32)
        host_lib.rvh_texture_tiles(lx, ly, lz, ny, pts.ctypes.data, n, tab.ctypes.data, noi.ctypes.data)
        assert np.array_equal(tab, noi), ny
        assert len(np.unique(noi)) >= 3                             # several tiles exercised


@pytest.mark.parametrize("variant", ["g1", "g4", "g8", "g4_replay"])
def test_sky_exit_keeps_every_hit(host_lib, oracle_world, variant):
    """The frame kernels' sky exit (World::ytop, rv_device.h trace): a ray
    with dir.y >= 0 that has risen to the highest solid row + 2 stops as a
    miss.  Every ray's result -- hit, undefined hit, position, normal, uv --
    equals the oracle's (the reference's full march); only the step counts
    shrink.  Rays start anywhere, half of them pointing up, on a 128^3 world
    whose terrain leaves open sky above it."""
    L = host_lib
    L.rvh_trace_rays_sky_exit.restype = C.c_int
    L.rvh_trace_rays_sky_exit.argtypes = [C.c_int] * 4 + [C.c_void_p] * 5 + [C.c_int64, C.c_void_p, C.c_void_p]
    from oracle import oracle as O
    ow = O.OracleWorld(7, 7, 7).build(gi_sweeps=-1)
    # open sky above the terrain: clear every voxel row from y = 90 up, then the CSDF again
    vox = ow.voxels()
    vox[:, 90:, :] = False
    ow.bits[:] = np.packbits(vox.ravel(), bitorder="little").view(np.uint32)
    ow.build_csdf()
    rng = np.random.default_rng(77)
    org, d, dist = random_rays(rng, 30000, (ow.X, ow.Y, ow.Z))
    up = rng.random(len(d)) < 0.5
    d[up, 1] = np.abs(d[up, 1])
    d[:200, 1] = 0.0                       # horizontal rays (dir.y == 0: y stays constant)
    d[200:400, 1] = -0.0
    g = np.zeros(len(dist), HIT)
    ytop = C.c_uint32()
    p = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    assert L.rvh_trace_rays_sky_exit(VARIANTS[variant], ow.lx, ow.ly, ow.lz, p(ow.bits), p(ow.csdf), p(org), p(d),
                                     p(dist), len(dist), p(g), C.byref(ytop)) == 0
    o = ow.trace_batch(org, d, dist)
    assert ytop.value == 1 + int(np.flatnonzero(vox.any(axis=(0, 2))).max()) + 1   # highest solid row + 2
    assert (g["hit"] == o["hit"]).all() and (g["undef"] == o["undef"]).all()
    assert np.array_equal(g["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(g["normal"], o["normal"])
    assert np.array_equal(g["u"].view(np.uint32), o["u"].view(np.uint32))
    assert np.array_equal(g["v"].view(np.uint32), o["v"].view(np.uint32))
    assert (g["sphere"] <= o["n_sphere"]).all()
    assert g["sphere"].sum() < 0.9 * o["n_sphere"].sum()   # the exit does cut the march
    assert g["hit"].mean() > 0.2


@pytest.mark.parametrize("g8", [0, 1])
@pytest.mark.parametrize("sky", ["cut", "full"])
def test_sun_exit_keeps_every_shadow_hit(host_lib, oracle_world, g8, sky):
    """The shadow rays' sun exit (trace_sun with World::horizon, built per 2x2-voxel
    column from the column tops for the sun direction, rv_device.h
    horizon_column): a ray toward the sun stops as a miss once it is above its
    column's horizon.  Shadow rays from the voxel surfaces (as the pre-pass,
    the reflection shadow and the GI update cast them) and from anywhere in the
    world give the oracle's hit / miss, position, normal and uv exactly, with
    fewer sphere steps -- on the full 128^3 terrain (no sky above it) and with
    open sky above row 90."""
    from oracle import oracle as O
    L = host_lib
    L.rvh_trace_sun.restype = C.c_int
    L.rvh_trace_sun.argtypes = [C.c_int] * 4 + [C.c_void_p] * 5 + [C.c_int64, C.c_void_p, C.c_void_p]
    ow = O.OracleWorld(7, 7, 7).build(gi_sweeps=-1)
    if sky == "cut":
        vox = ow.voxels()
        vox[:, 90:, :] = False
        ow.bits[:] = np.packbits(vox.ravel(), bitorder="little").view(np.uint32)
        ow.build_csdf()
    sun = np.ascontiguousarray(O.sun_dir(), np.float32)
    rng = np.random.default_rng(9)
    # surface points: primary hits of random rays, offset along the normal as the kernels do
    org0, d0, dist0 = random_rays(rng, 40000, (ow.X, ow.Y, ow.Z))
    h0 = ow.trace_batch(org0, d0, dist0)
    sel = (h0["hit"] != 0) & (h0["undef"] == 0)
    surf = (h0["pos"][sel] + h0["normal"][sel] * np.float32(0.1)).astype(np.float32)
    org = np.ascontiguousarray(np.concatenate([surf, org0[:10000]]), np.float32)
    dist = np.zeros(len(org), np.float32)
    dirs = np.ascontiguousarray(np.broadcast_to(sun, org.shape), np.float32)
    g = np.zeros(len(org), HIT)
    hz = np.zeros((ow.Z // 2) * (ow.X // 2), np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    assert L.rvh_trace_sun(g8, ow.lx, ow.ly, ow.lz, p(ow.bits), p(ow.csdf), p(sun), p(org), p(dist), len(org), p(g),
                           p(hz)) == 0
    o = ow.trace_batch(org, dirs, dist)
    assert (g["hit"] == o["hit"]).all() and (g["undef"] == o["undef"]).all()
    assert np.array_equal(g["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(g["normal"], o["normal"])
    assert np.array_equal(g["u"].view(np.uint32), o["u"].view(np.uint32))
    assert np.array_equal(g["v"].view(np.uint32), o["v"].view(np.uint32))
    assert (g["sphere"] <= o["n_sphere"]).all()
    assert 0.1 < o["hit"].mean() < 0.9                      # shadowed and lit points both
    assert g["sphere"].sum() < 0.8 * o["n_sphere"].sum()    # the horizon does cut the march
    assert hz.min() < hz.max()                               # the horizon varies over the terrain


@pytest.mark.parametrize("g8", [0, 1])
def test_column_skip_keeps_every_hit(host_lib, g8):
    """The DDA's empty-column skip (trace COL = true, rv_device.h; the water reflections of the pipelined
    and grouped launches): a look-ahead group whose lowest row is at or above the highest solid row of the
    3x3 brick columns around its first cell issues no voxel gathers.  Rays that skim just above the terrain
    -- ascending, level and descending (the iy - G bound), from the surface tops and from the water plane
    at grazing angles -- give the same hit, position, normal, uv and step counts as the same traversal
    without the skip (both with the sky exit and the dtop table built as rv_abi.cpp's world_top builds
    it), and the oracle's hits; the skip must fire on a good share of the groups."""
    from oracle import oracle as O
    L = host_lib
    L.rvh_trace_col.restype = C.c_int
    L.rvh_trace_col.argtypes = [C.c_int] * 5 + [C.c_void_p] * 5 + [C.c_int64, C.c_void_p]
    ow = O.OracleWorld(7, 7, 7).build(gi_sweeps=-1)
    vox = ow.voxels()                                         # [z, y, x]
    top = np.where(vox.any(axis=1), ow.Y - 1 - np.argmax(vox[:, ::-1, :], axis=1), 0)   # highest solid y per (z, x)
    rng = np.random.default_rng(21)
    n = 12000
    x = rng.integers(0, ow.X, n)
    z = rng.integers(0, ow.Z, n)
    org = np.stack([x + rng.uniform(0, 1, n), top[z, x] + 1 + rng.uniform(0.05, 4.0, n), z + rng.uniform(0, 1, n)],
                   1).astype(np.float32)
    water = rng.uniform(size=n) < 0.3                         # reflection-like starts on the water plane
    org[water, 1] = np.float32(31.0) + rng.uniform(0.0, 1.0, water.sum()).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[:, 1] = rng.uniform(-0.25, 0.25, n) * np.hypot(d[:, 0], d[:, 2])   # grazing, up and down
    d[rng.uniform(size=n) < 0.05, 1] = 0.0                                 # exactly level
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    dist = np.zeros(n, np.float32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)   # noqa: E731
    out = []
    for col in (1, 0):
        g = np.zeros(n, HIT)
        assert L.rvh_trace_col(g8, col, ow.lx, ow.ly, ow.lz, p(ow.bits), p(ow.csdf), p(np.ascontiguousarray(org)),
                               p(np.ascontiguousarray(d)), p(dist), n, p(g)) == 0
        out.append(g)
    a, b = out
    for k in ("hit", "undef", "sphere", "dda", "check"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("pos", "normal", "u", "v"):
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k
    o = ow.trace_batch(org, d, dist)
    assert np.array_equal(a["hit"], o["hit"]) and np.array_equal(a["undef"], o["undef"])
    assert np.array_equal(a["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(a["normal"], o["normal"])
    assert np.array_equal(a["u"].view(np.uint32), o["u"].view(np.uint32))
    assert np.array_equal(a["v"].view(np.uint32), o["v"].view(np.uint32))
    skipped = a["pad"].sum()                                    # col_skip: groups known empty
    groups = (a["dda"].astype(np.int64) + (8 if g8 else 4) - 1) // (8 if g8 else 4)
    assert b["pad"].sum() == 0 and skipped > 0.05 * groups.sum(), (skipped, groups.sum())
    desc = d[:, 1] < 0
    assert a["pad"][desc].sum() > 0 and a["pad"][~desc].sum() > 0   # both branches of the row bound fire
