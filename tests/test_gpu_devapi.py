"""The reference-signature device API (include/rvgrt_device.h) on the GPU.

Kernels written the way the reference's call its __device__ functions
(trace(float3, float3, half, bits, csdf) -> hitInfo, approximateCSDF,
traceCone x2, sampleTexture, sampleSky, IsSolid, getDistance x2;
include/raytracing_functions.cuh:14-84) run over reference-layout buffers
(x-fastest bit words, linear CSDF, uchar4 GI) of a 128 x 64 x 128 world and
are compared bit for bit with the CPU oracle on the same world.  The test
harness tests/devapi/librvgrt_devapi_test.so is built by build().
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import random_rays

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "devapi", "build", "librvgrt_devapi_test.so")
DIMS = (7, 6, 7)

HITINFO = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("uv", "<u2", 2), ("hit", "u1"),
                    ("pad", "u1", 3), ("its", "<i4")])


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def load():
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
    L = C.CDLL(LIB)
    for name in ("rvt_trace", "rvt_approx", "rvt_cone", "rvt_texture", "rvt_sky", "rvt_lookup", "rvt_dims",
                 "rvt_frame"):
        getattr(L, name).restype = C.c_int
    return L


def test_devapi_library_exports_and_layout():
    """CPU: the harness loads, exports its entry points and was built for the
    test world; hitInfo is the reference's 36 bytes."""
    L = load()
    d = (C.c_int * 3)()
    assert L.rvt_dims(d) == 36 == HITINFO.itemsize
    assert tuple(d) == DIMS


@pytest.fixture(scope="module")
def world(oracle_world):
    return oracle_world(*DIMS, gi_sweeps=1)


@pytest.mark.gpu
def test_devapi_trace_bit_exact(world):
    L = load()
    rng = np.random.default_rng(99)
    org, dirs, dist = random_rays(rng, 20000, (world.X, world.Y, world.Z))
    out = np.zeros(len(dist), HITINFO)
    rc = L.rvt_trace(_p(world.bits), C.c_size_t(world.bits.nbytes), _p(world.csdf), C.c_size_t(world.csdf.nbytes),
                     _p(org), _p(dirs), _p(dist), len(dist), _p(out))
    assert rc == 0, f"hip error {rc}"
    o = world.trace_batch(org, dirs, dist)
    assert np.array_equal(out["hit"].astype(bool), o["hit"].astype(bool))
    assert np.array_equal(out["pos"].view(np.uint32), o["pos"].view(np.uint32))
    assert np.array_equal(out["normal"], o["normal"])
    uv = out["uv"].view(np.float16).astype(np.float32)
    assert np.array_equal(uv[:, 0], o["u"]) and np.array_equal(uv[:, 1], o["v"])
    assert np.array_equal(out["its"], o["its"])          # major + DDA loop entries, as the reference counts
    assert out["hit"].mean() > 0.2


@pytest.mark.gpu
def test_devapi_approximate_csdf(world, oracle):
    L = load()
    rng = np.random.default_rng(5)
    org, dirs, _ = random_rays(rng, 4000, (world.X, world.Y, world.Z))
    out = np.zeros((len(org), 3), np.float32)
    assert L.rvt_approx(_p(world.csdf), C.c_size_t(world.csdf.nbytes), _p(org), _p(dirs), len(org), _p(out)) == 0
    w = world.c
    want = np.array([[(p := oracle.lib().or_approximate_csdf(C.byref(w), oracle.F3(*o), oracle.F3(*d))).x, p.y, p.z]
                     for o, d in zip(org, dirs)], np.float32)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32))
    assert (want[:, 0] == -100).any() and (want[:, 0] != -100).any()


@pytest.mark.gpu
def test_devapi_cones_texture_sky(world, oracle, atlas):
    L = load()
    rng = np.random.default_rng(11)
    # cones from surface points (primary hits) in unnormalised lerp directions, as computeColor makes them
    org, dirs, dist = random_rays(rng, 6000, (world.X, world.Y, world.Z))
    h = world.trace_batch(org, dirs, dist)
    sel = np.flatnonzero(h["hit"] & (h["undef"] == 0))[:2000]
    pos = np.ascontiguousarray(h["pos"][sel])
    cd = rng.normal(size=(len(sel), 3)).astype(np.float32) * 0.7
    gi = world.gi
    o8 = np.zeros((len(sel), 3), np.float32)
    of = np.zeros_like(o8)
    assert L.rvt_cone(_p(world.csdf), C.c_size_t(world.csdf.nbytes), _p(gi), C.c_size_t(gi.nbytes), _p(pos), _p(cd),
                      len(sel), _p(o8), _p(of)) == 0
    w = world.c
    want = np.array([[(c := oracle.lib().or_trace_cone(C.byref(w), oracle.F3(*p), oracle.F3(*d), None)).x, c.y, c.z]
                     for p, d in zip(pos, cd)], np.float32)
    assert np.array_equal(o8.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(of.view(np.uint32), want.view(np.uint32))   # float4 overload: same march, same texels
    assert (want != 0).any()

    # sampleTexture at the hits' uv (half values) and positions
    uv = np.ascontiguousarray(np.stack([h["u"][sel], h["v"][sel]], 1).astype(np.float32))
    at = np.ascontiguousarray(atlas)
    tex = np.zeros((len(sel), 3), np.float32)
    assert L.rvt_texture(_p(at), at.shape[1], at.shape[0], _p(uv), _p(pos), len(sel), _p(tex)) == 0
    ow = oracle.OracleWorld(*DIMS, atlas=at)
    wt = ow.c
    want = np.array([[(c := oracle.lib().or_sample_texture(C.byref(wt), float(u), float(v), oracle.F3(*p))).x, c.y, c.z]
                     for (u, v), p in zip(uv, pos)], np.float32)
    assert np.array_equal(tex.view(np.uint32), want.view(np.uint32))
    assert len(np.unique(tex, axis=0)) > 10

    # sampleSky, including directions at the sun
    sun = oracle.sun_dir()
    sd = rng.normal(size=(3000, 3)).astype(np.float32)
    sd /= np.linalg.norm(sd, axis=1, keepdims=True)
    sd[:20] = sun
    sky = np.zeros((len(sd), 3), np.float32)
    assert L.rvt_sky(_p(np.ascontiguousarray(sd)), _p(sun), len(sd), _p(sky)) == 0
    want = np.array([[(c := oracle.lib().or_sample_sky(oracle.F3(*d), oracle.F3(*sun))).x, c.y, c.z] for d in sd],
                    np.float32)
    assert np.array_equal(sky.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_devapi_issolid_getdistance(world):
    """IsSolid wraps coordinates like toIndex (include/cumath.cuh:33-38);
    getDistance(int3) truncates toward zero and clamps, getDistance(float3)
    truncates floor(p)*0.5 and clamps (include/raytracing_functions.cuh:35-67)."""
    L = load()
    rng = np.random.default_rng(3)
    n = 20000
    X, Y, Z = world.X, world.Y, world.Z
    ip = np.ascontiguousarray(rng.integers(-300, 300, (n, 3)).astype(np.int32))
    fp = np.ascontiguousarray(rng.uniform(-20, 160, (n, 3)).astype(np.float32))
    solid = np.zeros(n, np.int32)
    di = np.zeros(n, np.int32)
    df = np.zeros(n, np.float32)
    assert L.rvt_lookup(_p(world.bits), C.c_size_t(world.bits.nbytes), _p(world.csdf), C.c_size_t(world.csdf.nbytes),
                        _p(ip), _p(fp), n, _p(solid), _p(di), _p(df)) == 0
    u = ip.astype(np.int64).astype(np.uint64)
    idx = (u[:, 0] & np.uint64(X - 1)) | ((u[:, 1] & np.uint64(Y - 1)) << np.uint64(DIMS[0])) | \
          ((u[:, 2] & np.uint64(Z - 1)) << np.uint64(DIMS[0] + DIMS[1]))
    want = (world.bits[(idx >> np.uint64(5)).astype(np.int64)] >> (idx & np.uint64(31)).astype(np.uint32)) & 1
    assert np.array_equal(solid, want.astype(np.int32))
    S = np.array([X // 2, Y // 2, Z // 2])
    cs = world.csdf.reshape(Z // 2, Y // 2, X // 2)
    c = np.clip(np.trunc(ip / 2.0).astype(np.int64), 0, S - 1)
    assert np.array_equal(di, cs[c[:, 2], c[:, 1], c[:, 0]].astype(np.int32))
    c = np.clip(np.trunc(np.floor(fp) * np.float32(0.5)).astype(np.int64), 0, S - 1)
    assert np.array_equal(df, cs[c[:, 2], c[:, 1], c[:, 0]].astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("pose", ["land", "water"])
def test_devapi_reference_kernels_frame(world, oracle, atlas, pose):
    """renderKernel / distApproximationKernel with the reference's argument
    lists (include/rvgrt_kernels.h; src/StateRender.cu:200-286), launched as
    drawCUDA launches them after its three constant uploads, into pitched
    outputs: the frame (RGBA8, motion vectors, depth) and the half-res images
    equal the oracle's bit for bit -- with drawCUDA's c_cam layout, so time =
    the uploaded jitterY and jitter (0, 0) (Appendix R1), and minDist's
    reference texel fetch (RV_F_REF_FETCH)."""
    import rvgrt_amd as rv
    L = load()
    W, H = 192, 128
    if pose == "land":
        pos, yaw, pitch = (100.0, 50.0, 110.0), 2.44, -3.4415927
    else:
        pos, yaw, pitch = (64.0, 40.0, 120.0), 3.14, -3.2
    cam, vp = rv.camera_from_pose(pos, np.float32(yaw), np.float32(pitch), W, H)
    _, pvp = rv.camera_from_pose((pos[0] + 0.5, pos[1], pos[2]), np.float32(yaw + 0.01), np.float32(pitch), W, H)
    d = rv.camera_dict(cam, vp)
    sun = oracle.sun_dir()
    t_up, jx_up, jy_up = 5.25, 0.0007, 0.37   # what drawCUDA packs as time, jitterX, jitterY
    cam18 = np.array([*d["pos"], *d["fo"], *d["ri"], *d["up"], *sun, t_up, jx_up, jy_up], np.float32)
    vpa, pvpa = np.ascontiguousarray(vp, np.float32).ravel(), np.ascontiguousarray(pvp, np.float32).ravel()
    at = np.ascontiguousarray(atlas)
    color = np.zeros((H, W, 4), np.uint8)
    mv = np.zeros((H, W, 2), np.uint16)
    depth = np.zeros((H, W), np.uint16)
    hd = np.zeros((H // 2, W // 2), np.float32)
    hs = np.zeros_like(hd)
    rc = L.rvt_frame(_p(world.bits), C.c_size_t(world.bits.nbytes), _p(world.csdf), C.c_size_t(world.csdf.nbytes),
                     _p(world.gi), C.c_size_t(world.gi.nbytes), _p(at), at.shape[1], at.shape[0], _p(cam18),
                     _p(vpa), _p(pvpa), W, H, _p(color), _p(mv), _p(depth), _p(hd), _p(hs))
    assert rc == 0, f"hip error {rc}"
    ow = oracle.OracleWorld(*DIMS, atlas=at)
    ow.bits[:] = world.bits
    ow.csdf[:] = world.csdf
    ow.gi[:] = world.gi
    fr = oracle.make_frame(W, H, rv.RV_FLAGS_REFERENCE | rv.RV_F_REF_FETCH, d, time=jy_up, jx=0.0, jy=0.0, pvp=pvpa)
    ref = oracle.render(ow, fr, want_stats=False)
    assert np.array_equal(hd.view(np.uint32), ref["halfdist"].view(np.uint32))
    assert np.array_equal(hs, ref["halfshadow"])
    assert np.array_equal(color, ref["rgba"])
    assert np.array_equal(mv, ref["mv"]) and np.array_equal(depth, ref["depth"])
    assert len(np.unique(color.reshape(-1, 4), axis=0)) > 50 and (mv != 0).any()
