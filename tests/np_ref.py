"""Independent numpy restatement of the reference's noise, CSDF and DDA
(test infrastructure).  Written separately from oracle/rv_oracle.c so the two
restatements cross-check each other bit for bit: numpy float32 arithmetic is
IEEE round-to-nearest per operation, exactly like the C oracle built with
-ffp-contract=off.

References: include/TerrainGeneration.cuh:25-356, src/CoarseArray.cu:11-152,
src/raytracing_functions.cu:65-202, include/raytracing_functions.cuh:23-67.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32
u32 = np.uint32


def hash3(x, y, z):
    """include/TerrainGeneration.cuh:25-44 on int arrays."""
    with np.errstate(over="ignore"):
        x = np.asarray(x).astype(np.int64).astype(u32)
        y = np.asarray(y).astype(np.int64).astype(u32)
        z = np.asarray(z).astype(np.int64).astype(u32)
        k = (x * u32(73856093)) ^ (y * u32(19349663)) ^ (z * u32(83492791))
        k = (k ^ u32(61)) ^ (k >> u32(16))
        k = k * u32(9)
        k = k ^ (k >> u32(4))
        k = k * u32(0x27D4EB2D)
        k = k ^ (k >> u32(15))
    return k


def hash2(x, y):
    with np.errstate(over="ignore"):
        x = np.asarray(x).astype(np.int64).astype(u32)
        y = np.asarray(y).astype(np.int64).astype(u32)
        k = (x * u32(73856093)) ^ (y * u32(19349663))
        k = (k ^ u32(61)) ^ (k >> u32(16))
        k = k * u32(9)
        k = k ^ (k >> u32(4))
        k = k * u32(0x27D4EB2D)
        k = k ^ (k >> u32(15))
    return k


def _grad_dot3(h, x, y, z):
    h = h & u32(15)
    gx = np.where(h & u32(1), f32(1), f32(-1)).astype(f32)
    gy = np.where(h & u32(2), f32(1), f32(-1)).astype(f32)
    gz = np.where(h & u32(4), f32(1), f32(-1)).astype(f32)
    gz = np.where(h < 8, f32(0), gz).astype(f32)
    gx = np.where((h >= 8) & (h < 12), f32(0), gx).astype(f32)
    gy = np.where(h >= 12, f32(0), gy).astype(f32)
    return (gx * x + gy * y) + gz * z


def simplex3D(px, py, pz):
    px, py, pz = (np.asarray(v, f32) for v in (px, py, pz))
    F3 = f32(1.0) / f32(3.0)
    G3 = f32(1.0) / f32(6.0)
    s = ((px + py) + pz) * F3
    i = np.floor(px + s).astype(np.int64)
    j = np.floor(py + s).astype(np.int64)
    k = np.floor(pz + s).astype(np.int64)
    t = (i + j + k).astype(f32) * G3
    x0 = px - (i.astype(f32) - t)
    y0 = py - (j.astype(f32) - t)
    z0 = pz - (k.astype(f32) - t)
    cxy = (x0 >= y0).astype(np.int64)
    cxz = (x0 >= z0).astype(np.int64)
    cyz = (y0 >= z0).astype(np.int64)
    i1 = cxy & cxz
    j1 = (1 - cxy) & cyz
    k1 = (1 - cxz) & (1 - cyz)
    i2 = 1 - ((1 - cxy) & (1 - cxz))
    j2 = 1 - (cxy & (1 - cyz))
    k2 = 1 - (cxz & cyz)
    two, three = f32(2.0) * G3, f32(3.0) * G3
    pts = [(x0, y0, z0, i, j, k),
           (x0 - i1.astype(f32) + G3, y0 - j1.astype(f32) + G3, z0 - k1.astype(f32) + G3, i + i1, j + j1, k + k1),
           (x0 - i2.astype(f32) + two, y0 - j2.astype(f32) + two, z0 - k2.astype(f32) + two, i + i2, j + j2, k + k2),
           (x0 - f32(1) + three, y0 - f32(1) + three, z0 - f32(1) + three, i + 1, j + 1, k + 1)]
    n = []
    for (x, y, z, a, b, c) in pts:
        t0 = ((f32(0.5) - x * x) - y * y) - z * z
        t0 = np.maximum(f32(0), t0)
        t0 = t0 * t0
        n.append((t0 * t0) * _grad_dot3(hash3(a, b, c), x, y, z))
    return f32(96.0) * (((n[0] + n[1]) + n[2]) + n[3])


def simplex2D(px, py):
    px, py = (np.asarray(v, f32) for v in (px, py))
    s3 = np.sqrt(f32(3.0))
    F2 = (s3 - f32(1.0)) * f32(0.5)
    G2 = (f32(3.0) - s3) * f32(0.5)
    s = (px + py) * F2
    i = np.floor(px + s).astype(np.int64)
    j = np.floor(py + s).astype(np.int64)
    t = (i + j).astype(f32) * G2
    x0 = (px - i.astype(f32)) + t
    y0 = (py - j.astype(f32)) + t
    i1 = (x0 > y0).astype(np.int64)
    j1 = 1 - i1
    pts = [(x0, y0, i, j), ((x0 - i1.astype(f32)) + G2, (y0 - j1.astype(f32)) + G2, i + i1, j + j1),
           ((x0 - f32(1)) + f32(2) * G2, (y0 - f32(1)) + f32(2) * G2, i + 1, j + 1)]
    n = []
    for (x, y, a, b) in pts:
        h = hash2(a, b) & u32(7)
        gx = np.where(h & u32(1), f32(1), f32(-1)).astype(f32)
        gy = np.where(h & u32(2), f32(1), f32(-1)).astype(f32)
        gy = np.where(h < 4, f32(0), gy).astype(f32)
        gx = np.where(h >= 4, f32(0), gx).astype(f32)
        tt = (f32(0.5) - x * x) - y * y
        tt = np.maximum(f32(0), tt)
        tt = tt * tt
        n.append((tt * tt) * (gx * x + gy * y))
    return f32(70.0) * ((n[0] + n[1]) + n[2])


def fbm3D(x, y, z, octaves, freq, lac, pers):
    x, y, z = (np.asarray(v, f32) for v in (x, y, z))
    total = np.zeros(np.broadcast(x, y, z).shape, f32)
    amp = f32(1.0)
    freq, lac, pers = f32(freq), f32(lac), f32(pers)
    for _ in range(octaves):
        total = total + simplex3D(x * freq, y * freq, z * freq) * amp
        freq = freq * lac
        amp = amp * pers
    return total


def evaluate(x, y, z):
    """include/TerrainGeneration.cuh:284-356 (vectorised)."""
    x, y, z = (np.asarray(v, f32) for v in (x, y, z))
    biome = (simplex2D(x * f32(0.005), z * f32(0.005)) + f32(1.0)) * f32(0.5)
    amp = f32(60.0) + biome * (f32(400.0) - f32(60.0))
    density = f32(10.0) - y
    density = density + fbm3D(x, y, z, 7, 0.002, 2.1, 0.45) * amp
    cave_raw = fbm3D(x + f32(123.456), y, z, 3, 0.009, 2.1, 0.45)
    cave_norm = (cave_raw + f32(1.0)) * f32(0.5)
    spaghetti = np.abs(cave_raw) < f32(0.025)
    region = (simplex3D(x * f32(0.006), y * f32(0.006), z * f32(0.006)) + f32(1.0)) * f32(0.5)
    cavern = (region > f32(0.65)) & (cave_norm < f32(0.3))
    carve = (density > f32(0)) & (spaghetti | cavern)
    density = np.where(carve, density - f32(2.0), density).astype(f32)
    return np.where(y <= f32(30.0), f32(100.0), density).astype(f32)


def csdf_3pass(solid: np.ndarray) -> np.ndarray:
    """src/CoarseArray.cu:37-152 on a coarse solid grid [z, y, x] (bool);
    out-of-range neighbours skipped (Appendix R3)."""
    SZ, SY, SX = solid.shape
    dx = np.full(solid.shape, 64, np.int64)
    for z in range(SZ):
        for y in range(SY):
            row = solid[z, y]
            for x in range(SX):
                if row[x]:
                    dx[z, y, x] = 0
                    continue
                m = 64
                for i in range(1, 65):
                    if i <= x and row[x - i]:
                        m = i
                        break
                for i in range(1, m):
                    if x + i < SX and row[x + i]:
                        m = i
                        break
                dx[z, y, x] = m

    def axis_pass(src, axis):
        out = np.zeros_like(src)
        n = src.shape[axis]
        it = np.nditer(src, flags=["multi_index"])
        for v in it:
            idx = it.multi_index
            cur = int(v)
            if cur == 0:
                continue
            m = f32(cur) * f32(cur)
            c = idx[axis]
            for off in range(1, 65):
                if f32(off * off) >= m:
                    break
                for cc in (c - off, c + off):
                    if 0 <= cc < n:
                        j = list(idx)
                        j[axis] = cc
                        nb = int(src[tuple(j)])
                        m = min(m, f32(f32(nb) * f32(nb) + f32(off) * f32(off)))
            out[idx] = int(min(f32(64.0), np.sqrt(f32(m))))
        return out

    dy = axis_pass(dx, 1)
    return axis_pass(dy, 0).astype(np.uint8)


def hround(v) -> np.float32:
    return f32(np.float16(f32(v)))


def trace_py(solid_fn, csdf_fn, dims, cam, d, dist_h):
    """Scalar pure-Python restatement of trace() (src/raytracing_functions.cu:85-202)
    on numpy float32 scalars.  solid_fn(x,y,z)->bool, csdf_fn(cx,cy,cz)->int
    (in-range coarse cell).  Returns (hit, undef, pos, normal, u, v)."""
    X, Y, Z = dims
    SX, SY, SZ = X // 2, Y // 2, Z // 2
    cam = [f32(c) for c in cam]
    d = [f32(c) for c in d]
    cur = [cam[k] + d[k] * f32(dist_h) for k in range(3)]
    dd = [abs(f32(1.0) / d[k]) if d[k] != 0 else f32(1e10) for k in range(3)]
    st = [int(d[k] > 0) - int(d[k] < 0) for k in range(3)]

    def clamp(v, hi):
        return max(min(v, hi - 1), 0)

    def trunc_div2(v):
        return int(math.trunc(v / 2))

    for _major in range(5):
        for _it in range(100):
            if any(cur[k] < 0 for k in range(3)) or cur[0] >= f32(X) or cur[1] >= f32(Y) or cur[2] >= f32(Z):
                cur = [f32(-100.0)] * 3
                break
            c = [int(float(f32(math.floor(cur[k])) * f32(0.5))) for k in range(3)]   # int() truncates
            dv = f32(csdf_fn(clamp(c[0], SX), clamp(c[1], SY), clamp(c[2], SZ)))
            if dv <= f32(1.0):
                break
            cur = [cur[k] + d[k] * dv for k in range(3)]
        ip = [int(math.floor(cur[k])) for k in range(3)]
        tm = [((f32(ip[k]) + f32(1.0) - cur[k]) if st[k] > 0 else (cur[k] - f32(ip[k]))) * dd[k] for k in range(3)]
        mask = -128
        jumped = False
        for i in range(200):
            if (i & 7) == 7:
                dv = csdf_fn(clamp(trunc_div2(ip[0]), SX), clamp(trunc_div2(ip[1]), SY), clamp(trunc_div2(ip[2]), SZ))
                if dv > 2:
                    cen = [f32(ip[k]) + f32(0.5) for k in range(3)]
                    t = ((cen[0] - cur[0]) * d[0] + (cen[1] - cur[1]) * d[1]) + (cen[2] - cur[2]) * d[2]
                    por = [cur[k] + d[k] * t for k in range(3)]
                    cur = [por[k] + d[k] * (f32(dv) * f32(2.0)) for k in range(3)]
                    jumped = True
                    break
            if ip[0] < 0 or ip[1] < 0 or ip[2] < 0 or ip[0] >= X or ip[1] >= Y or ip[2] >= Z:
                return (False, False, None, None, 0.0, 0.0)
            if solid_fn(*ip):
                if mask == -128:
                    return (True, True, [f32(-500)] * 3, [f32(0)] * 3, 0.0, 0.0)
                a = mask
                pos = [cur[k] + d[k] * (tm[a] - dd[a]) for k in range(3)]
                nrm = [f32(0)] * 3
                nrm[a] = f32(-st[a])
                if a == 0:
                    u, v = hround(pos[1] - f32(ip[1])), hround(pos[2] - f32(ip[2]))
                    if st[0] == -1:
                        v = hround(f32(1.0) - v)
                elif a == 1:
                    u, v = hround(pos[0] - f32(ip[0])), hround(pos[2] - f32(ip[2]))
                else:
                    u, v = hround(pos[0] - f32(ip[0])), hround(pos[1] - f32(ip[1]))
                    if st[2] == 1:
                        u = hround(f32(1.0) - u)
                return (True, False, pos, nrm, u, v)
            if tm[0] < tm[1]:
                a = 0 if tm[0] < tm[2] else 2
            else:
                a = 1 if tm[1] < tm[2] else 2
            tm[a] = tm[a] + dd[a]
            ip[a] += st[a]
            mask = a
        if not jumped:
            break
    return (False, False, None, None, 0.0, 0.0)
