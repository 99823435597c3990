#!/usr/bin/env python3
"""Saturated-air census of the sphere-step chains (CPU, oracle world + host harness).

The CSDF is capped at SDF_MAX_DIST = 64 (/root/reference/include/CoarseArray.cuh:14), and inside air
whose cells all read 64, approximateCSDF's next position is pos + dir*64 whatever the gather returns
(src/raytracing_functions.cu:74-79).  A skip that knew a cell is saturated without gathering it would
take that same float step with no dependent gather.  This census measures, on the product traversal's
own step sequence (sky exit, sun exit; validated step for step against the host build of
include/rvgrt/rv_device.h), how many sphere steps read 64:
  * over all pre-pass rays of the config's frame (camera ray + its sun-shadow ray,
    distApproximationKernel, src/StateRender.cu:255-286), a random sample;
  * on the longest lane of each of the 64 longest waves (8x8 half-res tiles): the chains that end a
    latency-bound launch;
and what a radius-encoded skip would remove: at a saturated cell whose nearest non-saturated coarse
cell is r cells away (Chebyshev), every position within 2(r - 2) voxels (L-inf) is in saturated
cells, so floor((2(r - 2) - 1) / (64 max|dir_i|)) further steps need no gather.  The chain's gather
rounds with that skip are reported beside the plain ones.

usage: python tools/sat_census.py [config] [pose]      -> JSON on stdout
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

f32 = np.float32


class Replay:
    """Scalar replay of rv::trace (G-cell look-ahead groups with the stop search, sky exit YL, the sun
    exit for sun rays) recording every sphere step's CSDF byte and radius."""

    def __init__(self, csdf, rad, dims, ytop, hz, G):
        self.csdf, self.rad = csdf, rad          # (SZ, SY, SX) uint8 each
        self.X, self.Y, self.Z = dims
        self.ytop, self.hz, self.G = ytop, hz, G

    def trace(self, bits_fn, cam, d, sun=False):
        X, Y, Z = self.X, self.Y, self.Z
        cam = [f32(c) for c in cam]
        d = [f32(c) for c in d]
        cur = list(cam)
        dd = [abs(f32(1.0) / d[k]) if d[k] != 0 else f32(1e10) for k in range(3)]
        st = [int(d[k] > 0) - int(d[k] < 0) for k in range(3)]
        YL = min(Y, self.ytop) if st[1] >= 0 else Y
        mx = max(abs(float(v)) for v in d)
        rec = {"sphere": 0, "sat": 0, "rounds_plain": 0, "rounds_skip": 0, "dda_rounds": 0, "dda": 0,
               "dseq": []}   # dseq: per sphere march, the CSDF bytes its steps read (tools/spec_census.py)
        free = 0
        for _major in range(5):
            oob = False
            seq = []
            rec["dseq"].append(seq)
            for _it in range(100):
                fx, fy, fz = (int(math.floor(float(v))) for v in cur)
                oob = not (0 <= fx < X and 0 <= fy < YL and 0 <= fz < Z)
                if sun and not oob:
                    oob = fy >= int(self.hz[(min(fz, Z - 1) >> 1) * (X >> 1) + (min(fx, X - 1) >> 1)])
                if oob:
                    break
                cx, cy, cz = fx >> 1, fy >> 1, fz >> 1
                dv = int(self.csdf[cz, cy, cx])
                seq.append(dv)
                rec["sphere"] += 1
                rec["rounds_plain"] += 1
                if free > 0:
                    free -= 1                      # known saturated: no gather
                else:
                    rec["rounds_skip"] += 1
                    if dv == 64:
                        r = int(self.rad[cz, cy, cx])
                        free = max(0, int((2 * (r - 2) - 1) // (64.0 * mx))) if r > 2 else 0
                if dv == 64:
                    rec["sat"] += 1
                if dv <= 1:
                    break
                cur = [cur[k] + d[k] * f32(dv) for k in range(3)]
            free = 0
            if oob:
                return rec
            ip = [int(math.floor(float(cur[k]))) for k in range(3)]
            tm = [((f32(ip[k]) + f32(1.0) - cur[k]) if st[k] > 0 else (cur[k] - f32(ip[k]))) * dd[k]
                  for k in range(3)]
            jumped = False
            groups_open = -1
            for i in range(200):
                if i // self.G != groups_open:
                    groups_open = i // self.G
                    rec["dda_rounds"] += 1
                if (i & 7) == 7:
                    dv = int(self.csdf[min(max(ip[2] // 2 if ip[2] >= 0 else -((-ip[2]) // 2), 0), self.csdf.shape[0] - 1),
                                       min(max(ip[1] // 2 if ip[1] >= 0 else -((-ip[1]) // 2), 0), self.csdf.shape[1] - 1),
                                       min(max(ip[0] // 2 if ip[0] >= 0 else -((-ip[0]) // 2), 0), self.csdf.shape[2] - 1)])
                    if dv > 2:
                        cen = [f32(ip[k]) + f32(0.5) for k in range(3)]
                        t = ((cen[0] - cur[0]) * d[0] + (cen[1] - cur[1]) * d[1]) + (cen[2] - cur[2]) * d[2]
                        por = [cur[k] + d[k] * t for k in range(3)]
                        cur = [por[k] + d[k] * (f32(dv) * f32(2.0)) for k in range(3)]
                        jumped = True
                        break
                if not (0 <= ip[0] < X and 0 <= ip[1] < YL and 0 <= ip[2] < Z):
                    return rec
                rec["dda"] += 1
                if bits_fn(*ip):
                    return rec
                if tm[0] < tm[1]:
                    a = 0 if tm[0] < tm[2] else 2
                else:
                    a = 1 if tm[1] < tm[2] else 2
                tm[a] = tm[a] + dd[a]
                ip[a] += st[a]
            if not jumped:
                return rec
        return rec


def setup(cfg_name, pose):
    """The oracle world, the config's pre-pass rays traced on the host, and the replay (shared with
    tools/spec_census.py)."""
    from scipy import ndimage
    from oracle import oracle as O
    from rvgrt_amd.configs import CONFIGS, pose_f32
    from test_host_trace import HIT as HOST_HIT

    cfg = CONFIGS[cfg_name]
    lg = cfg.log2_n
    O.set_threads(os.cpu_count() or 8)
    t0 = time.time()
    cache = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"sat_census_world_{lg}.npz")
    ow = O.OracleWorld(lg, lg, lg)
    if os.path.exists(cache):                    # the oracle world of an earlier run
        z = np.load(cache)
        ow.bits[:] = z["bits"]
        ow.csdf[:] = z["csdf"]
    else:
        ow.fill().build_csdf()
        np.savez(cache, bits=ow.bits, csdf=ow.csdf)
    print(f"world {cfg.n}^3 built in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    N = cfg.n
    S = N // 2
    cs = ow.csdf.reshape(S, S, S)
    t0 = time.time()
    rad = ndimage.distance_transform_cdt(cs == 64, metric="chessboard").astype(np.int32)
    rad = np.minimum(rad, 255).astype(np.uint8)
    print(f"radius map in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)

    pos, yaw, pitch = pose_f32(cfg, pose)
    W, H = cfg.width, cfg.height
    cam = O.camera_from_pose(pos, yaw, pitch, W, H)
    hw, hh = W // 2, H // 2
    ix, iy = np.meshgrid(np.arange(hw, dtype=np.float32), np.arange(hh, dtype=np.float32))
    x = (ix + np.float32(0.5)) / np.float32(hw)
    y = (iy + np.float32(0.5)) / np.float32(hh)
    nx = (x * np.float32(2) - np.float32(1)).ravel()
    ny = (y * np.float32(2) - np.float32(1)).ravel()
    fo, ri, up = (np.asarray(cam[k], np.float32) for k in ("fo", "ri", "up"))
    d = fo[None, :] + ri[None, :] * nx[:, None] + up[None, :] * ny[:, None]
    d = (d * (np.float32(1.0) / np.sqrt((d * d).sum(1, dtype=np.float32)))[:, None]).astype(np.float32)
    n = len(d)
    org = np.ascontiguousarray(np.broadcast_to(np.asarray(cam["pos"], np.float32), (n, 3)))
    zero = np.zeros(n, np.float32)

    # the product traversal on the host: camera rays at look-ahead 8 with the sky exit, shadow rays through
    # trace_sun (sky + sun exits); oracle hits for positions/normals
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "host")], check=True)
    L = C.CDLL(os.path.join(ROOT, "tests", "host", "build", "librvhost.so"))
    P = C.c_void_p
    L.rvh_trace_rays_sky_exit.argtypes = [C.c_int] * 4 + [P] * 5 + [C.c_int64, P, P]
    L.rvh_trace_sun.argtypes = [C.c_int] * 4 + [P] * 5 + [C.c_int64, P, P]
    hc = np.zeros(n, HOST_HIT)
    ytop = C.c_uint32()
    L.rvh_trace_rays_sky_exit(3, lg, lg, lg, ow.bits.ctypes.data_as(P), ow.csdf.ctypes.data_as(P),
                              org.ctypes.data_as(P), np.ascontiguousarray(d).ctypes.data_as(P),
                              zero.ctypes.data_as(P), C.c_int64(n), hc.ctypes.data_as(P), C.byref(ytop))
    hit = hc["hit"] != 0
    sun = O.sun_dir()
    o2 = (hc["pos"] + hc["normal"] * np.float32(0.1)).astype(np.float32)[hit]
    m = len(o2)
    hs = np.zeros(m, HOST_HIT)
    hz = np.zeros((N // 2) * (N // 2), np.uint32)
    L.rvh_trace_sun(1, lg, lg, lg, ow.bits.ctypes.data_as(P), ow.csdf.ctypes.data_as(P),
                    sun.ctypes.data_as(P), np.ascontiguousarray(o2).ctypes.data_as(P),
                    np.zeros(m, np.float32).ctypes.data_as(P), C.c_int64(m), hs.ctypes.data_as(P),
                    hz.ctypes.data_as(P))
    # chain length per half-res pixel (sphere steps + DDA rounds at G = 8), as tools/chain_census.py
    G = 8
    s1 = hc["sphere"].astype(np.int64)
    d1 = (hc["dda"].astype(np.int64) + G - 1) // G
    s2 = np.zeros(n, np.int64)
    d2 = np.zeros(n, np.int64)
    s2[hit] = hs["sphere"]
    d2[hit] = (hs["dda"].astype(np.int64) + G - 1) // G
    tot = (s1 + d1 + s2 + d2).reshape(hh, hw)
    th, tw = hh // 8, hw // 8
    t = tot[:th * 8, :tw * 8].reshape(th, 8, tw, 8).transpose(0, 2, 1, 3).reshape(th * tw, 64)
    arg = t.argmax(1)
    wmax = t[np.arange(len(t)), arg]
    order = np.argsort(-wmax)[:64]
    # lanes (half-res pixel index) of the 64 longest waves' longest lanes
    tiles = order
    lanes = []
    for ti, a in zip(tiles, arg[tiles]):
        ty_, tx_ = divmod(int(ti), tw)
        py_, px_ = ty_ * 8 + a // 8, tx_ * 8 + a % 8
        lanes.append(py_ * hw + px_)
    rng = np.random.default_rng(5)
    sample = rng.choice(n, 3000, replace=False)

    bits = ow.bits
    lx = lg

    def solid(x_, y_, z_):
        i = x_ | (y_ << lx) | (z_ << (2 * lx))
        return (int(bits[i >> 5]) >> (i & 31)) & 1

    rp = Replay(cs, rad, (N, N, N), int(ytop.value), hz, G)
    hit_index = np.full(n, -1, np.int64)
    hit_index[np.flatnonzero(hit)] = np.arange(m)
    return dict(rp=rp, solid=solid, org=org, d=d, lanes=lanes, sample=sample, hc=hc, hs=hs, hit=hit, o2=o2,
                hit_index=hit_index, sun=sun, d1=d1, d2=d2, cs=cs, rad=rad, ytop=ytop, G=G)


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    pose = sys.argv[2] if len(sys.argv) > 2 else "P0"
    e = setup(cfg_name, pose)
    rp, solid, org, d, lanes, sample = e["rp"], e["solid"], e["org"], e["d"], e["lanes"], e["sample"]
    hc, hs, hit, o2, hit_index, sun, d1, d2 = (e[k] for k in ("hc", "hs", "hit", "o2", "hit_index", "sun", "d1", "d2"))
    cs, rad, ytop, G = e["cs"], e["rad"], e["ytop"], e["G"]

    def census(idx):
        agg = {k: {"sphere": 0, "sat": 0, "rounds_plain": 0, "rounds_skip": 0} for k in ("camera", "shadow")}
        chains = []
        for i in idx:
            a = rp.trace(solid, org[i], d[i])
            assert a["sphere"] == hc["sphere"][i] and a["dda"] == hc["dda"][i], ("camera replay", i, a, hc[i])
            c_plain = a["rounds_plain"] + d1[i]
            c_skip = a["rounds_skip"] + d1[i]
            for k in agg["camera"]:
                agg["camera"][k] += a[k]
            if hit[i]:
                j = hit_index[i]
                b = rp.trace(solid, o2[j], sun, sun=True)
                assert b["sphere"] == hs["sphere"][j] and b["dda"] == hs["dda"][j], ("shadow replay", i, b, hs[j])
                c_plain += b["rounds_plain"] + d2[i]
                c_skip += b["rounds_skip"] + d2[i]
                for k in agg["shadow"]:
                    agg["shadow"][k] += b[k]
            chains.append((int(c_plain), int(c_skip)))
        for k in agg:
            s = agg[k]
            s["sat_frac"] = round(s["sat"] / max(s["sphere"], 1), 4)
        ch = np.array(chains)
        return agg, {"mean_plain": float(ch[:, 0].mean()), "mean_skip": float(ch[:, 1].mean()),
                     "max_plain": int(ch[:, 0].max()), "max_skip": int(ch[:, 1].max())}

    t0 = time.time()
    top_agg, top_chain = census(lanes)
    all_agg, all_chain = census(sample)
    print(f"replayed in {time.time() - t0:.1f} s (step counts equal the host build's for every ray)",
          file=sys.stderr, flush=True)
    out = {"config": cfg_name, "pose": pose, "G": G, "ytop": int(ytop.value),
           "csdf_saturated_frac": float((cs == 64).mean()),
           "radius_ge_22_frac_of_saturated": float((rad >= 22).sum() / max((cs == 64).sum(), 1)),
           "top64_waves_longest_lanes": {"steps": top_agg, "chain_rounds": top_chain},
           "random_3000_rays": {"steps": all_agg, "chain_rounds": all_chain}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
