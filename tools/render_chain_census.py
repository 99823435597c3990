#!/usr/bin/env python3
"""The C3 drop-in frame's critical chain, both halves (CPU, oracle + tests/np_shade.py; not product code).

The flow launch's last render waves wait for the slowest pre-pass tile (tools/flow_waves.py) and then run
~100 us more.  This replays that frame (C3, 1024^3, 1920x1080, pose P0, after 1 GI sweep): the pre-pass
camera ray's dependent gather rounds per half-res texel (sphere steps + look-ahead-8 DDA groups), the
slowest tiles, and for the full-res pixels whose half-res window reads the slowest tile, the primary ray's
rounds from its start distance minDist - 8 (src/StateRender.cu:182-198).  A texel whose pre-pass ray
misses stores 300 - 8, so horizon pixels start their primary ray at 292 and march again almost as far as
the pre-pass ray did: the frame is two chained ~140-round chains.

usage: python tools/render_chain_census.py > profiles/r06/render_chain_c3.txt
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle import oracle as O
from rvgrt_amd.atlas import load_atlas
from rvgrt_amd.configs import CONFIGS, pose_f32, camera_path
import np_shade as S
cfg = CONFIGS['c3']; W, H = cfg.width, cfg.height
ow = O.OracleWorld(10, 10, 10, atlas=load_atlas()); ow.fill(); ow.build_csdf(); ow.gi_init(); ow.gi_update(0)
pos, yaw, pitch = pose_f32(cfg, 'P0')
cam = O.camera_from_pose(pos, yaw, pitch, W, H)
tr = lambda o, d, t: ow.trace_batch(np.ascontiguousarray(o, np.float32), np.ascontiguousarray(d, np.float32), np.ascontiguousarray(t, np.float32))
sun = S.sun_dir()
hd, hs = S.prepass(tr, cam, sun, W, H, 0.0, 0.0)
# pre-pass chain per half-res texel: camera + shadow
hh, hw = hd.shape
iy, ix = np.mgrid[0:hh, 0:hw]
x = ((ix.ravel().astype(np.float32) + 0.5) / hw).astype(np.float32); y = ((iy.ravel().astype(np.float32) + 0.5) / hh).astype(np.float32)
d = S.ray_dirs(cam, x, y, 0, 0)
h = tr(np.broadcast_to(np.asarray(cam['pos'], np.float32), d.shape), d, np.zeros(len(d), np.float32))
ppr = (h['n_sphere'] + (h['n_dda'] + 7) // 8).reshape(hh, hw)
tiles = ppr.reshape(hh // 8 if hh % 8 == 0 else hh // 8, 8, -1, 8) if hh % 8 == 0 else None
# tile max
th = (hh + 7) // 8; tw = (hw + 7) // 8
pad = np.zeros((th * 8, tw * 8), np.int64); pad[:hh, :hw] = ppr
tmax = pad.reshape(th, 8, tw, 8).max(axis=(1, 3))
order = np.dstack(np.unravel_index(np.argsort(-tmax.ravel())[:5], tmax.shape))[0]
print('slowest pre-pass tiles (by, bx, rounds):', [(int(a), int(b), int(tmax[a, b])) for a, b in order])
by, bx = order[0]
# render pixels whose 8x8 window depends on that tile: full-res pixels with x in [bx*16-2 .. ] approx
X0, Y0 = bx * 16 - 4, by * 16 - 4
py, px = np.mgrid[max(Y0, 0):min(Y0 + 24, H), max(X0, 0):min(X0 + 24, W)]
xs = (px.ravel().astype(np.float32) / W).astype(np.float32); ys = (py.ravel().astype(np.float32) / H).astype(np.float32)
dist = S.min_dist(hd, xs, ys, False)
dd = S.ray_dirs(cam, xs, ys, 0, 0)
org = np.broadcast_to(np.asarray(cam['pos'], np.float32), dd.shape)
hp = tr(org, dd, S.hround(dist))
prim = hp['n_sphere'] + (hp['n_dda'] + 7) // 8
water = (hp['hit'] != 0) & (hp['pos'][:, 1] < 31.001)
print('render pixels', len(xs), 'hit', (hp['hit'] != 0).mean(), 'water', water.mean())
print('primary rounds: p50 %d p90 %d max %d' % (np.percentile(prim, 50), np.percentile(prim, 90), prim.max()))
print('dist min/med', dist.min(), np.median(dist), 'hit dist med', np.median(np.linalg.norm(hp['pos'] - org, axis=1)))
if water.any():
    hw_ = hp[water]; dw = dd[water]
    nx = S.fbm3D(hw_['pos'][:, 0], hw_['pos'][:, 2], np.zeros(len(hw_), np.float32), 3, 0.06, 2.0, 0.6)
    ny = S.fbm3D(hw_['pos'][:, 2], hw_['pos'][:, 0], np.full(len(hw_), 112, np.float32), 3, 0.06, 2.0, 0.6)
    dn = S.normalize(hw_['normal'] + S.v3(nx * np.float32(0.1), ny * np.float32(0.1), np.zeros(len(hw_), np.float32)))
    rd = dw - S.scale(dn, 2 * S.dot(dw, dn))
    rh = tr(hw_['pos'], rd, np.full(len(rd), 0.001, np.float32))
    rr = rh['n_sphere'] + (rh['n_dda'] + 3) // 4
    print('reflection rounds: p50 %d max %d' % (np.percentile(rr, 50), rr.max()))
