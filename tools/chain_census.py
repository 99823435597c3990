#!/usr/bin/env python3
"""Dependent-gather chains of the pre-pass rays, per half-res pixel and per wave (CPU, oracle).

A latency-bound launch (a rank's tile share at one frame per launch, C3 flow frames) ends with its
longest chain of dependent gathers.  This census restates, from the oracle's per-ray
step counts (or_trace_batch: sphere steps, DDA cells, every-8th-step checks, its), how long the
pre-pass's chains are and what they are made of:
  sphere rounds : one dependent CSDF gather per sphere step (data-dependent, cannot overlap);
  DDA rounds    : one gather round per look-ahead group of G cells (G = 8 for the pre-pass,
                  rv_shade.h RV_G_PREPASS), per DDA segment (a segment ends at a hit, the grid edge
                  or a check that jumps);
for the camera ray and its shadow ray (distApproximationKernel, src/StateRender.cu:255-286).  A wave
is an 8x8 half-res tile; its chain is its longest lane's.  Prints the distribution and, for the
longest waves, the split sphere / DDA rounds -- the ceiling of any scheme that shortens the DDA part
(e.g. lanes of a tail wave gathering further cells of the surviving rays).

usage: python tools/chain_census.py [config] [pose] [G]
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rounds(h, G):
    """Dependent gather rounds of each ray: sphere steps + DDA look-ahead groups per segment."""
    sph = h["n_sphere"].astype(np.int64)
    dda = h["n_dda"].astype(np.int64)
    seg = np.maximum(h["its"].astype(np.int64) - dda - 1, 0)   # major iterations that ran a DDA walk
    seg = np.where(dda > 0, np.maximum(seg, 1), seg)
    ddar = (dda + G * seg - 1) // G if G > 1 else dda
    ddar = np.where(dda > 0, np.maximum(ddar, seg), 0)
    return sph, ddar


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    pose = sys.argv[2] if len(sys.argv) > 2 else "P0"
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    from oracle import oracle as O
    from rvgrt_amd.configs import CONFIGS, pose_f32
    cfg = CONFIGS[cfg_name]
    O.set_threads(os.cpu_count() or 8)
    t0 = time.time()
    ow = O.OracleWorld(cfg.log2_n, cfg.log2_n, cfg.log2_n).build(gi_sweeps=-1)
    print(f"world {cfg.n}^3 built in {time.time() - t0:.1f} s", flush=True)
    pos, yaw, pitch = pose_f32(cfg, pose)
    W, H = cfg.width, cfg.height
    cam = O.camera_from_pose(pos, yaw, pitch, W, H)
    hw, hh = W // 2, H // 2
    # prepass_eval: the half-res pixel centre through ray_dir (rv_frame.h; jitter 0 as ref_compat maps it)
    ix, iy = np.meshgrid(np.arange(hw, dtype=np.float32), np.arange(hh, dtype=np.float32))
    x = (ix + np.float32(0.5)) / np.float32(hw)
    y = (iy + np.float32(0.5)) / np.float32(hh)
    nx = (x * np.float32(2) - np.float32(1)).ravel()
    ny = (y * np.float32(2) - np.float32(1)).ravel()
    fo, ri, up = (np.asarray(cam[k], np.float32) for k in ("fo", "ri", "up"))
    d = fo[None, :] + ri[None, :] * nx[:, None] + up[None, :] * ny[:, None]
    d = (d / np.sqrt((d * d).sum(1, dtype=np.float32))[:, None]).astype(np.float32)
    n = len(d)
    org = np.broadcast_to(np.asarray(cam["pos"], np.float32), (n, 3))
    t0 = time.time()
    h1 = ow.trace_batch(org, d, np.zeros(n, np.float32))
    hit = h1["hit"] != 0
    sun = O.sun_dir()
    p1 = h1["pos"].astype(np.float32)
    n1 = h1["normal"].astype(np.float32)
    o2 = (p1 + n1 * np.float32(0.1))[hit]
    h2 = ow.trace_batch(o2, np.broadcast_to(sun, (len(o2), 3)), np.zeros(len(o2), np.float32))
    print(f"{n} camera rays + {len(o2)} shadow rays traced in {time.time() - t0:.1f} s", flush=True)
    s1, d1 = rounds(h1, G)
    s2 = np.zeros(n, np.int64)
    d2 = np.zeros(n, np.int64)
    a, b = rounds(h2, G)
    s2[hit], d2[hit] = a, b
    # the oracle's shadow ray has no sun exit; count its sphere steps as they are (an upper bound)
    tot = s1 + d1 + s2 + d2
    img = tot.reshape(hh, hw)
    parts = np.stack([s1, d1, s2, d2], 1).reshape(hh, hw, 4)
    # waves: 8x8 half-res tiles
    th, tw = hh // 8, hw // 8
    t = img[:th * 8, :tw * 8].reshape(th, 8, tw, 8).transpose(0, 2, 1, 3).reshape(th * tw, 64)
    p = parts[:th * 8, :tw * 8].reshape(th, 8, tw, 8, 4).transpose(0, 2, 1, 3, 4).reshape(th * tw, 64, 4)
    arg = t.argmax(1)
    wmax = t[np.arange(len(t)), arg]
    wpart = p[np.arange(len(t)), arg]
    order = np.argsort(-wmax)
    res = {"config": cfg_name, "pose": pose, "G": G, "rays": int(n), "waves": int(len(t)),
           "ray_rounds_pct": {q: float(np.percentile(tot, q)) for q in (50, 90, 99, 99.9, 100)},
           "wave_rounds_pct": {q: float(np.percentile(wmax, q)) for q in (50, 90, 99, 99.9, 100)}}
    top = order[:64]
    sp = wpart[top]
    res["top64_waves_mean_split"] = {"cam_sphere": float(sp[:, 0].mean()), "cam_dda_rounds": float(sp[:, 1].mean()),
                                     "shadow_sphere": float(sp[:, 2].mean()), "shadow_dda_rounds": float(sp[:, 3].mean())}
    res["top8_waves"] = [[int(v) for v in wpart[i]] for i in order[:8]]
    dd = h1["n_dda"].astype(np.int64)
    res["cam_dda_cells_pct"] = {q: float(np.percentile(dd, q)) for q in (50, 99, 100)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
