#!/usr/bin/env python3
"""Gather coherence per site of the pipelined reference frame.

Runs with the RV_GATHER_DIAG variant library (RVGRT_LIB=rvgrt_amd/variants/
gdiag/librvgrt_hip.so; build: make -C rvgrt_amd/csrc OUT=../variants/gdiag/
librvgrt_hip.so OBJDIR=build_gdiag DEFS=-DRV_GATHER_DIAG=1).  Renders a few
frames of a config through the native pipelined loop (as bench.py does) and
prints, per gather site (kind of trace x phase): wave-level instructions,
lanes per instruction, distinct 128-B lines per instruction over the wave and
summed over its quarter-waves, and an L1-path cost estimate in CU cycles
(profiles/r01_ubench_gather.txt: ~4 cycles per quarter-wave line, >= 5 per
instruction).

usage: python tools/gather_diag.py [config] [frames]
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KINDS = ["pp_primary", "pp_shadow", "primary", "refl", "refl_shadow", "shadow", "gi_shadow", "gi_bounce",
         "other", "cone", "tex", "half", "giread", "output", "k14", "k15"]
PHASES = {"cone": ["csdf", "gi"], "half": ["dist", "shadow"], "giread": ["cell", "solid", "bounce"],
          "output": ["mv", "depth", "color"], "tex": ["atlas"]}
NPHASE, NMETRIC = 4, 4


def main():
    cfg_name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    nframes = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    import torch
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32

    L = rv._lib.load()
    fn = L.rv_gather_diag
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    nslot = 16 * NPHASE * NMETRIC
    buf = (C.c_ulonglong * nslot)()

    cfg = CONFIGS[cfg_name]
    torch.cuda.set_device(0)
    r = rv.StateRender((cfg.log2_n,) * 3, cfg.width, cfg.height, flags=cfg.flags, atlas=load_atlas())
    s = torch.cuda.current_stream()
    r.set_stream(s.cuda_stream)
    r.set_frames_in_flight(1 if cfg.gi_per_frame else 16)
    r.set_gi_async(1)
    r.set_pipeline(1)
    r.world_build()
    for k in range(cfg.gi_sweeps):
        r.gi_update(k)
    r.sync()
    pos, yaw, pitch = pose_f32(cfg, "P0")
    path = camera_path((pos, yaw, pitch), cfg.width, cfg.height, 3 + nframes + 2, pan=0.0005, ref_compat=True)
    r.render_frame_seq(path[:3], next_desc=path[3], flags=cfg.flags, gi_per_frame=cfg.gi_per_frame)
    r.sync()
    fn(None, 0, 1)
    r.render_frame_seq(path[3:3 + nframes], next_desc=path[3 + nframes], flags=cfg.flags,
                       gi_per_frame=cfg.gi_per_frame)
    r.sync()
    assert fn(buf, nslot, 0) == 0
    a = np.array(buf[:], dtype=np.float64).reshape(16, NPHASE, NMETRIC) / nframes
    rows = []
    tot_cost = 0.0
    for k, kind in enumerate(KINDS):
        for p in range(NPHASE):
            ins, lanes, wl, ql = a[k, p]
            if ins == 0:
                continue
            phase = PHASES.get(kind, ["sphere", "dda", "check", "p3"])[p]
            cost = max(4.0 * ql, 5.0 * ins)
            tot_cost += cost
            rows.append((kind, phase, ins, lanes, wl, ql, cost))
    print(f"{cfg_name}: per frame, {nframes} frames (pipelined launch: render k + pre-pass k+1 + GI k+1)")
    print(f"{'site':24s} {'instr(M)':>9s} {'lanes(M)':>9s} {'lanes/i':>7s} {'wlines/i':>8s} {'qlines/i':>8s} "
          f"{'cost(Mcyc)':>10s} {'share':>6s}")
    for kind, phase, ins, lanes, wl, ql, cost in sorted(rows, key=lambda t: -t[6]):
        print(f"{kind + '.' + phase:24s} {ins / 1e6:9.3f} {lanes / 1e6:9.2f} {lanes / ins:7.1f} {wl / ins:8.2f} "
              f"{ql / ins:8.2f} {cost / 1e6:10.2f} {cost / tot_cost:6.1%}")
    print(f"total L1-path cost estimate {tot_cost / 1e6:.1f} M CU-cycles per frame "
          f"= {tot_cost / 256 / 2.4e9 * 1e3:.3f} ms at 256 CUs x 2.4 GHz")
    out = os.path.join(ROOT, "gpurun_out", f"gather_diag_{cfg_name}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump({"config": cfg_name, "frames": nframes,
               "rows": [dict(site=f"{k}.{p}", instr=i, lanes=l, wlines=w, qlines=q, cost=c)
                        for k, p, i, l, w, q, c in rows]}, open(out, "w"), indent=1)
    r.close()


if __name__ == "__main__":
    main()
