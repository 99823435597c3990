#!/usr/bin/env python3
"""Longest wave of each part of the pipelined reference-frame launch
(k_ref_pipe: GI update | pre-pass | render), for a whole frame or one rank's
tile share, on ONE GPU: the latency floor of a launch.  Needs
a library built with -DRV_PIPE_DIAG=1 (RVGRT_LIB=rvgrt_amd/variants/diag/...,
see DESIGN.md s7) and RV_PIPE_WAVE_STATS=1 (the library prints the
table when the context is destroyed); for shares RV_GI_SHARD_PROBE=1.  Not
part of the product.

usage: python tools/pipe_waves.py config [nranks tile_px]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, pose_f32

    cfg = CONFIGS[sys.argv[1]]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    T = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    torch.cuda.set_device(0)
    W, H = cfg.width, cfg.height
    r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=load_atlas())
    if os.environ.get("RV_GI_SHARD_PROBE"):   # this tool's knob -> the library option
        r.set_option(rv.RV_OPT_GI_SHARD_PROBE, 1)
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    pos, yaw, pitch = pose_f32(cfg)
    cam, vp = rv.camera_from_pose(pos, yaw, pitch, W, H)
    if N > 0:
        r.set_tile_shard(T, 0, N)
    r.render_frames(8, cam, vp, gi_per_frame=True)
    r.sync()
    t0 = time.perf_counter()
    r.render_frames(64, cam, vp, gi_per_frame=True)
    r.sync()
    us = (time.perf_counter() - t0) / 64 * 1e6
    print(f"{cfg.name} {'whole frame' if N == 0 else f'rank 0 of {N}, {T}-px tiles'}: {us:.1f} us/frame", flush=True)
    r.close()


if __name__ == "__main__":
    main()
