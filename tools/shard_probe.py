#!/usr/bin/env python3
"""Per-rank render time of the screen-tile shard, measured on ONE GPU.

For every N and tile size, renders the share of each rank r < N with the
native loop (rv_render_frames, K frames per launch, no gather) and reports
the slowest rank's time per frame next to the whole frame's: the render-side
bound of the N-GPU strong scaling (the gather to rank 0 comes on top).  Used
to choose the shard tile size; not part of the product.

usage: python tools/shard_probe.py [config] [K] [tile sizes, e.g. 16,32,64]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_frame_us(r, cam, vp, frames, gi, reps=3):
    print(f"  [{time.strftime('%X')}] {frames} frames ...", flush=True)
    r.render_frames(frames, cam, vp, gi_per_frame=gi)      # warm: tile lists, cost order
    r.sync()
    best = 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        r.render_frames(frames, cam, vp, gi_per_frame=gi)
        r.sync()
        best = min(best, (time.perf_counter() - t0) / frames * 1e6)
    return best


def main():
    import faulthandler
    faulthandler.dump_traceback_later(45, repeat=True)   # a stuck call names itself
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, pose_f32

    cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sizes = [int(t) for t in (sys.argv[3] if len(sys.argv) > 3 else "16,32,64").split(",")]
    torch.cuda.set_device(0)
    W, H = cfg.width, cfg.height
    r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=load_atlas())
    # the tool's own knobs (tools/measure.sh): run-time options of the library (include/rvgrt.h rv_option)
    if os.environ.get("RV_GI_SHARD_PROBE"):
        r.set_option(rv.RV_OPT_GI_SHARD_PROBE, 1)
    if os.environ.get("RV_PIPE_ORDER"):
        r.set_option(rv.RV_OPT_PIPE_ORDER, int(os.environ["RV_PIPE_ORDER"], 16))
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    r.sync()
    pos, yaw, pitch = pose_f32(cfg)
    cam, vp = rv.camera_from_pose(pos, yaw, pitch, W, H)
    frames = max(4 * K, 32)   # the pipelined GI loop's prologue amortised over the call
    if int(os.environ.get("SHARD_GROUP", "0")) >= 2:
        frames = 128          # grouped frames: a longer call for the group loop's prologue
    r.set_frames_in_flight(K)
    r.set_frame_group(int(os.environ.get("SHARD_GROUP", "0")))   # grouped reference frames
    r.set_tile_shard(64, 0, 0)
    gi = cfg.gi_per_frame
    full = per_frame_us(r, cam, vp, frames, gi)
    print(f"{cfg.name}: whole frame {full:.1f} us/frame at K={K}", flush=True)
    for T in sizes:
        for N in [int(v) for v in os.environ.get("SHARD_NS", "2,4,8").split(",")]:
            t = []
            for rank in range(N):
                r.set_tile_shard(T, rank, N)
                t.append(per_frame_us(r, cam, vp, frames, gi))
            mx = max(t)
            print(f"  tile {T:2d} N={N}: slowest rank {mx:7.1f} us/frame, mean {sum(t) / N:7.1f}, "
                  f"render-bound speedup {full / mx:5.2f}x  ranks: " + " ".join(f"{v:.0f}" for v in t), flush=True)
    if os.environ.get("PROBE_ROOT"):
        # rank 0's extra work at any N: the whole frame's untile (and the gather path) --
        # one rank holding every tile, assembled locally and through a one-rank RCCL communicator
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        for T in sizes:
            r.set_tile_shard(T, 0, 1)
            local = per_frame_us(r, cam, vp, frames, gi)
            comm = rv.Comm(r, rv.Comm.unique_id(), 1, 0)
            r.render_frames(frames, cam, vp, gi_per_frame=gi, comm=comm)
            r.sync()
            best = 1e30
            for _ in range(3):
                t0 = time.perf_counter()
                r.render_frames(frames, cam, vp, gi_per_frame=gi, comm=comm)
                r.sync()
                best = min(best, (time.perf_counter() - t0) / frames * 1e6)
            comm.close()
            print(f"  tile {T:2d}, one rank holding every tile: local untile {local:7.1f} us/frame, "
                  f"RCCL path {best:7.1f} us/frame (whole frame {full:.1f})", flush=True)
        dist.destroy_process_group()
    if gi and os.environ.get("PROBE_STAGES"):
        # one frame at a time (no pipelining): stand-alone launch time of each stage for
        # rank 0's share -- which part's longest wave bounds a pipelined launch
        import rvgrt_amd._lib as L
        r.set_pipeline(0)
        for T in sizes:
            for N in (1, 8):
                r.set_tile_shard(T, 0, N)
                r.render_frames(8, cam, vp, gi_per_frame=True)
                r.timing_enable(40)
                r.render_frames(16, cam, vp, gi_per_frame=True)
                r.sync()
                ms, _ = r.timing_stages()
                n = r.timing_launches()
                r.timing_enable(0)
                print(f"  stages tile {T} rank 0 of {N}: " + ", ".join(
                    f"{k} {ms[k] / n[k] * 1e3:.0f} us" for k in L.STAGES if n[k]), flush=True)
        r.set_pipeline(1)
    r.set_tile_shard(64, 0, 0)
    r.close()


if __name__ == "__main__":
    main()
