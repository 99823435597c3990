#!/usr/bin/env python3
"""Host-side cost per frame of the screen-tile path, measured on ONE GPU.

Times (CPU wall per call, no device sync inside the loop, then the device
time of the same loop): rv_frame, rv_frame_tiles + rv_untile for the share
one of N ranks renders, torch.distributed.gather on a one-rank "nccl" group,
and a hipGraph (torch.cuda.CUDAGraph) replay of the tile frame.  Used to size
the multi-GPU frame loop; not part of the product.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def wall(fn, n):
    fn()                     # warm: allocations and first-use set-up stay out of the timing
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6


def main():
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas
    from rvgrt_amd.configs import CONFIGS, pose_f32
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    quick = len(sys.argv) > 2 and sys.argv[2] == "quick"   # rv_frame + per-rank tile shares only
    W, H = cfg.width, cfg.height
    r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=cfg.flags, atlas=load_atlas())
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    r.sync()
    pos, yaw, pitch = pose_f32(cfg)
    cam, vp = rv.camera_from_pose(pos, yaw, pitch, W, H)
    n = 200
    out = {}
    out["frame"] = wall(lambda: r.frame(cam, vp), n)
    # native loop, rank 0's share of an N-rank tile shard without the gather:
    # the per-rank render rate the multi-GPU loop can reach
    for N in (1, 8):
        for K in [int(k) for k in os.environ.get("HO_K", "1,2,4,8").split(",")]:
            r.set_frames_in_flight(K)
            r.set_tile_shard(64, 0, N)
            c, d = wall(lambda: r.render_frames(40, cam, vp), 10)
            out[f"native_N{N}_K{K}"] = (c / 40, d / 40)
    r.set_tile_shard(64, 0, 0)
    for K in (2, 3, 4):
        r.set_frames_in_flight(K)
        ss = [torch.cuda.Stream() for _ in range(K)]
        seq_no = [0]

        def frame_k():
            k = seq_no[0] % K
            seq_no[0] += 1
            r.set_stream(ss[k].cuda_stream)
            r.frame(cam, vp)
        out[f"frame_K{K}"] = wall(frame_k, n)
        c, d = wall(lambda: r.render_frames(20, cam, vp), n // 20)
        out[f"native_full_K{K}"] = (c / 20, d / 20)
    r.set_frames_in_flight(1)
    r.set_stream(stream.cuda_stream)
    T = 64
    ntiles = ((W + T - 1) // T) * ((H + T - 1) // T)
    for N in (1, 2, 4, 8):
        ids = np.arange(0, ntiles, N, dtype=np.int32)
        maxper = (ntiles + N - 1) // N
        tb = torch.empty(maxper * T * T * 4, dtype=torch.uint8, device="cuda")
        big = torch.empty(N * maxper * T * T * 4, dtype=torch.uint8, device="cuda")
        cat = np.full(N * maxper, -1, np.int32)
        cat[:len(ids)] = ids
        r.bind_tile_buffer(tb.data_ptr(), tb.numel())
        out[f"tiles_N{N}"] = wall(lambda: r.frame_tiles(cam, vp, ids, tile_px=T), n)
        for K in (2, 4):   # K frames in flight on K streams, one tile buffer per slot
            r.set_frames_in_flight(K)
            ss = [torch.cuda.Stream() for _ in range(K)]
            bufs = [torch.empty(maxper * T * T * 4, dtype=torch.uint8, device="cuda") for _ in range(K)]
            seq_no = [0]

            def tiles_k():
                k = seq_no[0] % K
                seq_no[0] += 1
                r.set_stream(ss[k].cuda_stream)
                r.bind_tile_buffer(bufs[k].data_ptr(), bufs[k].numel())
                r.frame_tiles(cam, vp, ids, tile_px=T)
            out[f"tiles_K{K}_N{N}"] = wall(tiles_k, n)
            r.set_frames_in_flight(1)
            r.set_stream(stream.cuda_stream)
            r.bind_tile_buffer(tb.data_ptr(), tb.numel())
        if quick:
            continue
        out[f"untile_N{N}"] = wall(lambda: r.untile(big.data_ptr(), cat, tile_px=T), n)
        lst = [big[:tb.numel()]]
        out[f"gather_N{N}"] = wall(lambda: dist.gather(tb, lst, dst=0), n)
        out[f"gather_async_N{N}"] = wall(lambda: dist.gather(tb, lst, dst=0, async_op=True).wait(), n)

        def seq():
            r.frame_tiles(cam, vp, ids, tile_px=T)
            big[:tb.numel()].copy_(tb)
            r.untile(big.data_ptr(), cat, tile_px=T)
        out[f"tiles+copy+untile_N{N}"] = wall(seq, n)
        # hipGraph of 8 tile frames (render + local copy + untile)
        try:
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                seq()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                r.set_stream(torch.cuda.current_stream().cuda_stream)
                for _ in range(8):
                    seq()
            r.set_stream(stream.cuda_stream)
            c, d = wall(g.replay, n // 8)
            out[f"graph8_N{N}"] = (c / 8, d / 8)
        except Exception as e:   # noqa: BLE001
            r.set_stream(stream.cuda_stream)
            out[f"graph8_N{N}"] = f"capture failed: {e!r}"[:200]
    for k, v in out.items():
        if isinstance(v, tuple):
            print(f"{k:28s} cpu {v[0]:8.1f} us/call   cpu+gpu {v[1]:8.1f} us/call")
        else:
            print(f"{k:28s} {v}")
    r.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
