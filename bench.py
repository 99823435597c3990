#!/usr/bin/env python3
"""bench.py -- Mrays/s and frames/s of the MI355X render path.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N>1
launched by torch.distributed.run, one rank per GPU.  One step = one frame
of the configured workload, inputs resident in HBM.  Default C4 (BASELINE
configs[3], the north star's 1-GPU target): 1024^3 procedural world,
3840x2160, the reference frame (half-res pre-pass, water reflection +
reflection shadow, 6-cone voxel GI) over a GI grid after 2 full sweeps, with
the reference's per-frame GI update (UpdateGIData, 262144 cells) before every
frame.  W untimed frames, then K timed frames bracketed by a barrier +
device synchronize on both sides; the time is the max over ranks.  Rank 0
prints ONE JSON line.  Before the W warm-up frames, --settle (default 100)
tops the untimed frames up to that many (reported as "settle_frames"): the
first frames of the camera path, rendered by the same loop, after which the
path starts again, so the warm-up and timed frames -- the views measured --
are the same as without it.  The GPU's clocks and caches need tens of ms
after the set-up's idle gaps, far more than a handful of 0.4-ms frames.
Only the camera restarts: the settle frames run the per-frame GI update too
(UpdateGIData before every drawCUDA, src/main.cpp:119-132), so the GI grid and
its rolling window are those of a run that has rendered the settle frames
already -- as in any longer run of the reference's loop, whose grid never
stops updating.

Drop-in leg (one GPU, C3-C5, --dropin-leg 1): after the timed region the same
context renders --steps more frames through renderLoop's own calls
(rv_update_gi_data, then rv_draw_cuda of that frame's camera; no camera
look-ahead), timed the same way, reported as "dropin" with its own roofline.

Multi-GPU: the frame is split into interleaved screen tiles (rv_set_tile_shard),
every rank renders its tiles of the same frame against its own locally
generated replica of the world and 1/N of the GI update's cells (RCCL
all-gather), and rank 0 gathers the packed tiles over RCCL and assembles the
frame: strong scaling of a fixed frame.  `--gpus N` is honoured either way:
under a launcher (torch.distributed.run) WORLD_SIZE must equal N; without one
(WORLD_SIZE unset, N > 1) this process starts N rank processes of itself
before touching the GPU and prints rank 0's line.

Loop modes.  `value` is measured in the same loop mode at every N, the one
N = 1 uses for the config (C4/C5: one pipelined launch per frame; C3: 8-frame
groups), so a 1 -> 8 curve compares like with like.  For reference frames the
line also reports the other mode ("modes": per-frame vs grouped 16-frame
launches), timed on the same context after the main region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(st: dict, px: int, halfpx: int, prepass: bool, stage: str, pp_hits: int = 0) -> int:
    """Bytes one launch of a stage must move (SURVEY.md s8(d) model, split by
    wavefront stage).  Traversal: 4 B per DDA voxel test, 1 B per CSDF read
    (sphere step or every-8th-step check); 5 B per cone step (1 B CSDF + 4 B
    GI); 16 B per texture sample.  Stage I/O: hit records (16 B position +
    4 B info), 4 B queue entries, 16 B secondary results, pre-pass outputs
    (4+4 B), 4 point + 4 bilinear half-res taps (32 B), outputs 10 B/px."""
    b = 4 * st["dda_steps"] + st["sphere_steps"] + st["csdf_checks"]
    b += 5 * st["cone_steps"] + 16 * st["tex_samples"]
    if stage == "pp_primary":   # 4 B distance per pixel; 16 B hit + 4 B queue per hit, else 4 B shadow
        b += halfpx * 4 + pp_hits * 20 + (halfpx - pp_hits) * 4
    elif stage == "pp_shadow":
        b += st["prepass_shadow"] * (4 + 16 + 4)
    elif stage == "primary":
        b += px * (20 + (16 if prepass else 0))
    elif stage == "shadow":
        b += st["shadow"] * (4 + 20 + 4)
    elif stage == "water":
        b += st["refl"] * (4 + 20 + 16)
    elif stage == "cones":
        b += (st["cones"] // 6) * (4 + 20 + 16)
    elif stage == "shade":
        b += px * (20 + 10 + (16 if prepass else 0))
    elif stage == "fused_prepass":   # k_prepass: 4 B distance + 4 B shadow per half-res pixel
        b += halfpx * 8
    elif stage == "fused_render":    # k_render: 10 B outputs; 4 min-dist + 4 bilinear taps (32 B)
        b += px * (10 + (32 if prepass else 0))
    return int(b)


def binding_limit(tj: dict, launch_ms: float):
    """What binds the profiled kernel, from its PMC summary (profiles/traffic_<config>.json, counters per
    launch summed over the 8 XCDs; GRBM_GUI_ACTIVE is per XCD, so /8): the busy fraction of the 256
    texture-data units (TD: the vector-memory return path of every gather), the VALU issue fraction (a
    wave64 VALU instruction takes 2 cycles of a SIMD: 2 per CU-cycle on 4 SIMDs) and the HBM traffic
    fraction of the 8 TB/s peak.  The largest names the limit."""
    c = tj.get("counters_avg_per_launch", {})
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if cyc <= 0:
        return None
    td = c.get("TD_TD_BUSY_sum", 0.0) / (256.0 * cyc)
    ta = c.get("TA_TA_BUSY_sum", 0.0) / (256.0 * cyc)
    valu = c.get("SQ_INSTS_VALU", 0.0) / (2.0 * 256.0 * cyc)
    hbm = tj.get("hbm_bytes_per_launch", 0) / (launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS if launch_ms > 0 else 0.0
    fr = {"td_busy": td, "valu_issue": valu, "hbm_traffic": hbm}
    name = max(fr, key=fr.get)
    label = {"td_busy": "vector-memory return path (TD busy)", "valu_issue": "VALU issue",
             "hbm_traffic": "HBM bandwidth"}[name]
    return {"name": label, "td_busy": round(td, 3), "ta_busy": round(ta, 3), "valu_issue": round(valu, 3),
            "hbm_traffic": round(hbm, 3), "source": os.path.relpath(tj.get("_path", ""), ROOT) if tj.get("_path") else None}


def bench_config(name, resolution=None, world=None):
    """CONFIGS[name], or its frame at another size ("WxH", any >= 2, odd too) and / or on a cubic world
    of another size (`world` = log2 of the side, 4..11)."""
    import dataclasses
    import re
    from rvgrt_amd.configs import CONFIGS
    cfg = CONFIGS[name]
    if resolution:
        rw, rh = (int(v) for v in resolution.lower().split("x"))
        if rw < 2 or rh < 2:
            raise SystemExit(f"--resolution {resolution}: each side must be >= 2")
        cfg = dataclasses.replace(cfg, width=rw, height=rh,
                                  describe=re.sub(r"\d+x\d+", f"{rw}x{rh}", cfg.describe, count=1))
    if world:
        if not 4 <= int(world) <= 11:
            raise SystemExit(f"--world {world}: log2 of the cube side, 4 .. 11")
        n = 1 << int(world)
        cfg = dataclasses.replace(cfg, log2_n=int(world),
                                  describe=re.sub(r"\d+\^3", f"{n}^3", cfg.describe, count=1))
    return cfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle", type=int, default=100,
                    help="untimed frames of the same loop before the --warmup frames bring the total untimed "
                         "frames to at least this many (0: off): a 4K frame is ~0.4 ms, and the GPU's clocks and "
                         "caches take tens of ms to settle after the set-up's idle gaps (20 timed frames after 5 "
                         "warm-up frames read 0.444 ms/frame, after 100 0.429, 200 after 20 0.425; "
                         "profiles/r04/settle.txt)")
    ap.add_argument("--config", default="c4",
                    help="c1..c5 (default c4: 1024^3, 3840x2160, the reference frame with 2-bounce GI and a GI "
                         "update every frame -- the north star's 1-GPU workload, BASELINE configs[3])")
    ap.add_argument("--pose", default="P0")
    ap.add_argument("--world", type=int, default=None,
                    help="log2 of a cubic world's side (4..11): the config's frame on another world size")
    ap.add_argument("--resolution", default=None,
                    help="WxH: the config's world and frame at another frame size (e.g. 1707x961, a DLSS render size)")
    ap.add_argument("--camera", default="path", choices=["path", "static"],
                    help="path (default): frames differ -- the reference's jitter sequence as drawCUDA maps it "
                         "with ref_compat (time), a yaw pan of --pan rad/frame, previous VP per frame; "
                         "static: one camera for every frame (round 1)")
    ap.add_argument("--pan", type=float, default=0.0005, help="yaw change per frame of the camera path (rad)")
    ap.add_argument("--tile-px", type=int, default=None,
                    help="screen-tile size of the N>1 shard (default: 16 px without the pre-pass, 64 with it; "
                         "tools/shard_probe.py: C2 at 8 ranks renders its slowest share in 19.6 us/frame at "
                         "16 px vs 30.9 at 64 px; the pipelined C4 share at 2/4/8 ranks in 288/181/162 us at "
                         "64 px vs 303/194/168 at 32, the half-res halo costing less)")
    ap.add_argument("--root-weight", type=float, default=None,
                    help="N>1 native loop: rank 0's share of tiles relative to the others (rank 0 also receives "
                         "and assembles every frame); default 1 - 0.019 (N-1): its measured assembly cost is "
                         "1.9%% of a whole frame's render (profiles/r01_shard_probe_c2_root.log)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU-baseline budget (rank 0, N=1); 0 disables")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (default 0: every core this process may use -- nproc, bounded by a "
                         "cgroup CPU quota)")
    ap.add_argument("--dump", default="", help="write the rank-0 frame as PNG here")
    ap.add_argument("--path", default="fused", choices=["fused", "wavefront"],
                    help="frame path: per-pixel megakernels (default) or wavefront stage kernels")
    ap.add_argument("--stream-priority", type=int, default=-1,
                    help="torch stream priority of the frame stream (0: the default stream)")
    ap.add_argument("--gi-per-frame", type=int, default=None,
                    help="experiments only: override the config's per-frame GI update (0/1)")
    ap.add_argument("--gi-async", type=int, default=1, help="overlap the GI update with the previous render")
    ap.add_argument("--pipe", type=int, default=1,
                    help="native loop, per-frame GI + pre-pass (C3-C5), one GPU: one k_ref_pipe launch per frame "
                         "runs render k | GI update k+1 | pre-pass k+1 (0: one frame at a time)")
    ap.add_argument("--group", type=int, default=None,
                    help="native loop, reference frames (C3-C5): frames per launch of the grouped loop "
                         "(rv_set_frame_group; GI update split into traced records + a per-frame combine, "
                         "phase A sharded over the ranks); 0 = the per-frame pipeline")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 collective backend; gloo (host-staged gather, ranks may share a GPU) "
                         "only rehearses the multi-rank path")
    ap.add_argument("--inflight", type=int, default=None,
                    help="frame slots (default 16; C2 on one GPU: 8 -> 0.1427, 16 -> 0.1403, 32 -> 0.1420 ms/frame): "
                         "the native loop renders groups of "
                         "that many frames per launch (the group's tail is shared by its frames; its RCCL "
                         "gather overlaps the next group); the Python loop puts frame k on stream k %% n; "
                         "1 = one frame at a time")
    ap.add_argument("--loop", default="native", choices=["native", "python", "drawcuda"],
                    help="frame loop: rv_render_frames (C++: slots, streams, RCCL gather, untile), the "
                         "per-frame Python loop over the same library calls (torch.distributed gather), or "
                         "drawcuda: renderLoop's own calls, rv_update_gi_data then rv_draw_cuda, one frame per "
                         "call and no knowledge of the next camera (the drop-in path, src/main.cpp:119-132)")
    ap.add_argument("--flow", type=int, default=1,
                    help="python/drawcuda loops: one k_ref_flow launch per frame (rv_set_flow; 0 = drawCUDA's "
                         "two launches with the GI update on the side stream)")
    ap.add_argument("--flags", type=int, default=None,
                    help="experiments only: override the config's RV_F_* flags")
    ap.add_argument("--alt-mode", type=int, default=1,
                    help="reference frames, native loop: after the timed region, time the other loop mode (per-frame "
                         "pipelined launches vs grouped launches of --alt-group frames) and report both under "
                         "\"modes\"; 0 = off")
    ap.add_argument("--alt-group", type=int, default=16,
                    help="frames per launch of the grouped mode the alternate leg times (default 16)")
    ap.add_argument("--rehearse", action="store_true",
                    help="no GPU: only the rank plumbing (spawn or launcher, gloo process group, barrier, max-over-"
                         "ranks timing) and one JSON line -- the CPU test of --gpus N")
    ap.add_argument("--dropin-leg", type=int, default=1,
                    help="one GPU, native loop, reference frames (C3-C5): after the timed region, time the same "
                         "number of frames through renderLoop's own calls (rv_update_gi_data, then rv_draw_cuda, "
                         "one frame per call, no knowledge of the next camera: src/main.cpp:119-132) and report "
                         "them as \"dropin\" (ms/frame, cold latency, that loop's roofline); 0 = off")
    args = ap.parse_args()

    # --gpus N: under a launcher WORLD_SIZE must agree; without one, start the N ranks here, before any
    # GPU call (this process never initialises the GPU: it only waits for its children)
    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is None and args.gpus > 1:
        return spawn_ranks(args.gpus, sys.argv[1:])
    if env_ws is not None and int(env_ws) != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_ws} ranks")
        return 2
    if args.rehearse:
        return rehearse(args)

    import torch
    import rvgrt_amd as rv
    from rvgrt_amd.atlas import load_atlas, write_png
    from rvgrt_amd.configs import CONFIGS, camera_path, pose_f32

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world_size > 1:
        import torch.distributed as dist
        if args.dist_backend == "gloo":   # rehearsal: ranks may share the GPUs there are
            local_rank = local_rank % torch.cuda.device_count()
            torch.cuda.set_device(local_rank)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local_rank)

    def barrier():
        if dist is not None:
            dist.barrier()

    cfg = bench_config(args.config, args.resolution, args.world)
    gi_per_frame = cfg.gi_per_frame if args.gi_per_frame is None else bool(args.gi_per_frame)
    W, H = cfg.width, cfg.height
    flags = cfg.flags if args.flags is None else args.flags
    prepass = bool(flags & rv.RV_F_PREPASS)
    atlas = load_atlas()

    # ---------------------------------------------------------------- world
    r = rv.StateRender((cfg.log2_n,) * 3, W, H, flags=flags, atlas=atlas, device=local_rank)
    if world_size > 1:
        # N > 1: the native loop's groups alternate over two streams, so one group's tail overlaps the
        # next (one rank's C2 share at 8 ranks 19.6 -> 19.1 us/frame, profiles/r01_shard_probe_c2_streams.log);
        # one GPU keeps one stream so each launch runs alone and its event time is the kernel's own
        r.set_option(rv.RV_OPT_BATCH_STREAMS, 2)
    # the frame stream runs at the highest priority: the library's GI side
    # stream is created at the lowest, so the GI kernel fills the frame's gaps
    stream = torch.cuda.Stream(device=dev, priority=args.stream_priority) if args.stream_priority else \
        torch.cuda.current_stream(dev)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)
    r.set_frame_path(args.path)
    # frame slots = frames per group of the native loop.  A per-frame GI update
    # serialises the renders (each reads the grid the previous update wrote):
    # with slots only the pre-pass is grouped (--inflight 8: C3 0.435 -> 0.393
    # ms, but C4 0.724 -> 0.816 ms: the GI kernel then overlaps only the
    # render, not the pre-pass), so GI configs default to one frame at a time.
    nfl = args.inflight if args.inflight is not None else (1 if gi_per_frame else 16)
    nfl = max(1, nfl if args.path == "fused" else 1)
    r.set_frames_in_flight(nfl)
    # frame k is submitted on streams[k % nfl] (streams[0] = the context's stream)
    streams = [stream] + [torch.cuda.Stream(device=dev, priority=args.stream_priority) for _ in range(nfl - 1)]
    r.set_gi_async(args.gi_async)
    r.set_pipeline(args.pipe)
    r.set_flow(args.flow)
    drawcuda = args.loop == "drawcuda"
    if drawcuda and world_size > 1:
        raise SystemExit("--loop drawcuda is the one-GPU drop-in loop")
    # Grouped reference frames (rv_set_frame_group) when a rank's render part is latency-bound (<= 48 K
    # waves of 64 pixels, as the latency-mode pipelined variant): the group's frames share one tail.
    # tools/shard_probe.py (profiles/r03/), 64-px tiles: C3 on one GPU 0.2234 -> 0.2063 ms
    # at 8 frames per launch (0.2089 at 16); the slowest C4 rank share at 8 ranks 163.5 -> 93.2 -> 87.7 us/frame
    # at 8 / 16, C5 198.1 -> 122.0 -> 114.1, at 4 ranks C4 182.4 -> 162.0 at 16.  Throughput-bound launches
    # keep the per-frame pipeline: C4 one GPU 0.491 -> 0.553 ms at 16, a 2-rank C4 share 278.9 -> 307.5 us.
    # The library caps the group by the GI grid (two groups' updates never overlap).
    # The mode is the one N = 1 runs for this config at every N (like-for-like scaling): C3's 1080p frame
    # (32 K waves) groups 8 frames, C4/C5 (130 K waves) run one pipelined launch per frame.  The other mode
    # is timed after the main region (--alt-mode).
    ref_frames = gi_per_frame and prepass and args.pipe and args.path == "fused"
    one_gpu_waves = W * H // 64
    group = args.group if args.group is not None else (8 if ref_frames and one_gpu_waves <= 49152 else 0)
    r.set_frame_group(group)
    t0 = time.perf_counter()
    r.world_build()
    for s in range(max(cfg.gi_sweeps, 0)):
        r.gi_update(s)
    r.sync()
    world_s = time.perf_counter() - t0
    log(f"[rank {rank}] world {cfg.n}^3 built in {world_s:.2f}s")

    pos, yaw, pitch = pose_f32(cfg, args.pose)
    # ---------------------------------------------------------------- camera path
    # Every frame differs, as in the reference's renderLoop: Character::Update's jitter sequence, mapped
    # as drawCUDA maps it with ref_compat (time <- jitterY, jitter 0; src/StateRender.cu:15-29), a yaw
    # pan of --pan rad per frame, and each frame's previous VP = the frame before's (motion vectors).
    # frames the run takes from the path: warm-up, timed, the stage-timing pass, 9 latency frames
    n_stage_frames = nfl * max(1, min(args.steps // nfl, 10)) if nfl > 1 else min(args.steps, 10)
    if group >= 2:   # whole groups: the timing pass records only full-group launches
        n_stage_frames = group * max(3, min(args.steps // group, 6))
    # --settle: untimed frames before the warm-up, taken from the start of the camera path, which then
    # starts again -- the warm-up and timed frames are the same frames (the same views) with or without it
    settle = max(0, args.settle - args.warmup)
    w0 = args.warmup                              # the first timed frame of the path
    alt_group = 0 if group >= 2 else max(2, args.alt_group)   # the alternate leg's frames per launch
    n_alt = (args.warmup + args.steps + 2 * max(alt_group, 1) + 5 * alt_group) if args.alt_mode else 0
    n_path = max(w0 + args.steps + n_stage_frames + 9 + 2 + 5 * max(group, 0) + n_alt, settle + 1)   # + the group-latency calls
    pan = args.pan if args.camera == "path" else 0.0
    path = camera_path((pos, yaw, pitch), W, H, n_path, pan=pan, ref_compat=args.camera == "path")
    if args.camera == "static":   # the round-1 bench: one camera, time 0, no jitter
        c0, vp0 = rv.camera_from_pose(pos, yaw, pitch, W, H)
        path = [rv.frame_desc(c0, vp0)] * (n_path + 1)
    cursor = [0]            # next frame of the path

    def take(k):
        a = cursor[0]
        cursor[0] += k
        return path[a:a + k], path[a + k]

    # ---------------------------------------------------------------- work census
    # Frames with counters on: rays per frame and algorithmic bytes, the mean
    # over 8 frames spread over the timed part of the path.
    census = np.linspace(w0, w0 + max(args.steps - 1, 0), 8).astype(int)
    r.stats_reset()
    for i in census:
        d = path[i]
        r.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                jx=d.jitter_x, jy=d.jitter_y,
                flags=flags | rv.RV_F_STATS | (rv.RV_F_REF_FETCH if drawcuda else 0))

    def mean_stats(st):
        return {k: int(round(v / len(census))) for k, v in st.items()}
    st_all = mean_stats(r.stats(-1))
    st_stage = {name: mean_stats(r.stats(k)) for k, name in enumerate(rv._lib.STAGES)}
    rays_per_frame = st_all["traces"]
    gi_stats = None
    if gi_per_frame:   # one UpdateGIData with step counters on: the GI update's algorithmic bytes
        r.set_gi_stats(1)
        r.stats_reset()
        r.update_gi_data()
        r.sync()
        gi_stats = r.stats(rv._lib.STAGES.index("gi"))
        r.set_gi_stats(0)
    megakernel = args.path == "fused"
    pp_hits = st_stage["pp_shadow"]["prepass_shadow"]
    stage_bytes = {name: algorithmic_bytes(st_stage[name], W * H, (W // 2) * (H // 2), prepass,
                                           {"pp_primary": "fused_prepass", "primary": "fused_render"}.get(name, name)
                                           if megakernel else name,
                                           pp_hits)
                   for name in rv._lib.STAGES if name != "gi"}
    if gi_stats is not None:   # traversal + 16 B texel + 4 B bounce GI read per texture sample, 8 B per cell
        gi_cells = min(262144, (cfg.n // 4) ** 3)
        stage_bytes["gi"] = (4 * gi_stats["dda_steps"] + gi_stats["sphere_steps"] + gi_stats["csdf_checks"]
                             + 20 * gi_stats["tex_samples"] + 8 * gi_cells)

    # ---------------------------------------------------------------- tiles
    T = args.tile_px if args.tile_px else (64 if prepass else 16)
    tiles_x, tiles_y = (W + T - 1) // T, (H + T - 1) // T
    ntiles = tiles_x * tiles_y
    my_tiles = np.arange(rank, ntiles, world_size, dtype=np.int32)
    max_per = (ntiles + world_size - 1) // world_size
    all_ids = [np.arange(q, ntiles, world_size, dtype=np.int32) for q in range(world_size)]
    if world_size > 1:
        # Double-buffered: frame k's gather (RCCL stream) overlaps frame k+1's
        # render; rank 0 scatters all ranks' tiles with one rv_untile call.
        nbuf = max(2, nfl)
        tbufs = [torch.empty(max_per * T * T * 4, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        big = ([torch.empty(world_size * max_per * T * T * 4, dtype=torch.uint8, device=dev) for _ in range(nbuf)]
               if rank == 0 else None)
        gather_lists = [list(b.chunk(world_size)) for b in big] if rank == 0 else [None] * nbuf
        cat_ids = np.full(world_size * max_per, -1, dtype=np.int32)   # -1: padding slot
        for q in range(world_size):
            cat_ids[q * max_per:q * max_per + len(all_ids[q])] = all_ids[q]
    pending = []
    frame_no = [0]
    serial = [False]        # timing pass: every frame on streams[0]
    native = args.loop == "native" and (world_size == 1 or args.dist_backend == "nccl")
    comm = None
    root_weight = None
    if native and world_size > 1:
        # RCCL communicator of the library (joins torch's librccl); id from rank 0.
        # Any rank that cannot load RCCL or create its side makes every rank
        # fall back to the Python loop's torch.distributed gather.
        root_weight = args.root_weight if args.root_weight is not None else 1.0 - 0.019 * (world_size - 1)
        r.set_tile_shard(T, rank, world_size, root_weight=root_weight)   # identical on every rank
        from rvgrt_amd.tiles import shard_owners
        my_tiles = np.flatnonzero(shard_owners(W, H, T, world_size, root_weight) == rank).astype(np.int32)
        uid = torch.zeros(rv.Comm.ID_BYTES + 1, dtype=torch.uint8, device=dev)
        if rank == 0:
            try:
                uid[:-1].copy_(torch.tensor(list(rv.Comm.unique_id()), dtype=torch.uint8))
                uid[-1] = 1
            except rv.RvError as e:
                log(f"[rank 0] rv_comm_unique_id failed ({e}); falling back to the Python loop")
        dist.broadcast(uid, src=0)
        ok = torch.tensor([int(uid[-1].item())], dtype=torch.int32, device=dev)
        if ok.item():
            try:
                comm = rv.Comm(r, bytes(uid[:-1].cpu().tolist()), world_size, rank)
            except rv.RvError as e:
                log(f"[rank {rank}] rv_comm_create failed ({e}); falling back to the Python loop")
                ok.zero_()
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if not ok.item():
            if comm is not None:
                comm.close()
                comm = None
            r.set_tile_shard(T, 0, 0)
            native = False
            my_tiles = np.arange(rank, ntiles, world_size, dtype=np.int32)   # the Python loop's interleave

    def run_native(k):
        r.set_stream(stream.cuda_stream)
        seq, nxt = take(k)
        r.render_frame_seq(seq, next_desc=nxt, flags=flags, gi_per_frame=gi_per_frame, comm=comm)

    def frame_args():
        d = take(1)[0][0]
        return (d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp)), \
            {"time": d.time, "jx": d.jitter_x, "jy": d.jitter_y, "flags": flags}

    def issue_gather(b):
        if args.dist_backend == "nccl":
            return dist.gather(tbufs[b], gather_lists[b], dst=0, async_op=True)
        host = tbufs[b].cpu()        # gloo rehearsal: host-staged, synchronous
        lst = [torch.empty_like(host) for _ in range(world_size)] if rank == 0 else None
        dist.gather(host, lst, dst=0)
        if rank == 0:
            big[b].copy_(torch.cat(lst).to(dev))
        return None

    def finish():
        work, b, s = pending.pop(0)
        with torch.cuda.stream(s):
            if work is not None:
                work.wait()          # this frame's stream waits for its gather (GPU-side)
            if rank == 0:
                r.set_stream(s.cuda_stream)
                r.untile(big[b].data_ptr(), cat_ids, tile_px=T)

    def step():
        k = frame_no[0]
        frame_no[0] += 1
        s = streams[0] if serial[0] else streams[k % nfl]
        if drawcuda:   # renderLoop (src/main.cpp:119-132): UpdateGIData, then drawCUDA of this frame's camera
            d = take(1)[0][0]
            r.set_stream(s.cuda_stream)
            if gi_per_frame:
                r.update_gi_data()
            c = d.cam   # ref_compat drawCUDA: time <- jitterY argument (src/StateRender.cu:15-29)
            r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                        np.ctypeslib.as_array(d.prev_vp), jitter_x=0.0, jitter_y=d.time)
            return
        fa, fk = frame_args()
        if world_size == 1:
            r.set_stream(s.cuda_stream)
            if gi_per_frame:
                r.update_gi_data()   # renderLoop: UpdateGIData before drawCUDA
            r.frame(*fa, **fk)
            return
        b = k % nbuf
        with torch.cuda.stream(s):
            r.set_stream(s.cuda_stream)
            if gi_per_frame:
                r.update_gi_data()
            r.bind_tile_buffer(tbufs[b].data_ptr(), tbufs[b].numel())
            r.frame_tiles(fa[0], fa[1], my_tiles, tile_px=T, prev_vp=fa[2], time=fk["time"], jx=fk["jx"],
                          jy=fk["jy"], flags=flags)
            work = issue_gather(b)   # the gather waits for this frame's render on stream s
        pending.append((work, b, s))
        if nfl == 1 and len(pending) > 1:
            finish()                 # one frame at a time: untile frame k-1 while k renders
        elif nfl > 1:
            finish()                 # frames in flight: untile on the frame's own stream

    def drain():
        while pending:
            finish()

    if settle:
        if native:
            run_native(settle)
        else:
            for _ in range(settle):
                step()
            drain()
        cursor[0] = 0        # the warm-up and timed frames start the path again
    if native:
        run_native(args.warmup)
    else:
        for _ in range(args.warmup):
            step()
        drain()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)

    t0 = time.perf_counter()
    if native:
        run_native(args.steps)
    else:
        for _ in range(args.steps):
            step()
        drain()
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    # Per-stage kernel times from HIP events on the context's streams, in a
    # separate pass of the same loop after the timed region, one record per
    # launch, as rocprof sees them.  The native loop launches groups of nfl
    # frames (frame slots); with a per-frame GI update only the pre-pass is
    # grouped and the render runs frame by frame.
    grouped = native and args.path == "fused" and nfl > 1
    # pipelined reference frames: every launch is k_ref_pipe (timed as stage "primary"); with N > 1
    # ranks a rank's launch holds its tiles and 1/N of the GI update's cells
    piped = native and args.path == "fused" and args.pipe and gi_per_frame and bool(flags & rv.RV_F_PREPASS)
    # flow frames (the per-frame loops): every frame is one k_ref_flow launch (stage "primary") holding
    # its pre-pass, its render and the next UpdateGIData's cells
    flowed = (not native and world_size == 1 and args.flow and args.path == "fused" and nfl == 1
              and bool(flags & rv.RV_F_PREPASS))
    gi_groups = grouped and gi_per_frame and bool(flags & rv.RV_F_PREPASS) and world_size == 1 and not piped
    fpl = nfl if (grouped and not gi_per_frame) else 1
    # grouped reference frames: the effective group size (the library caps it by the GI grid)
    ref_group = r.frame_group_effective() if piped and group >= 2 else 0
    if ref_group >= 2:
        fpl = ref_group
    stage_fpl = {name: fpl for name in rv._lib.STAGES}
    if gi_groups:
        stage_fpl["pp_primary"] = nfl
    if not grouped and ref_group < 2:   # (grouped reference frames keep whole groups: only launches whose
        n_stage_frames = min(args.steps, 10)   # three parts are all full are timed)
    serial[0] = True
    r.timing_enable(2 * n_stage_frames + 2)
    if native:
        run_native(n_stage_frames)
    else:
        for _ in range(n_stage_frames):
            step()
        drain()
    torch.cuda.synchronize(dev)
    per_stage_ms, _ = r.timing_stages()
    launches = r.timing_launches()
    r.timing_enable(0)
    barrier()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # single-frame latency: one frame per call, submitted and waited for alone (median of 9)
    # (the per-frame loops: the frame's UpdateGIData + drawCUDA calls from an idle device to completion)
    lat = []
    if native or world_size == 1:
        for _ in range(9):
            barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            if native:
                run_native(1)
            else:
                step()
                drain()
            torch.cuda.synchronize(dev)
            lat.append((time.perf_counter() - t1) * 1000.0)
    latency_ms = round(float(np.median(lat)), 4) if lat else None
    latency_mode = (("native loop, one-frame calls (each hands over the next frame's camera)" if native else
                     "cold renderLoop frame: UpdateGIData + drawCUDA of one frame from an idle device")
                    if lat else None)
    # grouped reference frames: a frame's latency in the timed loop is its whole group's -- submit F frames from an
    # idle device to the completion of their launch (the group's frames are delivered together)
    group_latency_ms = None
    if native and ref_group >= 2:
        gl = []
        for _ in range(5):
            barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            run_native(ref_group)
            torch.cuda.synchronize(dev)
            gl.append((time.perf_counter() - t1) * 1000.0)
        group_latency_ms = round(float(np.median(gl)), 4)

    # ---------------------------------------------------------------- the other loop mode
    # Reference frames in the native loop: the same context, world and camera path (continued), timed in the
    # mode the main region did not run -- per-frame pipelined launches vs grouped launches -- so both modes'
    # 1 -> N curves exist, each like with like.
    modes = None
    if args.alt_mode and native and ref_frames and bool(flags & rv.RV_F_PREPASS):
        def max_over_ranks(v):
            if dist is None:
                return v
            t = torch.tensor([v], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
        main_ms = elapsed * 1000.0 / args.steps
        main_name = "grouped" if ref_group >= 2 else "per_frame"
        modes = {main_name: {"frames_per_launch": ref_group if ref_group >= 2 else 1, "ms_per_step": round(main_ms, 4),
                             "value": round(rays_per_frame / main_ms / 1e3, 2), "latency_ms": group_latency_ms
                             if ref_group >= 2 else latency_ms, "steps": args.steps, "is_value": True}}
        r.set_frame_group(alt_group)
        eff = r.frame_group_effective()
        per = eff if eff >= 2 else 1
        n_alt_steps = ((args.steps + per - 1) // per) * per
        run_native(((max(args.warmup, per) + per - 1) // per) * per)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        run_native(n_alt_steps)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        alt_el = max_over_ranks(time.perf_counter() - t1)
        al = []
        for _ in range(3):
            barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            run_native(per)
            torch.cuda.synchronize(dev)
            al.append((time.perf_counter() - t1) * 1000.0)
        alt_ms = alt_el * 1000.0 / n_alt_steps
        modes["grouped" if eff >= 2 else "per_frame"] = {
            "frames_per_launch": per, "ms_per_step": round(alt_ms, 4),
            "value": round(rays_per_frame / alt_ms / 1e3, 2), "latency_ms": round(float(np.median(al)), 4),
            "steps": n_alt_steps, "is_value": False}
        r.set_frame_group(group)

    gather_check = None
    if world_size > 1 and rank == 0:   # the gathered frame must equal a one-GPU frame
        tiled = r.readback(rv.RV_IMAGE_COLOR).copy()
        d = path[cursor[0] - 1]   # the last frame rendered
        r.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time, jx=d.jitter_x,
                jy=d.jitter_y, flags=flags)
        full = r.readback(rv.RV_IMAGE_COLOR)
        nbad = int(np.count_nonzero(np.any(tiled != full, axis=-1)))
        gather_check = "exact" if nbad == 0 else f"{nbad} pixels differ"
    if args.dump and rank == 0:
        write_png(args.dump, r.readback(rv.RV_IMAGE_COLOR))

    ms_per_step = elapsed * 1000.0 / args.steps
    fps = args.steps / elapsed
    mrays = rays_per_frame * fps / 1e6

    # average launch time per stage, and its share of a frame
    avg_stage_ms = {k: (per_stage_ms[k] / launches[k] if launches[k] else 0.0) for k in per_stage_ms}
    frame_stage_ms = {k: avg_stage_ms[k] / stage_fpl[k] for k in avg_stage_ms}
    gi_ms = frame_stage_ms["gi"]
    pp_ms = frame_stage_ms["pp_primary"] + frame_stage_ms["pp_shadow"]
    render_ms = sum(v for k, v in frame_stage_ms.items() if k not in ("gi", "pp_primary", "pp_shadow"))
    # dominant kernel: the frame stage with the largest time per frame
    dom = max((k for k in frame_stage_ms if k != "gi"), key=lambda k: frame_stage_ms[k])
    kernel_names = {"pp_primary": "k_prepass" if megakernel else "k_wf_pp_primary",
                    "pp_shadow": "k_wf_pp_shadow",
                    "primary": ("k_ref_group" if ref_group else "k_ref_pipe" if piped else "k_ref_flow" if flowed else
                                "k_render_tiles" if world_size > 1 else "k_render")
                    if megakernel else "k_wf_primary",
                    "shadow": "k_wf_shadow",
                    "water": "k_wf_water", "cones": "k_wf_cones", "shade": "k_wf_shade"}
    dom_ms = avg_stage_ms[dom]
    dom_fpl = stage_fpl[dom]
    dom_bytes = stage_bytes[dom] * dom_fpl
    if (piped or flowed) and dom == "primary":   # the launch also runs a pre-pass and a GI update
        # (grouped: the next group's pre-pass and phase A of the group after; phase B's combine is a
        # separate small kernel, not counted here)
        dom_bytes = (stage_bytes["primary"] + stage_bytes["pp_primary"] + stage_bytes.get("gi", 0)) * dom_fpl
    if world_size > 1:   # per-GPU: this rank's share of the stage's bytes
        dom_bytes = dom_bytes * len(my_tiles) / ntiles
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic = None
    limit = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.config}" + ("" if args.pose == "P0" else f"_{args.pose}")
                         + ("_drawcuda" if flowed else "") + ".json")
    if os.path.exists(tpath) and world_size == 1:   # PMC summaries are of the one-GPU launch
        try:
            tj = json.load(open(tpath))
            tj["_path"] = tpath
            if tj.get("kernel", "").startswith(kernel_names[dom]) and tj.get("frames_per_launch", 1) == dom_fpl:
                traffic = tj.get("hbm_bytes_per_launch")
                limit = binding_limit(tj, dom_ms)
        except Exception:
            traffic = None
    g = st_stage[dom]        # counters of the dominant stage's launch (census frame)
    gathers = (g["sphere_steps"] + g["dda_steps"] + g["csdf_checks"] + 2 * g["cone_steps"]) * dom_fpl
    if (piped or flowed) and dom == "primary":
        for h in (st_stage["pp_primary"], gi_stats):
            gathers += (h["sphere_steps"] + h["dda_steps"] + h["csdf_checks"]) * dom_fpl
    if world_size > 1:
        gathers = gathers * len(my_tiles) / ntiles
    gather_rate = gathers / (dom_ms * 1e-3) if dom_ms > 0 else 0.0
    # "bound" names the axis the roofline is priced on (HBM bytes, the contract's hbm | mfma); what binds the
    # kernel is `limit` (PMC): the vector-memory return path (TD busy) against VALU issue and HBM traffic
    roofline = {"bound": "hbm", "limit": limit, "kernel": kernel_names[dom], "achieved": round(achieved, 2),
                "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                "traffic": traffic, "algorithmic_bytes_per_launch": int(dom_bytes),
                "avg_launch_ms": round(dom_ms, 4), "frames_per_launch": dom_fpl,
                # measured HBM bytes (PMC, profiles/traffic_<config>.json) per launch time against the peak:
                # the memory side's real load, beside frac's algorithmic bytes
                "traffic_frac": (round(traffic / (dom_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                                 if traffic and dom_ms > 0 else None),
                # what binds in practice: traversal gathers per second through the vector
                # L1 / texture path (no ceiling is claimed: coherent gathers cost less than the
                # scattered-gather micro-benchmark's ~1 lane per CU-cycle, so C2 runs above it)
                "gathers_per_launch": int(gathers), "gather_rate": round(gather_rate / 1e9, 2),
                "gather_unit": "G lane-gathers/s"}

    # ---------------------------------------------------------------- drop-in leg
    # renderLoop's own calls (src/main.cpp:119-132): UpdateGIData, then drawCUDA of the frame's camera, one
    # frame per call -- what a caller of the drop-in boundary gets (the native loop above hands over the next
    # frame's camera).  Same context, world and camera path; warm-up + timed frames, a timing pass for the
    # k_ref_flow launch's roofline and the cold latency of one renderLoop frame.
    dropin = None
    if (args.dropin_leg and native and world_size == 1 and not drawcuda and gi_per_frame and prepass
            and args.path == "fused" and args.flow):
        dropin = dropin_leg(r, stream, cfg, flags, pos, yaw, pitch, pan, args, gi_stats, traffic_dir=ROOT)

    # ---------------------------------------------------------------- CPU baseline
    cpu = None
    if rank == 0 and world_size == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(r, cfg, path[w0], flags, atlas, args.cpu_seconds, args.cpu_threads)

    if rank == 0:
        line = {
            "metric": f"Mrays/s ({cfg.name}: {cfg.describe}, pose {args.pose}, "
                      + (f"screen-tile split x{world_size} (RCCL gather))" if world_size > 1 else "1 GPU)"),
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_frames": settle,
            "ms_per_step": round(ms_per_step, 4),
            "fps": round(fps, 2),
            "latency_ms": latency_ms,
            "latency_mode": latency_mode,
            "group_latency_ms": group_latency_ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: procedural world from the reference Evaluate (seed 0), camera pose "
                    f"{args.pose} (reference defaults), random-free",
            "camera": ("per-frame: yaw pan %g rad/frame from the pose, the reference jitter sequence as "
                       "drawCUDA maps it with ref_compat (time <- jitterY), previous VP per frame; rays_per_frame "
                       "= mean of 8 census frames of the timed path" % pan) if args.camera == "path"
                      else "static: one camera, time 0, no jitter",
            "config": {"workload": cfg.name, "world": f"{cfg.n}^3", "resolution": f"{W}x{H}",
                       "flags": flags, "gi_sweeps": cfg.gi_sweeps, "gi_update_per_frame": gi_per_frame,
                       "parallelism": f"screen-tiles {T}px x{world_size}" if world_size > 1 else "single-gpu"},
            "rays_per_frame": rays_per_frame,
            # cone marches are reported separately
            "cone_steps_per_frame": st_all["cone_steps"],
            "cone_steps_per_s": round(st_all["cone_steps"] * fps, 1),
            "stage_ms": {"gi_update": round(gi_ms, 4), "prepass": round(pp_ms, 4), "render": round(render_ms, 4)},
            "frames_per_launch": {k: v for k, v in stage_fpl.items() if launches.get(k)},
            "kernel_ms": {k: round(v, 4) for k, v in avg_stage_ms.items()},   # per launch
            "path": args.path, "gi_async": bool(args.gi_async), "frames_in_flight": nfl,
            "pipelined": bool(piped),
            "flow": bool(flowed),
            # render waves of the flow launches that stopped waiting for their pre-pass tiles and evaluated
            # their half-res window themselves (rv_flow_info; 0 = every tile arrived through the hand-off)
            "flow_fallbacks": r.flow_info()[2] if flowed else None,
            "frame_group": ref_group,
            # both loop modes of the reference frame (value = the "is_value" one, the mode N = 1 runs)
            "modes": modes,
            "loop": "native" if native else "python",
            "gather": ("rccl" if native else args.dist_backend) if world_size > 1 else None,
            "root_weight": root_weight if world_size > 1 and native else None,
            "gather_check": gather_check,
            "roofline": roofline,
            "dropin": dropin,
            "cpu_baseline": cpu,
            "world_build_s": round(world_s, 3),
            "tex_table_bytes": int(r.tex_table_info()[1]),
            "stats": st_all,
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    r.close()
    if dist is not None:
        dist.destroy_process_group()


def spawn_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` without a launcher: N child processes of this script, one per GPU, with the
    environment torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR /
    MASTER_PORT on 127.0.0.1).  This parent never touches the GPU; it relays rank 0's stdout (the JSON
    line) and returns the first non-zero exit status (a failed rank ends the others)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for rk in range(n):
        env = dict(os.environ, RANK=str(rk), LOCAL_RANK=str(rk), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if rk == 0 else sys.stderr, start_new_session=True))
    out = procs[0].communicate()[0]
    rcs = [procs[0].returncode]
    for p in procs[1:]:
        try:
            rcs.append(p.wait(timeout=60 if rcs[0] == 0 else 10))
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            rcs.append(p.wait())
    for ln in out.decode(errors="replace").splitlines(keepends=True):   # the JSON line(s) to stdout, noise to stderr
        (sys.stdout if ln.startswith("{") else sys.stderr).write(ln)
    sys.stdout.flush()
    bad = [c for c in rcs if c != 0]
    if bad:
        log(f"bench.py: rank exit codes {rcs}")
    return bad[0] if bad else 0


def rehearse(args) -> int:
    """--rehearse: the multi-rank plumbing without a GPU -- a gloo process group over the ranks, the
    barrier-bracketed timed region (a host-side stand-in for the frames) and the max over ranks -- and
    rank 0's JSON line.  tests/test_bench_cli.py runs it on the CPU."""
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if ws > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.001 * (1 + rank))
    if ws > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "rehearsal (no GPU)", "value": None, "n_gpus": ws, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(el * 1000.0 / max(args.steps, 1), 4),
                          "rehearsal": True, "ranks_timed": ws}), flush=True)
    if ws > 1:
        dist.destroy_process_group()
    return 0


def dropin_leg(r, stream, cfg, flags, pos, yaw, pitch, pan, args, gi_stats, traffic_dir):
    """The drop-in leg: --warmup + --steps frames of renderLoop's calls (rv_update_gi_data, then
    rv_draw_cuda with ref_compat, one frame per call) on the bench's context, timed between two device
    synchronizes; then a timing pass of 10 frames (HIP events around each k_ref_flow launch on its stream)
    and the median cold latency of 9 renderLoop frames.  The roofline's algorithmic bytes are the flow
    launch's: the frame's render + pre-pass (census frames with the reference's minDist fetch, as
    rv_draw_cuda renders) + the GI window it computes ahead (the bench's GI census)."""
    import torch
    import rvgrt_amd as rv
    from rvgrt_amd.configs import camera_path

    W, H = cfg.width, cfg.height
    n = args.warmup + args.steps + 10 + 9
    path = camera_path((pos, yaw, pitch), W, H, n, pan=pan, ref_compat=True)
    dflags = flags | rv.RV_F_REF_FETCH
    r.set_stream(stream.cuda_stream)
    census = np.linspace(args.warmup, args.warmup + max(args.steps - 1, 0), 8).astype(int)
    r.stats_reset()
    for i in census:
        d = path[i]
        r.frame(d.cam, np.ctypeslib.as_array(d.vp), np.ctypeslib.as_array(d.prev_vp), time=d.time,
                jx=d.jitter_x, jy=d.jitter_y, flags=dflags | rv.RV_F_STATS)
    st = {name: {k: v / len(census) for k, v in r.stats(i).items()} for i, name in enumerate(rv._lib.STAGES)}
    rays = int(round(sum(v["traces"] for k, v in st.items() if k != "gi")))
    b = algorithmic_bytes(st["primary"], W * H, (W // 2) * (H // 2), True, "fused_render")
    b += algorithmic_bytes(st["pp_primary"], W * H, (W // 2) * (H // 2), True, "fused_prepass")
    if gi_stats is not None:
        b += (4 * gi_stats["dda_steps"] + gi_stats["sphere_steps"] + gi_stats["csdf_checks"]
              + 20 * gi_stats["tex_samples"] + 8 * min(262144, (cfg.n // 4) ** 3))
    cur = [0]

    def frame():
        d = path[cur[0]]
        cur[0] += 1
        r.update_gi_data()
        c = d.cam
        r.draw_cuda(c.pos[:], c.forward[:], c.up[:], c.right[:], np.ctypeslib.as_array(d.vp),
                    np.ctypeslib.as_array(d.prev_vp), jitter_x=0.0, jitter_y=d.time)

    _, fb0 = r.flow_info()[1:]
    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    r.timing_enable(22)
    for _ in range(10):
        frame()
    torch.cuda.synchronize()
    per_stage_ms, _ = r.timing_stages()
    launches = r.timing_launches()
    r.timing_enable(0)
    lat = []
    for _ in range(9):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        frame()
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t1) * 1000.0)
    active, nflow, fb = r.flow_info()
    launch_ms = per_stage_ms["primary"] / launches["primary"] if launches["primary"] else 0.0
    achieved = b / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    traffic, limit = None, None
    tpath = os.path.join(traffic_dir, "profiles", f"traffic_{cfg.name}" + ("" if args.pose == "P0" else f"_{args.pose}")
                         + "_drawcuda.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            tj["_path"] = tpath
            if tj.get("kernel", "").startswith("k_ref_flow"):
                traffic = tj.get("hbm_bytes_per_launch")
                limit = binding_limit(tj, launch_ms)
        except Exception:
            traffic = None
    ms = elapsed * 1000.0 / args.steps
    return {"loop": "renderLoop calls: rv_update_gi_data + rv_draw_cuda (ref_compat), one frame per call",
            "ms_per_step": round(ms, 4), "fps": round(1000.0 / ms, 2), "steps": args.steps, "warmup": args.warmup,
            "mrays_per_s": round(rays * 1000.0 / ms / 1e6, 2), "rays_per_frame": rays,
            "latency_ms": round(float(np.median(lat)), 4),
            "latency_mode": "cold renderLoop frame: UpdateGIData + drawCUDA of one frame from an idle device",
            "flow_active": bool(active), "flow_fallbacks": fb - fb0,
            "roofline": {"bound": "hbm", "limit": limit, "kernel": "k_ref_flow", "achieved": round(achieved, 2),
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": int(b),
                         "avg_launch_ms": round(launch_ms, 4), "frames_per_launch": 1,
                         "traffic_frac": (round(traffic / (launch_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)
                                          if traffic and launch_ms > 0 else None)}}


def host_cores():
    """(nproc, cgroup CPU quota in whole cores or None): nproc is what `nproc` prints (the affinity mask)."""
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return nproc, quota


def cpu_baseline(r, cfg, d, flags, atlas, budget_s, args_cpu_threads=0):
    """The CPU oracle (scalar DDA restatement, oracle/rv_oracle.c) on the host
    cores: same world (exported from the GPU; bit-identical to the oracle's
    own build, tests/test_gpu_parity.py), same camera and features, the frame
    render only (as rays_per_frame counts it).  Bounded sample:
    frames of <= 1080p are rendered whole, row band by row band in a spread
    order, until the budget is spent; 4K frames take the stride-16 row subset
    (rows y = 0 mod 16, i.e. 1/16 of the frame) in spread chunks.  The rate is
    traces / wall time, so a partial sample extrapolates by ray count."""
    import rvgrt_amd as rv
    from oracle import oracle as O

    nproc, quota = host_cores()
    # all the host cores this process may use: nproc (its CPU affinity), bounded by a cgroup CPU quota when
    # one is set (a GPU box's share of a larger machine); --cpu-threads overrides
    threads = args_cpu_threads or (min(nproc, quota) if quota else nproc)
    O.set_threads(threads)
    w = O.OracleWorld(cfg.log2_n, cfg.log2_n, cfg.log2_n, atlas=atlas)
    w.bits[:] = r.world_export(rv.RV_WORLD_BITS)
    w.csdf[:] = r.world_export(rv.RV_WORLD_CSDF)
    w.gi[:] = r.world_export(rv.RV_WORLD_GI)
    fr = O.make_frame(cfg.width, cfg.height, flags, rv.camera_dict(d.cam, np.ctypeslib.as_array(d.vp)), time=d.time,
                      jx=d.jitter_x, jy=d.jitter_y, pvp=np.ctypeslib.as_array(d.prev_vp))
    H = cfg.height
    stride = 16 if cfg.width * cfg.height > 1920 * 1080 else 1
    rows_all = np.arange(0, H, stride, dtype=np.int32)
    chunk = max(4 * threads, 32)
    chunks = [rows_all[i:i + chunk] for i in range(0, len(rows_all), chunk)]
    order = [c for k in range(4) for c in chunks[k::4]]        # spread over the image
    out = None

    def run(budget):
        nonlocal out
        t0 = time.perf_counter()
        rays = rows = 0
        while True:
            for c in order:
                out = O.render_rows(w, fr, c, out=out)
                rays += out["stats"]["traces"]
                rows += len(c)
                if time.perf_counter() - t0 >= budget:
                    return rays, rows, time.perf_counter() - t0

    rays, rows, dt = run(budget_s)
    O.set_threads(1)                           # the 1-core figure, ~1/4 of the budget
    rays1, _, dt1 = run(budget_s / 4)
    O.set_threads(threads)
    what = (f"stride-{stride} row subset ({len(rows_all)} of {H} rows)" if stride > 1 else "whole frames")
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "nproc": nproc, "cgroup_cpu_quota": quota,
            "value_1core": round(rays1 / dt1 / 1e6, 3),
            "sample": f"oracle/rv_oracle.c render of {what} of {cfg.name}: {rows} rows ({rows / H:.2f} frame "
                      f"heights) in {chunk}-row chunks on {threads} threads, {dt:.1f} s wall, {rays} traces, "
                      "same world/camera/flags; Mrays/s = traces / wall time"}


if __name__ == "__main__":
    sys.exit(main() or 0)
