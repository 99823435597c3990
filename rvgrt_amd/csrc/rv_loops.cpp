// rv_loops.cpp -- host side of librvgrt_hip.so, part 2 of the C ABI (include/rvgrt.h): the native frame
// loops (rv_render_frame_seq / rv_render_frames: batched, pipelined and grouped reference frames) and the
// screen-tile shard (rv_set_tile_shard*, the rank agreement check).  Context and helpers: rv_host.h.
#include "rv_host.h"

// Buffers of a batch set for B frames (images, half-res images, packed tiles
// of `slice` bytes per frame, rank 0's gather buffer of `gneed` bytes).
static rv_status bset_alloc(rv_ctx* c, BatchSet& b, int B, size_t slice, size_t gneed) {
    if (b.nb == B && b.slice == slice && b.gbytes == gneed) return RV_OK;
    const int H = c->cfg.height, W = c->cfg.width;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    HIP_TRY(c, hipDeviceSynchronize());
    hipFree(b.color); hipFree(b.mv); hipFree(b.depth); hipFree(b.hdist); hipFree(b.hshadow);
    hipFree(b.tbuf); hipFree(b.gbuf);
    b.color = nullptr; b.mv = nullptr; b.depth = nullptr; b.hdist = b.hshadow = nullptr;
    b.tbuf = b.gbuf = nullptr; b.nb = 0; b.pending = false;
    HIP_TRY(c, hipMalloc(&b.color, c->own_color_pitch * H * B));
    HIP_TRY(c, hipMalloc(&b.mv, c->own_mv_pitch * H * B));
    HIP_TRY(c, hipMalloc(&b.depth, c->own_depth_pitch * H * B));
    HIP_TRY(c, hipMalloc(&b.hdist, hbytes * B));
    HIP_TRY(c, hipMalloc(&b.hshadow, hbytes * B));
    if (slice) HIP_TRY(c, hipMalloc(&b.tbuf, slice * B));
    if (gneed) HIP_TRY(c, hipMalloc(&b.gbuf, gneed));
    if (!b.rendered) HIP_TRY(c, hipEventCreateWithFlags(&b.rendered, hipEventDisableTiming));
    if (!b.gathered) HIP_TRY(c, hipEventCreateWithFlags(&b.gathered, hipEventDisableTiming));
    b.nb = B; b.slice = slice; b.gbytes = gneed;
    return RV_OK;
}

// Copies frame `li` of a batch set into the active slot's images (the
// context's current output, what rv_readback returns).
static rv_status bset_publish(rv_ctx* c, const BatchSet& lb, size_t li, bool all, hipStream_t st) {
    const int W = c->cfg.width, H = c->cfg.height;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    const size_t cstride = c->own_color_pitch * H, mstride = c->own_mv_pitch * H, dstride = c->own_depth_pitch * H;
    HIP_TRY(c, hipMemcpy2DAsync(c->color, c->color_pitch, reinterpret_cast<const char*>(lb.color) + li * cstride,
                                c->own_color_pitch, (size_t)W * 4, H, hipMemcpyDeviceToDevice, st));
    if (!all) return RV_OK;
    HIP_TRY(c, hipMemcpy2DAsync(c->mv, c->mv_pitch, reinterpret_cast<const char*>(lb.mv) + li * mstride,
                                c->own_mv_pitch, (size_t)W * 4, H, hipMemcpyDeviceToDevice, st));
    HIP_TRY(c, hipMemcpy2DAsync(c->depth, c->depth_pitch, reinterpret_cast<const char*>(lb.depth) + li * dstride,
                                c->own_depth_pitch, (size_t)W * 2, H, hipMemcpyDeviceToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(c->hdist, reinterpret_cast<const char*>(lb.hdist) + li * hbytes, hbytes,
                              hipMemcpyDeviceToDevice, st));
    HIP_TRY(c, hipMemcpyAsync(c->hshadow, reinterpret_cast<const char*>(lb.hshadow) + li * hbytes, hbytes,
                              hipMemcpyDeviceToDevice, st));
    return RV_OK;
}

// Frames with a per-frame GI update and the pre-pass (the reference frame,
// C3-C5): the pre-pass reads only the static world, so it runs batched over
// a group of B frames (one launch, frame index in the grid); then frame by
// frame the GI update (kernel overlapping the previous render on the GI
// stream) and the render, which reads its frame's half-res images.
static rv_status render_gi_groups(rv_ctx* c, const Seq& q, int32_t flags, hipStream_t S) {
    const int frames = q.n;
    const int B = (int)c->slots.size();
    const int W = c->cfg.width, H = c->cfg.height;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    const size_t cstride = c->own_color_pitch * H, mstride = c->own_mv_pitch * H, dstride = c->own_depth_pitch * H;
    BatchSet& bs = c->bsets[0];
    if (rv_status as = bset_alloc(c, bs, B, bs.slice, bs.gbytes)) return as;
    slot_save(c);
    slot_load(c, 0);
    c->stream = S;
    if (rv_status ws = wait_all_frames(c)) return ws;   // frames of earlier calls, the last world write
    const FrameCam* cams = nullptr;
    if (!q.uniform(0, frames))
        if (rv_status us = upload_cams(c, q, S, &cams)) return us;
    int done = 0, last = 0;
    while (done < frames) {
        const int nb = std::min(B, frames - done);
        FrameParams f = make_params_d(c, q.at(done), flags);
        f.nbatch = (uint32_t)nb;
        if (cams) f.cams = cams + done;
        f.hdist = bs.hdist; f.hshadow = bs.hshadow; f.bs_half = hbytes;
        if (rv_status rs = run_stages(c, f, false, 1)) return rs;
        for (int j = 0; j < nb; j++) {
            if (rv_status gs = rv_update_gi_data(c)) return gs;
            FrameParams g = make_params_d(c, q.at(done + j), flags);
            g.hdist = reinterpret_cast<float*>(reinterpret_cast<char*>(bs.hdist) + (size_t)j * hbytes);
            g.hshadow = reinterpret_cast<float*>(reinterpret_cast<char*>(bs.hshadow) + (size_t)j * hbytes);
            g.color = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(bs.color) + (size_t)j * cstride);
            g.mv = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(bs.mv) + (size_t)j * mstride);
            g.depth = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(bs.depth) + (size_t)j * dstride);
            g.color_pitch = c->own_color_pitch; g.mv_pitch = c->own_mv_pitch; g.depth_pitch = c->own_depth_pitch;
            if (rv_status rs = run_stages(c, g, false, 2)) return rs;
            c->frame_seq++;
            last = j;
        }
        done += nb;
    }
    if (rv_status ps = bset_publish(c, bs, (size_t)last, true, S)) return ps;
    FrameSlot& s0 = c->slots[0];
    HIP_TRY(c, hipEventRecord(s0.done, S));
    s0.pending = true;
    s0.last_stream = S;
    return RV_OK;
}

// Pipelined reference frames (rv_set_pipeline; rvgrt.h).  On stream S:
//   prologue  GI update of frame 0 (kernel + copy-back), pre-pass of frame 0;
//   launch k  render k | GI update k+1 (grid k -> scratch) | pre-pass k+1,
//             one k_ref_pipe grid (the last launch renders only);
//   then      copy-back of update k+1's cells: in stream order after render
//             k, the last reader of grid k, and before render k+1.
// The half-res images alternate between two pairs (frame k & 1).
// With a tile shard and a communicator of N ranks, the launch renders
// this rank's tiles, the pre-pass covers their footprints, and the GI part
// computes this rank's 1/N of the update's cells; an RCCL all-gather of the
// cells (1 MiB per frame at RAYPS) on the comm stream precedes the copy-back,
// then the packed tiles of frame k go to rank 0 on the same stream while
// frame k+1 renders; rank 0 assembles frame k after launching frame k+1.
// Without a communicator an N > 1 shard renders its share only (its GI part
// covers the whole window, so its grid stays the reference's).
constexpr uint32_t PIPE_WSTAT_N = 32, PIPE_WSTAT_MAXB = 1u << 18;   // launches, workgroups per launch

// What a kept pre-pass was computed for: the camera fields the pre-pass
// reads, the pre-pass flag and the tile shard (its footprints).
static void pp_key(const rv_ctx* c, const rv_frame_desc& d, int32_t flags, float (&k)[24]) {
    std::memset(k, 0, sizeof(k));
    for (int i = 0; i < 3; i++) {
        k[i] = d.cam.pos[i]; k[3 + i] = d.cam.forward[i]; k[6 + i] = d.cam.right[i]; k[9 + i] = d.cam.up[i];
    }
    k[12] = d.jitter_x; k[13] = d.jitter_y;
    uint32_t h = 2166136261u;   // FNV-1a of the shard's tile ids
    for (int32_t t : c->shard_ids) h = (h ^ (uint32_t)t) * 16777619u;
    const int32_t iv[6] = {flags & RV_F_PREPASS, c->shard_n, c->shard_rank, c->shard_px, (int32_t)h, 0};
    std::memcpy(&k[14], iv, sizeof(iv));
}

static rv_status render_gi_pipe(rv_ctx* c, const Seq& q, int32_t flags, hipStream_t S, rv_comm* comm) {
    const int frames = q.n;
    const int W = c->cfg.width, H = c->cfg.height;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    const bool tiles = c->shard_n > 0, root = c->shard_rank == 0;
    const int N = tiles ? c->shard_n : 1, R = tiles ? c->shard_rank : 0, T = c->shard_px;
    const bool xchg = tiles && comm;   // GI shard + all-gather, tile gather to rank 0 (also for one rank)
    // timing probe (RV_OPT_GI_SHARD_PROBE, no communicator): this rank's GI share only, no exchange --
    // the grid is then NOT the reference's; only for sizing the multi-GPU loop on one GPU
    const bool probe = tiles && !comm && N > 1 && c->gi_shard_probe;
    const bool shard_gi = xchg || probe;
    const int bpp = c->gather_bpp;
    const size_t slice = tiles ? (size_t)c->shard_max * T * T * bpp : 0;
    const uint64_t n = n_gi(c), rays = c->cfg.gi_rays_per_frame;
    const uint64_t chunk = shard_gi ? (rays + N - 1) / N : 0;   // GI cells per rank (all-gather unit)
    for (auto& ph : c->pipe_half)
        for (int q2 = 0; q2 < 2; q2++)
            if (!ph[q2]) HIP_TRY(c, hipMalloc(&ph[q2], hbytes));
    if (!c->gi_tmp) HIP_TRY(c, hipMalloc(&c->gi_tmp, c->gi_bytes));
    if (tiles && (c->pipe_slice != slice || c->pipe_gbytes != (root ? slice * N : 0))) {
        HIP_TRY(c, hipDeviceSynchronize());
        for (int b = 0; b < 2; b++) {
            hipFree(c->pipe_tbuf[b]); hipFree(c->pipe_gbuf[b]);
            c->pipe_tbuf[b] = nullptr; c->pipe_gbuf[b] = nullptr;
            HIP_TRY(c, hipMalloc(&c->pipe_tbuf[b], slice ? slice : 1));
            if (root) HIP_TRY(c, hipMalloc(&c->pipe_gbuf[b], slice * N));
        }
        c->pipe_slice = slice; c->pipe_gbytes = root ? slice * N : 0;
    }
    if (shard_gi && (c->pipe_chunk != chunk || c->pipe_chunk_n != N)) {
        HIP_TRY(c, hipDeviceSynchronize());
        hipFree(c->pipe_gi_stage); hipFree(c->pipe_gi_all);
        c->pipe_gi_stage = nullptr; c->pipe_gi_all = nullptr;
        c->carry_gi = false;   // the kept shard lived in the old stage buffer
        HIP_TRY(c, hipMalloc(&c->pipe_gi_stage, chunk * 4));
        HIP_TRY(c, hipMalloc(&c->pipe_gi_all, chunk * N * 4));
        c->pipe_chunk = chunk; c->pipe_chunk_n = N;
    }
    for (hipEvent_t& e : c->pipe_ev)
        if (!e) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    slot_save(c);
    slot_load(c, 0);
    c->stream = S;
    if (rv_status ws = wait_all_frames(c)) return ws;   // frames of earlier calls, the last world write
    if (xchg) {   // the comm stream starts after the frames of earlier calls too
        HIP_TRY(c, hipEventRecord(c->pipe_ev[0], S));
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->pipe_ev[0], 0));
    }
    if (tiles) {
        if (rv_status us = upload_ids(c, c->untile_ids, c->shard_all.data(), (int)c->shard_all.size(), nullptr)) return us;
        if (rv_status ts = tile_list(c, c->shard_ids.data(), (int32_t)c->shard_ids.size(), T)) return ts;
    }
    auto peek_range = [&](uint32_t& fr, uint64_t& first, uint64_t& count) {   // rv_update_gi_data's next window
        fr = c->gi_frame;
        first = c->gi_offset;
        count = first + rays > n ? n - first : rays;
    };
    auto next_range = [&](uint32_t& fr, uint64_t& first, uint64_t& count) {   // ... and advance to the one after
        peek_range(fr, first, count);
        c->gi_frame++;
        if (c->gi_offset + rays >= n) c->gi_offset = 0;   // src/CoarseArray.cu:392-394
        else c->gi_offset += rays;
    };
    // work the previous call's last launch did for this call's first frame
    float key0[24];
    pp_key(c, q.at(0), flags, key0);
    uint32_t fr = 0;
    uint64_t first = 0, count = 0;
    peek_range(fr, first, count);
    const bool use_gi = c->pipe_carry && c->carry_gi && c->carry_world == c->world_ver &&
                        c->carry_n == (shard_gi ? N : 0) && c->carry_r == (shard_gi ? R : 0) &&
                        c->carry_chunk == chunk && c->carry_fr == fr && c->carry_first == first &&
                        c->carry_count == count;
    const bool use_pp = c->pipe_carry && c->carry_pp && c->carry_geom == c->geom_ver &&
                        std::memcmp(c->carry_key, key0, sizeof(key0)) == 0;
    const int base = use_pp ? c->carry_half : 0;   // frame k's half-res images: pipe_half[(base + k) & 1]
    c->carry_gi = c->carry_pp = false;
    auto half = [&](int k) { return (base + k) & 1; };
    auto tile_params = [&](FrameParams& f, int k) {
        if (!tiles) return;
        f.tiles = c->tiles.d; f.ntiles = (int)c->shard_ids.size(); f.tile_px = T; f.tiles_x = (W + T - 1) / T;
        f.tilebuf = c->pipe_tbuf[k & 1]; f.tile_bpp = bpp;
        f.chunk_order[CG_RENDER] = c->tile_order; f.chunk_cost[CG_RENDER] = c->tile_cost;
    };
    const World w = current_world(c);
    unsigned long long* cnt_gi = c->counters + (size_t)ST_GI * NCNT;
    next_range(fr, first, count);   // frame 0's update: every rank the whole window (identical grids) ...
    if (!use_gi) {
        launch_gi_update(S, c->gi, c->gi_tmp, w, sun_dir(), fr, first, count, cnt_gi, c->gi_stats);
        LAUNCH_CHECK(c);
        launch_copy_u32(S, c->gi + first, c->gi_tmp + first, count);
        LAUNCH_CHECK(c);
    } else if (xchg) {   // ... or kept from the previous call: this rank's share, exchanged now
        if (rv_status as = comm_all_gather(c, comm, c->pipe_gi_stage, c->pipe_gi_all, chunk * 4, c->comm_stream))
            return as;
        HIP_TRY(c, hipEventRecord(c->pipe_ev[1], c->comm_stream));
        HIP_TRY(c, hipStreamWaitEvent(S, c->pipe_ev[1], 0));
        launch_copy_u32(S, c->gi + first, c->pipe_gi_all, count);
        LAUNCH_CHECK(c);
    } else if (!probe) {
        launch_copy_u32(S, c->gi + first, c->gi_tmp + first, count);
        LAUNCH_CHECK(c);
    }
    if (!use_pp) {
        FrameParams f = make_params_d(c, q.at(0), flags);
        f.hdist = c->pipe_half[half(0)][0]; f.hshadow = c->pipe_half[half(0)][1];
        f.counters = c->counters + (size_t)ST_PP_PRIMARY * NCNT;
        tile_params(f, 0);
        if (tiles) launch_prepass_tiles(S, w, f); else launch_prepass(S, w, f);
        LAUNCH_CHECK(c);
    }
    const int tiles_x = (W + T - 1) / std::max(T, 1);
    auto untile = [&](int k) -> rv_status {   // rank 0: assemble frame k once its gather is done
        HIP_TRY(c, hipStreamWaitEvent(S, c->pipe_ev[2 + (k & 1)], 0));
        launch_untile(S, c->pipe_gbuf[k & 1], c->untile_ids.d, (int)c->shard_all.size(), T, tiles_x, W, H, c->color,
                      c->color_pitch, c->shard_max, 1, 0, bpp);
        LAUNCH_CHECK(c);
        return RV_OK;
    };
    for (int k = 0; k < frames; k++) {
        const bool last = k + 1 == frames;
        // every launch also runs the next frame's update and pre-pass; the last launch's are kept for the
        // next call (RV_PIPE_CARRY=0: the last launch renders only)
        const bool more = !last || c->pipe_carry;
        FrameParams f = make_params_d(c, q.at(k), flags);
        f.hdist = c->pipe_half[half(k)][0]; f.hshadow = c->pipe_half[half(k)][1];
        f.counters = c->counters + (size_t)ST_PRIMARY * NCNT;
        tile_params(f, k);
        if (xchg && k >= 2)   // tile buffer k & 1 is free once frame k-2's gather has read it
            HIP_TRY(c, hipStreamWaitEvent(S, c->pipe_ev[2 + (k & 1)], 0));
        PipeParams p{};
        p.gi_prev = c->gi;
        uint64_t mine = 0, mfirst = 0;
        if (more) {
            if (last) peek_range(p.gi_frame, first, count);
            else next_range(p.gi_frame, first, count);
            mfirst = first; mine = count;
            if (shard_gi) {
                mfirst = first + std::min<uint64_t>(count, (uint64_t)R * chunk);
                mine = std::min<uint64_t>(chunk, first + count - mfirst);
            }
            const rv_frame_desc& nd = last ? q.after() : q.at(k + 1);
            p.pp_pos = host_v(nd.cam.pos[0], nd.cam.pos[1], nd.cam.pos[2]);
            p.pp_fo = host_v(nd.cam.forward[0], nd.cam.forward[1], nd.cam.forward[2]);
            p.pp_ri = host_v(nd.cam.right[0], nd.cam.right[1], nd.cam.right[2]);
            p.pp_up = host_v(nd.cam.up[0], nd.cam.up[1], nd.cam.up[2]);
            p.pp_jx = nd.jitter_x; p.pp_jy = nd.jitter_y;
        }
        p.gi_first = mfirst; p.gi_count = mine;
        p.gi_next = shard_gi ? c->pipe_gi_stage : c->gi_tmp + first;
        p.pp_hdist = c->pipe_half[half(k + 1)][0]; p.pp_hshadow = c->pipe_half[half(k + 1)][1];
        p.pp_counters = c->counters + (size_t)ST_PP_PRIMARY * NCNT;
        p.gi_counters = cnt_gi;
        // latency-variant launches (a rank's share from 4 ranks, C3) run the GI cells on lane pairs
        const uint32_t rlen = pipe_len(f, PIPE_RENDER, 0);
        p.gi_pairs = (c->gi_pairs > 0 || (c->gi_pairs < 0 && tiles)) && pipe_latency_variant(f, rlen) ? 1u : 0u;
        const uint32_t lens[3] = {more ? pipe_len(f, PIPE_GI, p.gi_pairs ? 2 * mine : mine) : 0u,
                                  more ? pipe_len(f, PIPE_PP, 0) : 0u, rlen};
        for (int i = 0; i < 3; i++) {
            p.part[i] = (c->pipe_order >> (4 * (2 - i))) & 0xFu;
            p.len[i] = lens[p.part[i]];
        }
        if (RV_PIPE_DIAG && getenv("RV_PIPE_WAVE_STATS") && more) {   // diagnostics: summarised by rv_destroy
            const uint32_t nb = p.len[0] + p.len[1] + p.len[2];
            if (!c->pipe_wstat) HIP_TRY(c, hipMalloc(&c->pipe_wstat, (size_t)PIPE_WSTAT_N * PIPE_WSTAT_MAXB * 4));
            if (c->pipe_launches < PIPE_WSTAT_N && nb <= PIPE_WSTAT_MAXB) {
                p.wave_max = c->pipe_wstat + (size_t)c->pipe_launches * PIPE_WSTAT_MAXB;
                HIP_TRY(c, hipMemsetAsync(p.wave_max, 0xFF, (size_t)nb * 4, S));
                c->pipe_wnb[c->pipe_launches++] = nb;
            }
        }
        // timing (rv_timing_stages: stage ST_PRIMARY) records the full launches
        const bool timed = (more || frames == 1) && c->timing_n < c->timing_cap;
        const size_t e0 = (size_t)EV_PER_FRAME * c->timing_n;
        if (timed) { c->ev_stage[e0] = ST_PRIMARY; HIP_TRY(c, hipEventRecord(c->ev[e0], S)); }
        launch_ref_pipe(S, w, f, p);
        LAUNCH_CHECK(c);
        if (timed) {
            c->ev_stage[e0 + 1] = -1;
            HIP_TRY(c, hipEventRecord(c->ev[e0 + 1], S));
            c->ev_used[c->timing_n] = 2;
            c->timing_n++;
        }
        const bool apply = more && !last;   // this launch's update is frame k+1's: apply it now
        if (xchg) {
            HIP_TRY(c, hipEventRecord(c->pipe_ev[0], S));   // frame k rendered, shard k+1 computed
            HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->pipe_ev[0], 0));
            if (apply) {   // the update's cells from every rank, then the copy-back on S
                if (rv_status as = comm_all_gather(c, comm, c->pipe_gi_stage, c->pipe_gi_all, chunk * 4,
                                                   c->comm_stream))
                    return as;
                HIP_TRY(c, hipEventRecord(c->pipe_ev[1], c->comm_stream));
                HIP_TRY(c, hipStreamWaitEvent(S, c->pipe_ev[1], 0));
                launch_copy_u32(S, c->gi + first, c->pipe_gi_all, count);
        LAUNCH_CHECK(c);
            }
            // frame k's packed tiles to rank 0, after the all-gather on the comm stream
            if (root)
                HIP_TRY(c, hipMemcpyAsync(c->pipe_gbuf[k & 1], c->pipe_tbuf[k & 1], slice, hipMemcpyDeviceToDevice,
                                          c->comm_stream));
            if (rv_status gs = comm_group_start(c, comm)) return gs;
            if (root) {
                for (int r = 1; r < N; r++)
                    if (rv_status rs = comm_recv(c, comm, reinterpret_cast<char*>(c->pipe_gbuf[k & 1]) + (size_t)r * slice,
                                                 slice, r, c->comm_stream))
                        return rs;
            } else {
                if (rv_status ss = comm_send(c, comm, c->pipe_tbuf[k & 1], slice, 0, c->comm_stream)) return ss;
            }
            if (rv_status ge = comm_group_end(c, comm, c->comm_stream)) return ge;
            HIP_TRY(c, hipEventRecord(c->pipe_ev[2 + (k & 1)], c->comm_stream));
            if (root && k >= 1)   // frame k-1, whose gather overlapped this launch
                if (rv_status us = untile(k - 1)) return us;
        } else {
            if (apply && !probe)
                launch_copy_u32(S, c->gi + first, c->gi_tmp + first, count);
        LAUNCH_CHECK(c);
            if (tiles && N == 1) {   // one rank: assemble locally
                launch_untile(S, c->pipe_tbuf[k & 1], c->untile_ids.d, (int)c->shard_all.size(), T, tiles_x, W, H,
                              c->color, c->color_pitch, c->shard_max, 1, 0, bpp);
                LAUNCH_CHECK(c);
            }
        }
        if (last && more) {   // keep the next frame's update and pre-pass for the next call
            c->carry_gi = true;
            c->carry_fr = p.gi_frame; c->carry_first = first; c->carry_count = count;
            c->carry_n = shard_gi ? N : 0; c->carry_r = shard_gi ? R : 0; c->carry_chunk = chunk;
            c->carry_pp = true;
            c->carry_half = half(k + 1);
            c->carry_geom = c->geom_ver;
            pp_key(c, q.after(), flags, c->carry_key);
        }
        if (f.sched == SCHED_COST && ++c->frames_since_order >= (uint32_t)c->order_every) {
            c->frames_since_order = 0;
            if (tiles) {
                launch_chunk_order(S, c->tile_cost, c->tile_order, (uint32_t)f.ntiles, ((uint32_t)f.ntiles + 7u) & ~7u);
            } else {
                launch_chunk_order(S, c->chunk_cost[CG_PREPASS], c->chunk_order[CG_PREPASS], n_chunks(f.hw, f.hh),
                                   n_chunks_pad(f.hw, f.hh), c->chunk_cost[CG_RENDER],
                                   c->chunk_order[CG_RENDER], n_chunks(f.W, f.H), n_chunks_pad(f.W, f.H));
            }
            LAUNCH_CHECK(c);
        }
        c->frame_seq++;
    }
    if (xchg) {
        if (root)
            if (rv_status us = untile(frames - 1)) return us;
        HIP_TRY(c, hipEventRecord(c->pipe_ev[0], c->comm_stream));   // S sees the last gather done
        HIP_TRY(c, hipStreamWaitEvent(S, c->pipe_ev[0], 0));
    }
    // the last frame's half-res images become the slot's (rv_readback)
    const int lk = half(frames - 1);
    HIP_TRY(c, hipMemcpyAsync(c->hdist, c->pipe_half[lk][0], hbytes, hipMemcpyDeviceToDevice, S));
    HIP_TRY(c, hipMemcpyAsync(c->hshadow, c->pipe_half[lk][1], hbytes, hipMemcpyDeviceToDevice, S));
    if (rv_status ms = mark_world(c)) return ms;
    c->carry_world = c->world_ver;   // the kept update is valid until the next world/GI write
    FrameSlot& s0 = c->slots[0];
    HIP_TRY(c, hipEventRecord(s0.done, S));
    s0.pending = true;
    s0.last_stream = S;
    return RV_OK;
}

// Grouped reference frames (rv_set_frame_group; rvgrt.h).  Frames of the call in
// groups of F; group g = frames [gF, gF + n_g).  On stream S:
//   prologue  launch: pre-pass of group 0, phase A of groups 0 and 1; phase B of group 0
//   launch g  render g (overlay: group g's updates) | pre-pass g+1 | phase A of group g+2
//   then      apply(g): group g's updates from the ring into the grid (after render g, its last
//             reader of the old cells; before render g+1)
// Side stream SB: phase B of group g+2 once apply(g) and its records exist (the all-gather with a
// communicator): it overlaps launch g+1; launch g+2 waits for it.  The ring holds the updates of
// two consecutive groups at positions P (cumulative cell count, wrapping), so phase B of group h
// reads grid h-1's cells through one overlay of origin (s_{h-1}, P_{h-1}), and every other cell
// from the grid (complete through group h-2).  With a tile shard and a communicator the phase A
// cells of every update are split over the ranks (rank r: the r-th chunk of each window) and the
// records of a group all-gathered once; the packed tiles of group g go to rank 0 after launch g.
static int group_frames(const rv_ctx* c) {
    const uint64_t n = n_gi(c), rays = std::min<uint64_t>(c->cfg.gi_rays_per_frame, n);
    int F = std::min(c->group, 32);
    while (F >= 2 && (uint64_t)F * rays * 2 > n) F--;   // two groups' updates never overlap in the grid
    return F >= 2 ? F : 0;
}

static rv_status render_gi_group(rv_ctx* c, const Seq& q, int32_t flags, hipStream_t S, rv_comm* comm, int F) {
    const int frames = q.n;
    const int W = c->cfg.width, H = c->cfg.height;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    const bool tiles = c->shard_n > 0, root = c->shard_rank == 0;
    const int N = tiles ? c->shard_n : 1, R = tiles ? c->shard_rank : 0, T = c->shard_px;
    const bool xchg = tiles && comm;
    const bool probe = tiles && !comm && N > 1 && c->gi_shard_probe;
    const bool shard_gi = xchg || probe;
    const int bpp = c->gather_bpp;
    const size_t slice = tiles ? (size_t)c->shard_max * T * T * bpp : 0;
    const uint64_t ngi = n_gi(c), rays = std::min<uint64_t>(c->cfg.gi_rays_per_frame, ngi);
    const uint64_t chunk = shard_gi ? (rays + N - 1) / N : rays;   // phase-A cells per rank and window
    const int Nrec = shard_gi ? N : 1;
    uint64_t cap = 1;
    while (cap < 2 * (uint64_t)F * rays) cap <<= 1;                  // the ring: two groups' updates
    const uint32_t gmask = (uint32_t)(ngi - 1), cmask = (uint32_t)(cap - 1);
    const int G = (frames + F - 1) / F;
    auto nfr = [&](int g) { return g < G ? std::min(F, frames - g * F) : 0; };
    // buffers
    const size_t gneed = tiles && root ? slice * (size_t)F * (size_t)N : 0;
    for (BatchSet& b : c->gsets)
        if (rv_status as = bset_alloc(c, b, F, tiles ? slice : 0, gneed)) return as;
    const size_t nstage = 3 * (size_t)F * chunk, nall = 3 * (size_t)Nrec * F * chunk;
    if (c->grec_stage_n < nstage || c->grec_all_n < nall || c->gring_n < cap) {
        HIP_TRY(c, hipDeviceSynchronize());
        hipFree(c->grec_stage); hipFree(c->grec_all); hipFree(c->gring);
        c->grec_stage = nullptr; c->grec_all = nullptr; c->gring = nullptr;
        c->grec_stage_n = c->grec_all_n = c->gring_n = 0;
        HIP_TRY(c, hipMalloc(&c->grec_stage, nstage * sizeof(uint2)));
        HIP_TRY(c, hipMalloc(&c->grec_all, nall * sizeof(uint2)));
        HIP_TRY(c, hipMalloc(&c->gring, cap * 4));
        c->grec_stage_n = nstage; c->grec_all_n = nall; c->gring_n = cap;
        // a record slot nobody wrote (other ranks' chunks under the timing probe) reads as a solid cell;
        // on S: a plain hipMemset runs on the legacy stream, which does not order with S
        HIP_TRY(c, hipMemsetAsync(c->grec_all, 0, nall * sizeof(uint2), S));
    }
    for (hipEvent_t& e : c->gev)
        if (!e) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipEvent_t& ev_rendered = c->gev[0];
    hipEvent_t& ev_applied = c->gev[1];
    hipEvent_t& ev_allg = c->gev[2];
    hipEvent_t* ev_pb = &c->gev[3];        // [2] phase B of group h done (slot h & 1)
    hipEvent_t* ev_gath = &c->gev[5];      // [2] tile gather of group g done (slot g & 1)
    hipEvent_t& ev_tmp = c->gev[7];
    if (!c->grp_stream) HIP_TRY(c, hipStreamCreateWithPriority(&c->grp_stream, hipStreamNonBlocking, c->prio_hi));
    hipStream_t SB = c->grp_stream;
    slot_save(c);
    slot_load(c, 0);
    c->stream = S;
    if (rv_status ws = wait_all_frames(c)) return ws;   // frames of earlier calls, the last world write
    c->carry_gi = c->carry_pp = false;                 // the per-frame pipeline's kept work is stale now
    HIP_TRY(c, hipEventRecord(ev_tmp, S));             // SB and the comm stream start after that too
    HIP_TRY(c, hipStreamWaitEvent(SB, ev_tmp, 0));
    if (xchg) HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, ev_tmp, 0));
    if (tiles) {
        if (rv_status us = upload_ids(c, c->untile_ids, c->shard_all.data(), (int)c->shard_all.size(), nullptr)) return us;
        if (rv_status ts = tile_list(c, c->shard_ids.data(), (int32_t)c->shard_ids.size(), T)) return ts;
    }
    // the GI window of every frame of the call (rv_update_gi_data's sequence) and its ring position
    std::vector<uint32_t> wfr((size_t)frames), wfirst((size_t)frames), wcount((size_t)frames), wpos((size_t)frames + 1);
    {
        uint64_t off = c->gi_offset, pos = 0;
        for (int k = 0; k < frames; k++) {
            wfr[(size_t)k] = c->gi_frame + (uint32_t)k;
            wfirst[(size_t)k] = (uint32_t)off;
            wcount[(size_t)k] = (uint32_t)(off + rays > ngi ? ngi - off : rays);
            wpos[(size_t)k] = (uint32_t)(pos & cmask);
            pos += wcount[(size_t)k];
            off = off + rays >= ngi ? 0 : off + rays;   // src/CoarseArray.cu:392-394
        }
        wpos[(size_t)frames] = (uint32_t)(pos & cmask);
    }
    auto gsum = [&](int g, int j) {   // cells of group g's updates before its j-th
        uint64_t t = 0;
        for (int k = g * F; k < g * F + j; k++) t += wcount[(size_t)k];
        return (uint32_t)t;
    };
    // phase A of frame k's update: this rank's cells of its window
    auto window_share = [&](int k, uint32_t& mfirst, uint32_t& mine) {
        mfirst = wfirst[(size_t)k]; mine = wcount[(size_t)k];
        if (shard_gi) {
            mfirst = wfirst[(size_t)k] + (uint32_t)std::min<uint64_t>(wcount[(size_t)k], (uint64_t)R * chunk);
            mine = (uint32_t)std::min<uint64_t>(chunk, (uint64_t)wfirst[(size_t)k] + wcount[(size_t)k] - mfirst);
        }
    };
    // the per-frame table the launches read: camera, this rank's phase A cells, overlay length
    const FrameCam* cams = nullptr;
    if (rv_status us = upload_cams(c, q, S, &cams, [&](int k, FrameCam& fc) {
            window_share(k, fc.gi_first, fc.gi_count);
            fc.gi_ovlen = gsum(k / F, k % F + 1);   // frame k sees its own update
        }))
        return us;
    const World w = current_world(c);
    const int tiles_x = (W + T - 1) / std::max(T, 1);
    const size_t cstride = c->own_color_pitch * H, mstride = c->own_mv_pitch * H, dstride = c->own_depth_pitch * H;

    // phase A of groups [h0, h1): their frames are consecutive, window j = frame h0 * F + j
    auto set_phase_a = [&](GroupParams& gp, int h0, int h1) {
        gp.nw = 0;
        for (int h = h0; h < h1; h++) gp.nw += (uint32_t)nfr(h);
        if (!gp.nw) return;
        gp.gk0 = (uint32_t)(h0 * F);
        gp.gfr0 = wfr[(size_t)h0 * F];
        gp.gcams = cams + (size_t)h0 * F;
    };
    auto launch_group = [&](int g, bool timed) -> rv_status {
        // render part: group g (none in the prologue, g = -1); pre-pass of group g+1; phase A: group g+2
        // (the prologue: groups 0 and 1)
        FrameParams f = make_params_d(c, q.at(std::max(g, 0) * F), flags);
        f.cams = cams + (size_t)std::max(g, 0) * F;
        const BatchSet& bs = c->gsets[std::max(g, 0) & 1];
        f.color = bs.color; f.mv = bs.mv; f.depth = bs.depth;
        f.color_pitch = c->own_color_pitch; f.mv_pitch = c->own_mv_pitch; f.depth_pitch = c->own_depth_pitch;
        f.bs_color = cstride; f.bs_mv = mstride; f.bs_depth = dstride;
        f.hdist = bs.hdist; f.hshadow = bs.hshadow; f.bs_half = hbytes;
        f.counters = c->counters + (size_t)ST_PRIMARY * NCNT;
        if (tiles) {
            f.tiles = c->tiles.d; f.ntiles = (int)c->shard_ids.size(); f.tile_px = T; f.tiles_x = tiles_x;
            f.tilebuf = bs.tbuf; f.tile_bpp = bpp; f.bs_tile = slice;
            f.chunk_order[CG_RENDER] = c->tile_order; f.chunk_cost[CG_RENDER] = c->tile_cost;
        }
        GroupParams gp{};
        gp.nr = g >= 0 ? (uint32_t)nfr(g) : 0u;
        f.nbatch = std::max(gp.nr, 1u);
        gp.rlen1 = pipe_len(f, PIPE_RENDER, 0);
        gp.ov = c->gring; gp.gmask = gmask; gp.cmask = cmask;
        if (g >= 0) { gp.ov_s = wfirst[(size_t)g * F]; gp.ov_p = wpos[(size_t)g * F]; }
        const int hp = g + 1;   // the pre-pass's group
        gp.np = (uint32_t)nfr(hp);
        gp.plen1 = pipe_len(f, PIPE_PP, 0);
        if (gp.np) {
            gp.pcams = cams + (size_t)hp * F;
            gp.pp_hdist = c->gsets[hp & 1].hdist; gp.pp_hshadow = c->gsets[hp & 1].hshadow; gp.pp_bs = hbytes;
        }
        gp.rec = xchg ? c->grec_stage : c->grec_all;
        gp.F = (uint32_t)F; gp.chunk = (uint32_t)chunk;
        gp.rslot = (uint32_t)(xchg ? (size_t)F * chunk : (size_t)Nrec * F * chunk);
        gp.glen1 = (uint32_t)(((chunk + 63) / 64 + 7) & ~7ull);
        if (g < 0) set_phase_a(gp, 0, 2); else set_phase_a(gp, g + 2, g + 3);
        gp.pp_counters = c->counters + (size_t)ST_PP_PRIMARY * NCNT;
        gp.gi_counters = c->counters + (size_t)ST_GI * NCNT;
        const uint32_t lens[3] = {gp.nw * gp.glen1, gp.np * gp.plen1, gp.nr * gp.rlen1};
        for (int i = 0; i < 3; i++) {
            gp.part[i] = (c->pipe_order >> (4 * (2 - i))) & 0xFu;
            gp.len[i] = lens[gp.part[i]];
        }
        const bool tm = timed && c->timing_n < c->timing_cap;
        const size_t e0 = (size_t)EV_PER_FRAME * c->timing_n;
        if (tm) { c->ev_stage[e0] = ST_PRIMARY; HIP_TRY(c, hipEventRecord(c->ev[e0], S)); }
        launch_ref_group(S, w, f, gp);
        LAUNCH_CHECK(c);
        if (tm) {
            c->ev_stage[e0 + 1] = -1;
            HIP_TRY(c, hipEventRecord(c->ev[e0 + 1], S));
            c->ev_used[c->timing_n] = 2;
            c->timing_n++;
        }
        return RV_OK;
    };
    // phase B of group h on stream st: window j reads grid (frame before it) through the overlay of
    // origin group o = max(h - 1, 0)
    auto phase_b = [&](int h, hipStream_t st) -> rv_status {
        const int o = std::max(h - 1, 0);
        WorldOv wo;
        static_cast<World&>(wo) = w;
        wo.ov = c->gring; wo.gmask = gmask; wo.cmask = cmask;
        wo.ov_s = wfirst[(size_t)o * F]; wo.ov_p = wpos[(size_t)o * F];
        const uint2* recs = c->grec_all + (size_t)(h % 3) * Nrec * F * chunk;
        for (int j = 0; j < nfr(h); j++) {
            const int k = h * F + j;
            wo.ov_len = (h > 0 ? gsum(o, nfr(o)) : 0u) + gsum(h, j);
            const uint32_t dpos = (wo.ov_p + ((wfirst[(size_t)k] - wo.ov_s) & gmask)) & cmask;
            launch_gi_phase_b(st, wo, recs, (uint32_t)chunk, (uint32_t)F, (uint32_t)j, wfirst[(size_t)k],
                              wcount[(size_t)k], c->gring, dpos);
            LAUNCH_CHECK(c);
        }
        return RV_OK;
    };
    auto allgather = [&](int h) -> rv_status {   // group h's records from every rank (comm stream)
        if (rv_status as = comm_all_gather(c, comm, c->grec_stage + (size_t)(h % 3) * F * chunk,
                                           c->grec_all + (size_t)(h % 3) * Nrec * F * chunk,
                                           (size_t)F * chunk * sizeof(uint2), c->comm_stream))
            return as;
        HIP_TRY(c, hipEventRecord(ev_allg, c->comm_stream));
        return RV_OK;
    };
    auto untile = [&](int g) -> rv_status {   // rank 0: assemble group g once its gather is done
        HIP_TRY(c, hipStreamWaitEvent(S, ev_gath[g & 1], 0));
        launch_untile(S, c->gsets[g & 1].gbuf, c->untile_ids.d, (int)c->shard_all.size(), T, tiles_x, W, H,
                      c->gsets[g & 1].color, c->own_color_pitch, c->shard_max, nfr(g), cstride, bpp);
        LAUNCH_CHECK(c);
        return RV_OK;
    };

    // ---- prologue
    if (rv_status ls = launch_group(-1, false)) return ls;
    HIP_TRY(c, hipEventRecord(ev_rendered, S));
    if (xchg) {
        HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, ev_rendered, 0));
        if (rv_status as = allgather(0)) return as;
        HIP_TRY(c, hipStreamWaitEvent(S, ev_allg, 0));
    }
    if (rv_status ps = phase_b(0, S)) return ps;
    if (G > 1) {
        HIP_TRY(c, hipEventRecord(ev_tmp, S));   // phase B of group 0 written (group 1 reads it)
        HIP_TRY(c, hipStreamWaitEvent(SB, ev_tmp, 0));
        if (xchg) {
            if (rv_status as = allgather(1)) return as;
            HIP_TRY(c, hipStreamWaitEvent(SB, ev_allg, 0));
        }
        if (rv_status ps = phase_b(1, SB)) return ps;
        HIP_TRY(c, hipEventRecord(ev_pb[1], SB));
    }
    // ---- groups
    for (int g = 0; g < G; g++) {
        if (g >= 1) HIP_TRY(c, hipStreamWaitEvent(S, ev_pb[g & 1], 0));
        if (xchg && g >= 2) HIP_TRY(c, hipStreamWaitEvent(S, ev_gath[g & 1], 0));   // tile buffers of group g-2 sent
        // timing (rv_timing_stages): the steady-state launches, whose three parts are all full
        if (rv_status ls = launch_group(g, nfr(g) == F && nfr(g + 1) == F && nfr(g + 2) == F)) return ls;
        HIP_TRY(c, hipEventRecord(ev_rendered, S));
        launch_gi_apply(S, c->gring, c->gi, wfirst[(size_t)g * F], wpos[(size_t)g * F], gsum(g, nfr(g)), gmask, cmask);
        LAUNCH_CHECK(c);
        HIP_TRY(c, hipEventRecord(ev_applied, S));
        FrameParams fo = make_params_d(c, q.at(g * F), flags);   // SCHED_COST re-order after every group
        if (fo.sched == SCHED_COST) {
            if (tiles) {
                const uint32_t nt = (uint32_t)c->shard_ids.size();
                launch_chunk_order(S, c->tile_cost, c->tile_order, nt, (nt + 7u) & ~7u);
            } else {
                launch_chunk_order(S, c->chunk_cost[CG_PREPASS], c->chunk_order[CG_PREPASS], n_chunks(fo.hw, fo.hh),
                                   n_chunks_pad(fo.hw, fo.hh), c->chunk_cost[CG_RENDER],
                                   c->chunk_order[CG_RENDER], n_chunks(W, H), n_chunks_pad(W, H));
            }
            LAUNCH_CHECK(c);
        }
        if (xchg) {
            HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, ev_rendered, 0));
            if (g + 2 < G)
                if (rv_status as = allgather(g + 2)) return as;
            // the group's packed tiles to rank 0
            const BatchSet& bs = c->gsets[g & 1];
            const size_t sb = slice * (size_t)nfr(g);
            if (root) HIP_TRY(c, hipMemcpyAsync(bs.gbuf, bs.tbuf, sb, hipMemcpyDeviceToDevice, c->comm_stream));
            if (rv_status gs = comm_group_start(c, comm)) return gs;
            if (root) {
                for (int r = 1; r < N; r++)
                    if (rv_status rs = comm_recv(c, comm, reinterpret_cast<char*>(bs.gbuf) + (size_t)r * sb, sb, r,
                                                 c->comm_stream))
                        return rs;
            } else {
                if (rv_status ss = comm_send(c, comm, bs.tbuf, sb, 0, c->comm_stream)) return ss;
            }
            if (rv_status ge = comm_group_end(c, comm, c->comm_stream)) return ge;
            HIP_TRY(c, hipEventRecord(ev_gath[g & 1], c->comm_stream));
        }
        if (g + 2 < G) {   // phase B of group g+2 overlaps launch g+1
            HIP_TRY(c, hipStreamWaitEvent(SB, ev_applied, 0));
            HIP_TRY(c, hipStreamWaitEvent(SB, xchg ? ev_allg : ev_rendered, 0));
            if (rv_status ps = phase_b(g + 2, SB)) return ps;
            HIP_TRY(c, hipEventRecord(ev_pb[g & 1], SB));
        }
        if (xchg && root && g >= 1)
            if (rv_status us = untile(g - 1)) return us;
        if (tiles && !xchg && N == 1) {   // one rank without a communicator: assemble locally
            launch_untile(S, c->gsets[g & 1].tbuf, c->untile_ids.d, (int)c->shard_all.size(), T, tiles_x, W, H,
                          c->gsets[g & 1].color, c->own_color_pitch, c->shard_max, nfr(g), cstride, bpp);
            LAUNCH_CHECK(c);
        }
        c->frame_seq += (uint64_t)nfr(g);
    }
    if (xchg) {
        if (root)
            if (rv_status us = untile(G - 1)) return us;
        HIP_TRY(c, hipEventRecord(ev_tmp, c->comm_stream));   // S sees the last gather done
        HIP_TRY(c, hipStreamWaitEvent(S, ev_tmp, 0));
    }
    // the GI counters advance by the frames rendered; the last frame becomes the slot's output
    c->gi_frame += (uint32_t)frames;
    c->gi_offset = frames > 0 ? (wfirst[(size_t)frames - 1] + rays >= ngi ? 0 : wfirst[(size_t)frames - 1] + rays)
                              : c->gi_offset;
    if (rv_status ps = bset_publish(c, c->gsets[(G - 1) & 1], (size_t)nfr(G - 1) - 1, true, S)) return ps;
    if (rv_status ms = mark_world(c)) return ms;
    FrameSlot& s0 = c->slots[0];
    HIP_TRY(c, hipEventRecord(s0.done, S));
    s0.pending = true;
    s0.last_stream = S;
    return RV_OK;
}

extern "C" rv_status rv_get_frame_group(rv_ctx* c, int32_t* effective) {
    if (!c || !effective) return RV_ERR_INVALID;
    *effective = c->pipe && c->megakernel ? group_frames(c) : 0;
    return RV_OK;
}

// Batched frame loop: groups of B = (frame slots) frames, each group one
// launch per stage with the frame index in the grid (FrameParams::nbatch),
// one RCCL gather of the group's packed tiles and one untile.  Group j runs
// on stream j & 1 with batch set j & 1 and frame slot j & 1's scheduling
// state, so group j+1 fills group j's tail while group j is gathered.
static rv_status render_batches(rv_ctx* c, const Seq& q, int32_t flags, rv_comm* comm, bool own0, hipStream_t caller,
                                size_t slice) {
    const int frames = q.n;
    const int B = (int)c->slots.size();
    const bool tiles = c->shard_n > 0, root = c->shard_rank == 0;
    const int W = c->cfg.width, H = c->cfg.height, T = c->shard_px;
    // packed tiles travel as RGB24 (alpha is always 255): 3/4 of the gather bytes
    const int bpp = c->gather_bpp;
    if (tiles) slice = (size_t)c->shard_max * T * T * bpp;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    const size_t cstride = c->own_color_pitch * H, mstride = c->own_mv_pitch * H, dstride = c->own_depth_pitch * H;
    const size_t gneed = tiles && root ? slice * (size_t)B * (size_t)c->shard_n : 0;
    for (BatchSet& b : c->bsets)
        if (rv_status as = bset_alloc(c, b, B, slice, gneed)) return as;
    // groups run on one stream by default (each launch then runs alone: its
    // duration is the kernel's own, as rocprof reports it); RV_BATCH_STREAMS=2
    // alternates two streams so a group's tail overlaps the next group
    hipStream_t S[2] = {own0 ? c->fstreams[0] : caller, own0 ? c->fstreams[1] : c->fstreams[0]};
    if (c->batch_streams < 2) S[1] = S[0];
    slot_save(c);
    if (tiles) {   // device tile lists and both slots' orders, on the caller's stream
        c->stream = caller;
        if (rv_status us = upload_ids(c, c->untile_ids, c->shard_all.data(), (int)c->shard_all.size(), nullptr)) return us;
        for (int k = 0; k < 2; k++) {
            slot_load(c, k);
            if (rv_status ts = tile_list(c, c->shard_ids.data(), (int32_t)c->shard_ids.size(), T)) return ts;
            slot_save(c);
        }
    }
    HIP_TRY(c, hipEventRecord(c->ev_loop, caller));
    for (hipStream_t x : S) {   // the caller's work, the last world/GI write, frames of earlier calls
        HIP_TRY(c, hipStreamWaitEvent(x, c->ev_loop, 0));
        if (c->world_stream != x) HIP_TRY(c, hipStreamWaitEvent(x, c->ev_world, 0));
        for (const FrameSlot& sl : c->slots)
            if (sl.pending) HIP_TRY(c, hipStreamWaitEvent(x, sl.done, 0));
    }
    const FrameCam* cams = nullptr;   // per-frame cameras (uploaded on the caller's stream, before the groups)
    if (!q.uniform(0, frames))
        if (rv_status us = upload_cams(c, q, caller, &cams)) return us;
    HIP_TRY(c, hipEventRecord(c->ev_loop, caller));
    for (hipStream_t x : S) HIP_TRY(c, hipStreamWaitEvent(x, c->ev_loop, 0));
    int done = 0, last_nb = 0, last = 0;
    int prev_k = -1, prev_nb = 0;   // root: group gathered but not yet assembled
    auto untile_group = [&](int kk, int nbb) -> rv_status {
        BatchSet& g = c->bsets[kk];
        HIP_TRY(c, hipStreamWaitEvent(S[kk], g.gathered, 0));
        launch_untile(S[kk], g.gbuf, c->untile_ids.d, (int)c->shard_all.size(), T, (W + T - 1) / T, W, H, g.color,
                      c->own_color_pitch, c->shard_max, nbb, cstride, bpp);
        LAUNCH_CHECK(c);
        return RV_OK;
    };
    for (int j = 0; done < frames; j++) {
        // the remaining frames in equal groups of at most B (20 frames at B = 16: 10 + 10, not 16 + 4)
        const int groups = (frames - done + B - 1) / B;
        const int nb = (frames - done + groups - 1) / groups, k = j & 1;
        BatchSet& bs = c->bsets[k];
        c->stream = S[k];
        slot_save(c);
        slot_load(c, k);
        if (bs.pending && tiles && !root) HIP_TRY(c, hipStreamWaitEvent(S[k], bs.gathered, 0));   // tile buffer reuse
        FrameParams f = make_params_d(c, q.at(done), flags);
        f.nbatch = (uint32_t)nb;
        if (cams) f.cams = cams + done;
        f.color = bs.color; f.color_pitch = c->own_color_pitch; f.bs_color = cstride;
        f.mv = bs.mv; f.mv_pitch = c->own_mv_pitch; f.bs_mv = mstride;
        f.depth = bs.depth; f.depth_pitch = c->own_depth_pitch; f.bs_depth = dstride;
        f.hdist = bs.hdist; f.hshadow = bs.hshadow; f.bs_half = hbytes;
        if (tiles) {
            if (rv_status ts = tile_list(c, c->shard_ids.data(), (int32_t)c->shard_ids.size(), T)) return ts;
            f.tiles = c->tiles.d; f.ntiles = (int)c->shard_ids.size(); f.tile_px = T;
            f.tiles_x = (W + T - 1) / T;
            f.tilebuf = bs.tbuf; f.bs_tile = slice; f.tile_bpp = bpp;
            f.chunk_order[CG_RENDER] = c->tile_order; f.chunk_cost[CG_RENDER] = c->tile_cost;
        }
        if (rv_status rs = run_stages(c, f, tiles)) return rs;
        c->frame_seq += (uint64_t)nb;
        const int tx = (W + T - 1) / std::max(T, 1);
        if (tiles && comm) {
            HIP_TRY(c, hipEventRecord(bs.rendered, S[k]));
            HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, bs.rendered, 0));
            const size_t part = slice * (size_t)nb;   // one rank's frames of the group
            if (root) HIP_TRY(c, hipMemcpyAsync(bs.gbuf, bs.tbuf, part, hipMemcpyDeviceToDevice, c->comm_stream));
            if (rv_status gs = comm_group_start(c, comm)) return gs;
            if (root) {
                for (int q = 1; q < c->shard_n; q++)
                    if (rv_status rs = comm_recv(c, comm, reinterpret_cast<char*>(bs.gbuf) + (size_t)q * part, part, q, c->comm_stream)) return rs;
            } else {
                if (rv_status ss = comm_send(c, comm, bs.tbuf, part, 0, c->comm_stream)) return ss;
            }
            if (rv_status ge = comm_group_end(c, comm, c->comm_stream)) return ge;
            HIP_TRY(c, hipEventRecord(bs.gathered, c->comm_stream));
            if (root) {   // assemble the previous group now: its gather overlapped this group's render
                if (prev_k >= 0)
                    if (rv_status us = untile_group(prev_k, prev_nb)) return us;
                prev_k = k; prev_nb = nb;
            }
        } else if (tiles && c->shard_n == 1) {   // one rank without a communicator: assemble locally
            launch_untile(S[k], bs.tbuf, c->untile_ids.d, (int)c->shard_all.size(), T, tx, W, H, bs.color,
                          c->own_color_pitch, c->shard_max, nb, cstride, bpp);
            LAUNCH_CHECK(c);
        }
        bs.pending = true;
        done += nb; last_nb = nb; last = k;
    }
    if (prev_k >= 0)
        if (rv_status us = untile_group(prev_k, prev_nb)) return us;
    // the last frame becomes slot 0's images (rv_readback / rv_image_ptr)
    slot_save(c);
    slot_load(c, 0);
    c->stream = S[last];
    if (!tiles || root)
        if (rv_status ps = bset_publish(c, c->bsets[last], (size_t)(last_nb - 1), !tiles, S[last])) return ps;
    // slot 0 is "done" when both groups' streams are: the caller's stream waits for all of it
    HIP_TRY(c, hipEventRecord(c->ev_loop, S[last ^ 1]));
    HIP_TRY(c, hipStreamWaitEvent(S[last], c->ev_loop, 0));
    if (c->comm_stream) {
        HIP_TRY(c, hipEventRecord(c->ev_loop, c->comm_stream));
        HIP_TRY(c, hipStreamWaitEvent(S[last], c->ev_loop, 0));
    }
    FrameSlot& s0 = c->slots[0];
    HIP_TRY(c, hipEventRecord(s0.done, S[last]));
    s0.pending = true;
    s0.last_stream = S[last];
    HIP_TRY(c, hipStreamWaitEvent(caller, s0.done, 0));
    return RV_OK;
}

extern "C" {

rv_status rv_tile_shard_assign(int32_t width, int32_t height, int32_t tile_px, int32_t nranks, float root_weight,
                               int32_t* owner) {
    if (width <= 0 || height <= 0 || tile_px <= 0 || nranks <= 0 || !owner) return RV_ERR_INVALID;
    const int nt = ((width + tile_px - 1) / tile_px) * ((height + tile_px - 1) / tile_px);
    const double w0 = std::min(1.0, std::max(0.05, (double)root_weight));
    // Tiles are dealt in order to the rank with the fewest tiles per unit of weight (ties: the
    // lowest rank): equal weights give the plain interleave t = rank, rank + nranks, ...
    std::vector<int> cnt((size_t)nranks, 0);
    for (int t = 0; t < nt; t++) {
        int best = 0;
        double bv = 0.0;
        for (int q = 0; q < nranks; q++) {
            const double v = (double)(cnt[(size_t)q] + 1) / (q == 0 ? w0 : 1.0);
            if (q == 0 || v < bv) { best = q; bv = v; }
        }
        cnt[(size_t)best]++;
        owner[t] = best;
    }
    return RV_OK;
}

rv_status rv_set_tile_shard_weighted(rv_ctx* c, int32_t tile_px, int32_t rank, int32_t nranks, float root_weight) {
    if (!c || nranks < 0 || (nranks > 0 && (rank < 0 || rank >= nranks))) return RV_ERR_INVALID;
    if (nranks > 0 && (tile_px < 16 || (tile_px & 15))) return fail(c, RV_ERR_INVALID, "tile_px must be a multiple of 16");
    if (nranks > 0 && !(root_weight > 0.0f && root_weight <= 1.0f))   // turning sharding off takes any weight
        return fail(c, RV_ERR_INVALID, "root weight must be in (0, 1]");
    c->shard_n = nranks; c->shard_rank = rank; c->shard_px = tile_px; c->shard_w0 = root_weight;
    c->shard_ids.clear(); c->shard_all.clear(); c->shard_max = 0;
    if (nranks == 0) return RV_OK;
    const int tx = (c->cfg.width + tile_px - 1) / tile_px, ty = (c->cfg.height + tile_px - 1) / tile_px;
    const int nt = tx * ty;
    std::vector<int32_t> owner((size_t)nt);
    if (rv_status as = rv_tile_shard_assign(c->cfg.width, c->cfg.height, tile_px, nranks, root_weight, owner.data()))
        return fail(c, as, "rv_tile_shard_assign");
    std::vector<std::vector<int32_t>> own((size_t)nranks);
    for (int t = 0; t < nt; t++) own[(size_t)owner[(size_t)t]].push_back(t);
    for (const auto& o : own) c->shard_max = std::max(c->shard_max, (int)o.size());
    c->shard_ids = own[(size_t)rank];
    c->shard_all.assign((size_t)nranks * c->shard_max, -1);              // gathered layout, -1 = padding slot
    for (int q = 0; q < nranks; q++)
        for (size_t k = 0; k < own[(size_t)q].size(); k++) c->shard_all[(size_t)q * c->shard_max + k] = own[(size_t)q][k];
    return RV_OK;
}

rv_status rv_set_tile_shard(rv_ctx* c, int32_t tile_px, int32_t rank, int32_t nranks) {
    if (!c) return RV_ERR_INVALID;
    return rv_set_tile_shard_weighted(c, tile_px, rank, nranks, 1.0f);
}

rv_status rv_set_gather_bpp(rv_ctx* c, int32_t bpp) {
    if (!c || (bpp != 3 && bpp != 4)) return RV_ERR_INVALID;
    c->gather_bpp = bpp;
    return RV_OK;
}

// The ranks of a communicator must agree on everything that shapes the
// exchange (shard, deal weight, packing, frame size, GI window), or the
// slices and all-gathers would mismatch: checked with one all-gather of a
// hash at the start of EVERY rv_render_frame_seq / rv_render_frames call
// with a communicator (then a bounded host wait).  The exchange is
// unconditional so every rank issues the same collectives in the same
// order: a rank whose configuration changed after an agreed call and a rank
// whose did not both enter it, see the disagreement and return
// RV_ERR_INVALID before any tile or GI exchange is issued.
static rv_status verify_ranks(rv_ctx* c, rv_comm* comm, int32_t flags, int32_t gi_per_frame, int loop, int frames) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { for (int b = 0; b < 8; b++) { h ^= (v >> (8 * b)) & 255u; h *= 1099511628211ull; } };
    uint32_t w0;
    std::memcpy(&w0, &c->shard_w0, 4);
    mix((uint64_t)comm->nranks); mix((uint64_t)c->shard_n); mix((uint64_t)c->shard_px); mix((uint64_t)c->gather_bpp);
    mix(w0); mix((uint64_t)c->shard_max); mix((uint64_t)c->cfg.width); mix((uint64_t)c->cfg.height);
    mix((uint64_t)c->cfg.gi_rays_per_frame); mix((uint64_t)(flags & ~RV_F_STATS));
    // the loop the call takes (render_seq's own predicate: batched / grouped with its group size /
    // pipelined / GI groups / per frame) and the frame count shape the sequence of collectives too
    mix((uint64_t)loop); mix((uint64_t)gi_per_frame); mix((uint64_t)frames); mix((uint64_t)c->slots.size());
    for (int32_t t : c->shard_all) mix((uint64_t)(uint32_t)t);
    if (!c->comm_stream) HIP_TRY(c, hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    const size_t nr = (size_t)comm->nranks;
    if (!comm->vdev) HIP_TRY(c, hipMalloc(&comm->vdev, 8 * (nr + 1)));
    if (!comm->vhost) HIP_TRY(c, hipHostMalloc(&comm->vhost, 8 * (nr + 1), hipHostMallocDefault));
    // the pinned word holding this rank's hash is read by the upload below before the bounded wait returns
    comm->vhost[nr] = h;
    rv_status st = RV_OK;
    if (hipMemcpyAsync(comm->vdev + nr, comm->vhost + nr, 8, hipMemcpyHostToDevice, c->comm_stream) != hipSuccess)
        st = fail(c, RV_ERR_HIP, "hipMemcpyAsync");
    if (st == RV_OK) st = comm_all_gather(c, comm, comm->vdev + nr, comm->vdev, 8, c->comm_stream);
    if (st == RV_OK && hipMemcpyAsync(comm->vhost, comm->vdev, 8 * nr, hipMemcpyDeviceToHost, c->comm_stream) != hipSuccess)
        st = fail(c, RV_ERR_HIP, "hipMemcpyAsync");
    if (st == RV_OK) st = comm_wait_bounded(c, comm, comm_timeout_s());
    if (st != RV_OK) return st;
    for (size_t r = 0; r < nr; r++)
        if (comm->vhost[r] != h)
            return fail(c, RV_ERR_INVALID, "ranks disagree on the shard / deal weight / gather packing / frame config "
                                            "/ loop (rank " + std::to_string(r) + ")");
    comm->verified = h;
    return RV_OK;
}

static rv_status render_seq(rv_ctx* c, const Seq& q, int32_t flags, int32_t gi_per_frame, rv_comm* comm) {
    const int frames = q.n;
    if (comm) {
        // a communicator belongs to the context it was created on (rv_comm_destroy
        // detaches only that one, rv_sync / rv_destroy wait on it)
        if (comm->ctx != c) return fail(c, RV_ERR_INVALID, "communicator was created on another context");
        c->comm_attached = comm;
        // the loop this call takes: the same predicates as below
        const int ns = (int)c->slots.size(), gF0 = group_frames(c);
        const bool ref = gi_per_frame && (flags & RV_F_PREPASS) && c->megakernel && frames > 0;
        const int loop = (!gi_per_frame && ns > 1 && c->megakernel && frames > 0) ? 1
                         : (ref && c->pipe && gF0 >= 2 && !(flags & RV_F_STATS)) ? 100 + gF0
                         : (ref && c->pipe) ? 2
                         : (ref && c->shard_n == 0 && ns > 1) ? 3 : 0;
        if (rv_status vs = verify_ranks(c, comm, flags, gi_per_frame, loop, frames)) return vs;
    }
    if (!c->world_ready) return fail(c, RV_ERR_STATE, "rv_render_frames before world");
    if (comm && (c->shard_n != comm->nranks || c->shard_rank != comm->rank))
        return fail(c, RV_ERR_INVALID, "tile shard does not match the communicator");
    const int n = (int)c->slots.size();
    const bool tiles = c->shard_n > 0;
    const int T = c->shard_px;
    const size_t slice = (size_t)c->shard_max * T * T * 4;
    // streams of slots 1..n-1, the comm stream and buffers, created on first use
    int prio = 0;   // slot streams run at the caller stream's priority
    if (c->stream) HIP_TRY(c, hipStreamGetPriority(c->stream, &prio));
    if (!c->fstreams.empty() && c->fstream_prio != prio) {
        // only the streams depend on the priority; batch buffers and events stay
        HIP_TRY(c, hipDeviceSynchronize());
        for (hipStream_t fs : c->fstreams) hipStreamDestroy(fs);
        c->fstreams.clear();
    }
    c->fstream_prio = prio;
    // slot 0 runs on the caller's stream unless that is the legacy NULL
    // stream (which would serialise with the others): then on a stream of its own
    const bool own0 = c->stream == nullptr;
    const int nown = own0 ? n : n - 1;
    while ((int)c->fstreams.size() < nown) {
        hipStream_t st;
        HIP_TRY(c, hipStreamCreateWithPriority(&st, hipStreamNonBlocking, prio));
        c->fstreams.push_back(st);
    }
    if (!c->ev_loop) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_loop, hipEventDisableTiming));
    if (tiles) {
        if (comm && !c->comm_stream) HIP_TRY(c, hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        const bool root = c->shard_rank == 0;
        const size_t gneed = root ? slice * (size_t)c->shard_n : 0;
        for (FrameSlot& sl : c->slots) {
            if (sl.tbytes != slice || sl.gbytes != gneed) {
                HIP_TRY(c, hipDeviceSynchronize());
                hipFree(sl.tbuf); hipFree(sl.gbuf);
                sl.tbuf = nullptr; sl.gbuf = nullptr; sl.tbytes = sl.gbytes = 0;
                HIP_TRY(c, hipMalloc(&sl.tbuf, slice));
                if (gneed) HIP_TRY(c, hipMalloc(&sl.gbuf, gneed));
                sl.tbytes = slice; sl.gbytes = gneed;
            }
        }
    }
    hipStream_t caller = c->stream;
    uint32_t* saved_ext = c->ext_tilebuf; size_t saved_ext_bytes = c->ext_tilebuf_bytes;
    rv_status st = RV_OK;
    // the loop's streams start after the caller's work so far
    HIP_TRY(c, hipEventRecord(c->ev_loop, caller));
    for (hipStream_t fs : c->fstreams) HIP_TRY(c, hipStreamWaitEvent(fs, c->ev_loop, 0));
    if (c->comm_stream) HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, c->ev_loop, 0));
    if (!gi_per_frame && n > 1 && c->megakernel && frames > 0) {
        st = render_batches(c, q, flags, comm, own0, caller, slice);
        c->ext_tilebuf = saved_ext; c->ext_tilebuf_bytes = saved_ext_bytes;
        c->stream = caller;
        return st;
    }
    const int gF = group_frames(c);
    if (gi_per_frame && (flags & RV_F_PREPASS) && c->pipe && c->megakernel && frames > 0 && gF >= 2 &&
        !(flags & RV_F_STATS)) {
        hipStream_t S = own0 ? c->fstreams[0] : caller;
        st = render_gi_group(c, q, flags, S, comm, gF);
        c->stream = caller;
        if (st != RV_OK) return st;
        if (S != caller) HIP_TRY(c, hipStreamWaitEvent(caller, c->slots[0].done, 0));
        return RV_OK;
    }
    if (gi_per_frame && (flags & RV_F_PREPASS) && c->pipe && c->megakernel && frames > 0) {
        hipStream_t S = own0 ? c->fstreams[0] : caller;
        st = render_gi_pipe(c, q, flags, S, comm);
        c->stream = caller;
        if (st != RV_OK) return st;
        if (S != caller) HIP_TRY(c, hipStreamWaitEvent(caller, c->slots[0].done, 0));
        return RV_OK;
    }
    if (gi_per_frame && (flags & RV_F_PREPASS) && !tiles && n > 1 && c->megakernel && frames > 0) {
        hipStream_t S = own0 ? c->fstreams[0] : caller;
        st = render_gi_groups(c, q, flags, S);
        c->stream = caller;
        if (st != RV_OK) return st;
        if (S != caller) HIP_TRY(c, hipStreamWaitEvent(caller, c->slots[0].done, 0));
        return RV_OK;
    }
    for (int k = 0; k < frames && st == RV_OK; k++) {
        const int s = (int)(c->frame_seq % (uint64_t)n);   // the slot begin_frame will pick
        // per-frame GI updates serialise the frames: one stream then
        const int si = gi_per_frame ? 0 : s;
        c->stream = own0 ? c->fstreams[si] : (si == 0 ? caller : c->fstreams[si - 1]);
        if (gi_per_frame && (st = rv_update_gi_data(c)) != RV_OK) break;
        const rv_frame_desc& d = q.at(k);
        if (!tiles) { st = rv_frame(c, &d.cam, d.vp, d.prev_vp, d.time, d.jitter_x, d.jitter_y, flags); continue; }
        FrameSlot& sl = c->slots[s];
        c->ext_tilebuf = sl.tbuf; c->ext_tilebuf_bytes = sl.tbytes;
        st = rv_frame_tiles(c, &d.cam, d.vp, d.prev_vp, d.time, d.jitter_x, d.jitter_y, flags, c->shard_ids.data(),
                            (int32_t)c->shard_ids.size(), T);
        if (st != RV_OK) break;
        HIP_TRY(c, hipEventRecord(sl.done, c->stream));   // the render, also with one slot
        sl.pending = true;
        if (comm) {   // gather to rank 0 on the comm stream, in frame order on every rank
            HIP_TRY(c, hipStreamWaitEvent(c->comm_stream, sl.done, 0));
            if (c->shard_rank == 0)
                HIP_TRY(c, hipMemcpyAsync(sl.gbuf, sl.tbuf, slice, hipMemcpyDeviceToDevice, c->comm_stream));
            if (rv_status gs = comm_group_start(c, comm)) return gs;
            if (c->shard_rank == 0) {
                for (int q = 1; q < c->shard_n; q++)
                    if (rv_status rs = comm_recv(c, comm, reinterpret_cast<char*>(sl.gbuf) + (size_t)q * slice, slice, q, c->comm_stream)) return rs;
            } else {
                if (rv_status ss = comm_send(c, comm, sl.tbuf, slice, 0, c->comm_stream)) return ss;
            }
            if (rv_status ge = comm_group_end(c, comm, c->comm_stream)) return ge;
            HIP_TRY(c, hipEventRecord(sl.gathered, c->comm_stream));
            HIP_TRY(c, hipStreamWaitEvent(c->stream, sl.gathered, 0));   // slot reuse after the send
            if (c->shard_rank == 0)
                st = rv_untile(c, sl.gbuf, c->shard_all.data(), (int32_t)c->shard_all.size(), T);
            else
                st = end_frame(c);
        } else if (c->shard_n == 1) {   // one rank, no communicator: assemble locally
            st = rv_untile(c, sl.tbuf, c->shard_all.data(), (int32_t)c->shard_all.size(), T);
        }
    }
    c->ext_tilebuf = saved_ext; c->ext_tilebuf_bytes = saved_ext_bytes;
    c->stream = caller;
    if (st != RV_OK) return st;
    // the caller's stream sees every frame of the loop complete
    for (const FrameSlot& sl : c->slots)
        if (sl.pending) HIP_TRY(c, hipStreamWaitEvent(caller, sl.done, 0));
    if (c->slots.size() == 1 && own0) {   // one slot on an own stream: no slot event was recorded
        HIP_TRY(c, hipEventRecord(c->ev_loop, c->fstreams[0]));
        HIP_TRY(c, hipStreamWaitEvent(caller, c->ev_loop, 0));
    }
    return RV_OK;
}

rv_status rv_render_frame_seq(rv_ctx* c, int32_t frames, const rv_frame_desc* seq, const rv_frame_desc* next,
                              int32_t flags, int32_t gi_per_frame, rv_comm* comm) {
    if (!c || frames < 0 || (frames > 0 && !seq)) return RV_ERR_INVALID;
    if (!c->world_ready) return fail(c, RV_ERR_STATE, "rv_render_frame_seq before world");
    if (comm && (c->shard_n != comm->nranks || c->shard_rank != comm->rank))
        return fail(c, RV_ERR_INVALID, "tile shard does not match the communicator");
    if (frames == 0) return RV_OK;
    Seq q;
    q.d = seq; q.stride = 1; q.n = frames; q.next = next;
    return render_seq(c, q, flags, gi_per_frame, comm);
}

rv_status rv_render_frames(rv_ctx* c, int32_t frames, const rv_camera* cam, const float* vp16, const float* pvp16,
                           float time, float jx, float jy, int32_t flags, int32_t gi_per_frame, rv_comm* comm) {
    if (!c || !cam || frames < 0) return RV_ERR_INVALID;
    if (!c->world_ready) return fail(c, RV_ERR_STATE, "rv_render_frames before world");
    if (comm && (c->shard_n != comm->nranks || c->shard_rank != comm->rank))
        return fail(c, RV_ERR_INVALID, "tile shard does not match the communicator");
    if (frames == 0) return RV_OK;
    rv_frame_desc d;
    d.cam = *cam;
    for (int i = 0; i < 16; i++) {
        d.vp[i] = vp16 ? vp16[i] : (i % 5 == 0 ? 1.0f : 0.0f);
        d.prev_vp[i] = pvp16 ? pvp16[i] : d.vp[i];
    }
    d.time = time; d.jitter_x = jx; d.jitter_y = jy;
    Seq q;
    q.d = &d; q.stride = 0; q.n = frames;
    return render_seq(c, q, flags, gi_per_frame, comm);
}

}  // extern "C"
