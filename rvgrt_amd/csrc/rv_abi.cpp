// rv_abi.cpp -- host side of librvgrt_hip.so, part 1 of the C ABI (include/rvgrt.h): contexts, world build /
// import / export, the GI update, single frames (flow frames, drawCUDA), readback and stats.  The frame
// loops are in rv_loops.cpp, the transport in rv_comm.cpp; the context they share in rv_host.h.  Every entry
// point converts failures into rv_status + message.
#include "rv_host.h"

extern "C" {

int32_t rv_abi_version(void) { return RVGRT_ABI_VERSION; }

const char* rv_last_error(const rv_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

rv_status rv_create(const rv_config* cfg, int32_t device, rv_ctx** out) {
    if (!cfg || !out) return RV_ERR_INVALID;
    *out = nullptr;
    if (cfg->log2_x < 4 || cfg->log2_y < 4 || cfg->log2_z < 4 || cfg->log2_x > 13 || cfg->log2_y > 13 ||
        cfg->log2_z > 13)
        return RV_ERR_INVALID;
    // brick records must stay below 4 GiB (32-bit gather offsets): <= 2^34 voxels
    if (cfg->log2_x + cfg->log2_y + cfg->log2_z > 34) return RV_ERR_INVALID;
    if (cfg->width < 2 || cfg->height < 2) return RV_ERR_INVALID;   // any parity: half-res images floor(W/2) x floor(H/2)
    if (cfg->width > 32768 || cfg->height > 32768) return RV_ERR_INVALID;   // images < 4 GiB: 32-bit offsets
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return RV_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RV_ERR_NO_DEVICE;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RV_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return RV_ERR_NO_DEVICE;

    rv_ctx* c = new rv_ctx();
    c->device = device;
    c->cfg = *cfg;
    if (c->cfg.gi_rays_per_frame == 0) c->cfg.gi_rays_per_frame = 64 * 64 * 64;
    c->lx = cfg->log2_x; c->ly = cfg->log2_y; c->lz = cfg->log2_z;
    World& w = c->w;
    w.X = 1 << c->lx; w.Y = 1 << c->ly; w.Z = 1 << c->lz;
    w.lbx = c->lx - 3; w.lbxy = (c->lx - 3) + (c->ly - 3);
    w.lbz = c->lz - 3; w.lbzy = (c->lz - 3) + (c->ly - 3);
    w.SX = w.X / 2; w.SY = w.Y / 2; w.SZ = w.Z / 2;
    w.GX = w.X / 4; w.GY = w.Y / 4; w.GZ = w.Z / 4;
    w.fX = (float)w.X; w.fY = (float)w.Y; w.fZ = (float)w.Z;
    world_set_regions(w, ((uint64_t)w.X * w.Y * w.Z) / 512);
    // 128 B per 512 voxels (bits and CSDF regions), then the sun horizon (rv_device.h horizon_at)
    c->brick_bytes = dtop_byte(w.coff, w.X, w.Z) + dtop_bytes(w.X, w.Z);
    c->gi_bytes = n_gi(c) * 4;

    auto cleanup_fail = [&](rv_status s, const char* what) {
        std::string m = std::string("rv_create: ") + what;
        rv_destroy(c);
        (void)m;
        return s;
    };
    if (hipMalloc(&c->brick, c->brick_bytes) != hipSuccess) return cleanup_fail(RV_ERR_OOM, "bricks");
    if (hipMalloc(&c->gi, c->gi_bytes) != hipSuccess) return cleanup_fail(RV_ERR_OOM, "gi");
    hipMemset(c->brick, 0, horizon_byte(w.coff));
    hipMemset(reinterpret_cast<char*>(c->brick) + horizon_byte(w.coff), 0xFF, horizon_bytes(w.X, w.Z));   // no sun exit
    hipMemset(reinterpret_cast<char*>(c->brick) + dtop_byte(w.coff, w.X, w.Z), 0x7F, dtop_bytes(w.X, w.Z));   // no skip
    hipMemset(c->gi, 0, c->gi_bytes);
    // atlas
    int aw = cfg->atlas_rgba8 ? cfg->atlas_w : 256, ah = cfg->atlas_rgba8 ? cfg->atlas_h : 256;
    if (aw <= 0 || ah <= 0) return cleanup_fail(RV_ERR_INVALID, "atlas dims");
    w.aw = aw; w.ah = ah;
    // held in World's tiled layout (rv_device.h atlas_tiled_off): 128-B lines of 2D texel blocks
    std::vector<uint32_t> tiled(atlas_tiled_texels(aw, ah), 0u);
    for (int r = 0; r < ah; r++)
        for (int q = 0; q < aw; q++) {
            uint32_t t = 0xFF808080u;   // grey without an atlas
            if (cfg->atlas_rgba8) std::memcpy(&t, static_cast<const uint8_t*>(cfg->atlas_rgba8) + 4 * ((size_t)r * aw + q), 4);
            tiled[atlas_tiled_off(aw, r, q)] = t;
        }
    if (hipMalloc(&c->atlas, tiled.size() * 4) != hipSuccess) return cleanup_fail(RV_ERR_OOM, "atlas");
    hipMemcpy(c->atlas, tiled.data(), tiled.size() * 4, hipMemcpyHostToDevice);
    c->cfg.atlas_rgba8 = nullptr;
    // frame slot 0 (more with rv_set_frames_in_flight)
    int W = cfg->width, H = cfg->height;
    c->own_color_pitch = align256((size_t)W * 4);
    c->own_mv_pitch = align256((size_t)W * 4);
    c->own_depth_pitch = align256((size_t)W * 2);
    c->color_pitch = c->own_color_pitch; c->mv_pitch = c->own_mv_pitch; c->depth_pitch = c->own_depth_pitch;
    c->slots.resize(1);
    if (!slot_alloc(c, c->slots[0])) return cleanup_fail(RV_ERR_OOM, "frame slot");
    slot_load(c, 0);
    if (hipMalloc(&c->counters, NSTAGE * NCNT * sizeof(unsigned long long)) != hipSuccess)
        return cleanup_fail(RV_ERR_OOM, "counters");
    hipMemset(c->counters, 0, NSTAGE * NCNT * sizeof(unsigned long long));
    {   // wavefront stage buffers
        size_t npx = (size_t)W * H, nhalf = (size_t)(W / 2) * (H / 2);
        bool ok = hipMalloc(&c->hpos, npx * 16) == hipSuccess && hipMalloc(&c->hinfo, npx * 4) == hipSuccess &&
                  hipMalloc(&c->hsec, npx * 16) == hipSuccess && hipMalloc(&c->pphit, nhalf * 16) == hipSuccess &&
                  hipMalloc(&c->qcount, QCOUNT_BYTES) == hipSuccess;
        if (!ok) return cleanup_fail(RV_ERR_OOM, "wavefront buffers");
        hipMemset(c->qcount, 0, QCOUNT_BYTES);   // queues themselves: sized per frame by ensure_queues
    }
#ifdef RV_WAVE_TRACE
    if (getenv("RV_WAVE_TRACE")) {
        c->wtrace_bytes = (size_t)sched_grid<8, 8>(SCHED_COST, W, H) * 32;   // one 32-B record per 8x8-pixel wave tile
        if (hipMalloc(&c->wtrace, c->wtrace_bytes) != hipSuccess) return cleanup_fail(RV_ERR_OOM, "wave trace");
        hipMemset(c->wtrace, 0, c->wtrace_bytes);
    }
#endif
    if (hipEventCreateWithFlags(&c->ev_world, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_gi_done, hipEventDisableTiming) != hipSuccess ||
        hipDeviceGetStreamPriorityRange(&c->prio_lo, &c->prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c->gi_stream, hipStreamNonBlocking, gi_prio(c)) != hipSuccess)
        return cleanup_fail(RV_ERR_HIP, "gi stream/events");
    if (hipDeviceSynchronize() != hipSuccess) return cleanup_fail(RV_ERR_HIP, "init sync");
    *out = c;
    return RV_OK;
}

void rv_destroy(rv_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->comm_attached) {   // a communicator still open: never hang on a dead peer
        if (comm_wait_bounded(c, c->comm_attached, comm_timeout_s()) == RV_OK) hipDeviceSynchronize();
        comm_detach(c->comm_attached);
    } else {
        hipDeviceSynchronize();   // every frame slot's stream
    }
    hipFree(c->brick); hipFree(c->gi); hipFree(c->gi_tmp); hipFree(c->atlas); hipFree(c->tex);
    for (auto& ph : c->pipe_half) { hipFree(ph[0]); hipFree(ph[1]); }
    for (int q = 0; q < 2; q++) { hipFree(c->pipe_tbuf[q]); hipFree(c->pipe_gbuf[q]); }
    hipFree(c->pipe_gi_stage); hipFree(c->pipe_gi_all);
    for (hipEvent_t e : c->pipe_ev) if (e) hipEventDestroy(e);
    if (c->flow_wtrace) {   // RV_FLOW_WAVE_TRACE: header {len0, len1, len2, n}, then 4 dwords per workgroup
        std::vector<uint32_t> h((size_t)c->flow_wtrace_n * 4 + 4);
        h[0] = c->flow_wlen[0]; h[1] = c->flow_wlen[1]; h[2] = c->flow_wlen[2]; h[3] = c->flow_wtrace_n;
        if (hipMemcpy(h.data() + 4, c->flow_wtrace, (size_t)c->flow_wtrace_n * 16, hipMemcpyDeviceToHost) == hipSuccess)
            if (FILE* fp = fopen(getenv("RV_FLOW_WAVE_TRACE"), "wb")) { fwrite(h.data(), 4, h.size(), fp); fclose(fp); }
        hipFree(c->flow_wtrace);
    }
    if (c->pipe_wstat) {   // RV_PIPE_WAVE_STATS: per part, the longest wave and the 99th percentile per launch
        const char* names[3] = {"gi", "prepass", "render"};
        double mx[3] = {0, 0, 0}, p99[3] = {0, 0, 0};
        uint32_t used = 0;
        for (uint32_t i = 4; i < c->pipe_launches; i++, used++) {   // the first launches warm the cost order
            std::vector<uint32_t> h(c->pipe_wnb[i]);
            if (hipMemcpy(h.data(), c->pipe_wstat + (size_t)i * (1u << 18), h.size() * 4, hipMemcpyDeviceToHost) !=
                hipSuccess)
                break;
            for (int q = 0; q < 3; q++) {
                std::vector<uint32_t> v;
                for (uint32_t r : h)
                    if (r != 0xFFFFFFFFu && (r >> 30) == (uint32_t)q) v.push_back(r & 0x3FFFFFFFu);
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                mx[q] += v.back();
                p99[q] += v[(size_t)(0.99 * (double)(v.size() - 1))];
            }
        }
        for (int q = 0; used && q < 3; q++)
            fprintf(stderr, "[rvgrt] pipe waves %-8s longest %7.1f us  p99 %7.1f us  (mean over %u launches)\n",
                    names[q], mx[q] / used / 100.0, p99[q] / used / 100.0, used);
        hipFree(c->pipe_wstat);
    }
    if (!c->slots.empty()) slot_save(c);
    for (FrameSlot& sl : c->slots) slot_free(sl);
    hipFree(c->counters);
    hipFree(c->d_top);
    hipFree(c->coltop);
    hipFree(c->tiles.d); hipFree(c->untile_ids.d);
    hipFree(c->tilebuf);
    hipFree(c->hpos); hipFree(c->hinfo); hipFree(c->hsec); hipFree(c->pphit); hipFree(c->qcount);
    for (int q = 0; q < NQUEUE; q++) hipFree(c->wq[q]);
    for (hipEvent_t e : c->ev) hipEventDestroy(e);
#ifdef RV_WAVE_TRACE
    if (c->wtrace) {   // env RV_WAVE_TRACE=<file>: dump the last frame's wave records
        std::vector<uint32_t> h(c->wtrace_bytes / 4);
        if (hipMemcpy(h.data(), c->wtrace, c->wtrace_bytes, hipMemcpyDeviceToHost) == hipSuccess) {
            if (FILE* fp = fopen(getenv("RV_WAVE_TRACE"), "wb")) { fwrite(h.data(), 4, h.size(), fp); fclose(fp); }
        }
        hipFree(c->wtrace);
    }
#endif
    if (c->gi_stream) { hipStreamSynchronize(c->gi_stream); hipStreamDestroy(c->gi_stream); }
    hipFree(c->grec_stage); hipFree(c->grec_all); hipFree(c->gring);
    for (hipEvent_t e : c->gev) if (e) hipEventDestroy(e);
    if (c->grp_stream) hipStreamDestroy(c->grp_stream);
    for (BatchSet* bs : {&c->bsets[0], &c->bsets[1], &c->gsets[0], &c->gsets[1]}) {
        BatchSet& b = *bs;
        hipFree(b.color); hipFree(b.mv); hipFree(b.depth); hipFree(b.hdist); hipFree(b.hshadow);
        hipFree(b.tbuf); hipFree(b.gbuf);
        if (b.rendered) hipEventDestroy(b.rendered);
        if (b.gathered) hipEventDestroy(b.gathered);
    }
    for (hipStream_t fs : c->fstreams) hipStreamDestroy(fs);
    if (c->comm_stream) hipStreamDestroy(c->comm_stream);
    if (c->ev_loop) hipEventDestroy(c->ev_loop);
    if (c->ev_world) hipEventDestroy(c->ev_world);
    hipFree(c->flow_half); hipFree(c->flow_fb);
    if (c->ev_spec) hipEventDestroy(c->ev_spec);
    if (c->ev_flow) hipEventDestroy(c->ev_flow);
    hipFree(c->cam_dev);
    if (c->cam_host) hipHostFree(c->cam_host);
    if (c->cam_ev) hipEventDestroy(c->cam_ev);
    if (c->ev_gi_done) hipEventDestroy(c->ev_gi_done);
    delete c;
}

rv_status rv_set_stream(rv_ctx* c, void* s) {
    if (!c) return RV_ERR_INVALID;
    c->stream = (hipStream_t)s;
    return RV_OK;
}

rv_status rv_set_option(rv_ctx* c, int32_t opt, int64_t v) {
    if (!c) return RV_ERR_INVALID;
    switch (opt) {
    case RV_OPT_PIPE_ORDER: {   // a permutation of the parts PIPE_GI / PIPE_PP / PIPE_RENDER
        const uint32_t a = (uint32_t)(v >> 8 & 0xF), b = (uint32_t)(v >> 4 & 0xF), d = (uint32_t)(v & 0xF);
        if (v < 0 || v > 0x210 || a > 2 || b > 2 || d > 2 || a == b || b == d || a == d)
            return fail(c, RV_ERR_INVALID, "RV_OPT_PIPE_ORDER: not a permutation of 0, 1, 2");
        c->pipe_order = (uint32_t)v;
        c->carry_gi = c->carry_pp = false;
        return RV_OK;
    }
    case RV_OPT_BATCH_STREAMS:
        if (v != 1 && v != 2) return fail(c, RV_ERR_INVALID, "RV_OPT_BATCH_STREAMS: 1 or 2");
        c->batch_streams = (int)v;
        return RV_OK;
    case RV_OPT_FLOW_SPIN:
        if (v < 0 || v > (1 << 30)) return fail(c, RV_ERR_INVALID, "RV_OPT_FLOW_SPIN: 0 .. 2^30");
        c->flow_spin = (uint32_t)v;
        return RV_OK;
    case RV_OPT_FLOW_FORCE_FALLBACK:
        c->flow_force_fallback = v != 0;
        return RV_OK;
    case RV_OPT_GI_PAIRS:
        if (v < -1 || v > 1) return fail(c, RV_ERR_INVALID, "RV_OPT_GI_PAIRS: -1, 0 or 1");
        c->gi_pairs = (int)v;
        return RV_OK;
    case RV_OPT_GI_SHARD_PROBE:
        c->gi_shard_probe = v != 0;
        return RV_OK;
    default:
        return fail(c, RV_ERR_INVALID, "unknown option " + std::to_string(opt));
    }
}

rv_status rv_get_option(rv_ctx* c, int32_t opt, int64_t* v) {
    if (!c || !v) return RV_ERR_INVALID;
    switch (opt) {
    case RV_OPT_PIPE_ORDER: *v = c->pipe_order; return RV_OK;
    case RV_OPT_BATCH_STREAMS: *v = c->batch_streams; return RV_OK;
    case RV_OPT_FLOW_SPIN: *v = c->flow_spin; return RV_OK;
    case RV_OPT_FLOW_FORCE_FALLBACK: *v = c->flow_force_fallback ? 1 : 0; return RV_OK;
    case RV_OPT_GI_PAIRS: *v = c->gi_pairs; return RV_OK;
    case RV_OPT_GI_SHARD_PROBE: *v = c->gi_shard_probe ? 1 : 0; return RV_OK;
    default: return fail(c, RV_ERR_INVALID, "unknown option " + std::to_string(opt));
    }
}

// Frames in flight: frame k takes slot k % n; its stream first waits for
// the slot's previous frame (the slot's buffers are reused) and for the last
// world/GI write (which may have been issued on another stream).
static rv_status begin_frame(rv_ctx* c) {
    const int n = (int)c->slots.size();
    if (n > 1) {
        const int s = (int)(c->frame_seq % (uint64_t)n);
        slot_save(c);
        slot_load(c, s);
        FrameSlot& sl = c->slots[s];
        // cross-stream waits only: same-stream work is already ordered
        if (sl.pending && sl.last_stream != c->stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, sl.done, 0));
        if (sl.world_seen != c->world_ver || sl.last_stream != c->stream) {
            if (c->world_stream != c->stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_world, 0));
            sl.world_seen = c->world_ver;
        }
        sl.last_stream = c->stream;
        sl.submitted = c->frame_seq;
    } else if (c->world_stream != c->stream) {
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_world, 0));
    }
    c->frame_seq++;
    return RV_OK;
}

RV_HIDDEN rv_status end_frame(rv_ctx* c) {
    if (c->slots.size() > 1) {
        FrameSlot& sl = c->slots[c->cur_slot];
        HIP_TRY(c, hipEventRecord(sl.done, c->stream));
        sl.pending = true;
    }
    return RV_OK;
}

// Before anything that rewrites state frames read (world, GI grid, device
// tile lists): `stream` waits for every frame still in flight.
RV_HIDDEN rv_status wait_all_frames(rv_ctx* c) {
    if (c->world_stream != c->stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_world, 0));   // write after write
    if (c->slots.size() > 1)
        for (const FrameSlot& sl : c->slots)
            if (sl.pending) HIP_TRY(c, hipStreamWaitEvent(c->stream, sl.done, 0));
    return RV_OK;
}

// Everything that writes the world or the GI grid runs on `stream`; the GI
// side stream waits on this mark before it reads them.
RV_HIDDEN rv_status mark_world(rv_ctx* c) {
    HIP_TRY(c, hipEventRecord(c->ev_world, c->stream));
    c->world_ver++;
    c->world_stream = c->stream;
    return RV_OK;
}

// Uploads `src` to ids unless it equals the cached list; *changed tells.
RV_HIDDEN rv_status upload_ids(rv_ctx* c, DevIds& ids, const int32_t* src, int n, bool* changed) {
    const bool same = ids.d && ids.h.size() == (size_t)n && (n == 0 || memcmp(ids.h.data(), src, (size_t)n * 4) == 0);
    if (changed) *changed = !same;
    if (same) return RV_OK;
    if (rv_status ws = wait_all_frames(c)) return ws;   // frames in flight may read the old list
    if ((size_t)n > ids.cap || !ids.d) {
        HIP_TRY(c, c->slots.size() > 1 ? hipDeviceSynchronize() : hipStreamSynchronize(c->stream));
        hipFree(ids.d);
        ids.d = nullptr;
        ids.cap = 0;
        HIP_TRY(c, hipMalloc(&ids.d, (size_t)(n > 0 ? n : 1) * 4));
        ids.cap = (size_t)(n > 0 ? n : 1);
    }
    ids.h.assign(src, src + n);   // the copy reads this stable host buffer
    if (n > 0) HIP_TRY(c, hipMemcpyAsync(ids.d, ids.h.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    return RV_OK;
}

rv_status rv_set_frame_path(rv_ctx* c, int32_t path) {
    if (!c || (path != RV_PATH_FUSED && path != RV_PATH_WAVEFRONT)) return RV_ERR_INVALID;
    if (path == RV_PATH_WAVEFRONT && c->slots.size() > 1)
        return fail(c, RV_ERR_STATE, "the wavefront path runs one frame at a time");
    c->megakernel = path == RV_PATH_FUSED;
    return RV_OK;
}

rv_status rv_set_frames_in_flight(rv_ctx* c, int32_t n) {
    if (!c || n < 1 || n > 32) return RV_ERR_INVALID;
    if (n > 1 && !c->megakernel) return fail(c, RV_ERR_STATE, "frames in flight need the fused path");
    HIP_TRY(c, hipDeviceSynchronize());
    slot_save(c);
    while ((int)c->slots.size() > n) { slot_free(c->slots.back()); c->slots.pop_back(); }
    while ((int)c->slots.size() < n) {
        c->slots.emplace_back();
        if (!slot_alloc(c, c->slots.back())) {
            slot_free(c->slots.back());
            c->slots.pop_back();
            slot_load(c, 0);
            return fail(c, RV_ERR_OOM, "frame slot");
        }
    }
    slot_load(c, 0);
    c->frame_seq = 0;
    return RV_OK;
}

rv_status rv_set_gi_async(rv_ctx* c, int32_t on) {
    if (!c) return RV_ERR_INVALID;
    c->gi_async = on != 0;
    return RV_OK;
}

rv_status rv_set_pipeline(rv_ctx* c, int32_t on) {
    if (!c) return RV_ERR_INVALID;
    c->pipe = on != 0;
    c->carry_gi = c->carry_pp = false;
    return RV_OK;
}

rv_status rv_tex_table_info(rv_ctx* c, int32_t* active, uint64_t* bytes) {
    if (!c) return RV_ERR_INVALID;
    if (active) *active = c->tex != nullptr;
    if (bytes) *bytes = c->tex ? (uint64_t)c->w.X * c->w.tex_ny * c->w.Z * 4 : 0;
    return RV_OK;
}

rv_status rv_set_flow(rv_ctx* c, int32_t on) {
    if (!c) return RV_ERR_INVALID;
    c->flow = on != 0;
    c->spec_gi = false;
    return RV_OK;
}

rv_status rv_flow_info(rv_ctx* c, int32_t* active, uint64_t* launches, uint64_t* fallbacks) {
    if (!c) return RV_ERR_INVALID;
    // in effect: on, one frame slot, the megakernel path (flow_eligible's frame-independent part)
    if (active) *active = c->flow && c->megakernel && c->slots.size() == 1;
    if (launches) *launches = c->flow_launches;
    if (fallbacks) {
        *fallbacks = 0;
        if (c->flow_fb) {
            // the last flow launch may have run on another stream than the current one (rv_set_stream
            // between frames): wait for the event recorded after it
            if (c->ev_flow) HIP_TRY(c, hipEventSynchronize(c->ev_flow));
            unsigned long long v = 0;
            HIP_TRY(c, hipMemcpy(&v, c->flow_fb, 8, hipMemcpyDeviceToHost));
            *fallbacks = v;
        }
    }
    return RV_OK;
}

rv_status rv_set_frame_group(rv_ctx* c, int32_t n) {
    if (!c || n < 0 || n > 32) return RV_ERR_INVALID;
    c->group = n;
    c->carry_gi = c->carry_pp = false;
    return RV_OK;
}

rv_status rv_set_gi_stats(rv_ctx* c, int32_t on) {
    if (!c) return RV_ERR_INVALID;
    c->gi_stats = on != 0;
    return RV_OK;
}

rv_status rv_sync(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    if (c->comm_attached) return comm_wait_bounded(c, c->comm_attached, comm_timeout_s());   // never hangs on a peer
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->slots.size() > 1)
        for (const FrameSlot& sl : c->slots)
            if (sl.pending) HIP_TRY(c, hipEventSynchronize(sl.done));
    return RV_OK;
}

// sampleTexture's tile table (World::tex, rv_device.h tex_index): 4 B per voxel of the rows below the sky
// exit (World::ytop rounded up to 8), a function of the voxel coordinates only, so it is built once, after
// the first world build or bits import (bench.py's world_build_s includes it) and kept through rebuilds (a
// hit above its rows takes the noise).  It is optional -- a context without it evaluates the noise in
// the kernels, with identical tiles -- so it is only allocated when it leaves room: the memory this
// context may still allocate (CSDF build scratch, the GI scratch grid, two grouped-frame sets of 32
// frames, the pipelined loop's buffers) plus 1 GiB, and at most half the device's free memory (other
// contexts on the GPU).  rv_config.tex_table -1: never; 1: whenever the allocation succeeds.
static rv_status tex_table(rv_ctx* c) {
    if (c->tex_tried) return RV_OK;
    c->tex_tried = true;
    if (c->cfg.tex_table < 0) return RV_OK;
    const bool force = c->cfg.tex_table > 0;
    const uint32_t ny = std::min((uint32_t)c->w.Y, (c->w.ytop + 7u) & ~7u);
    const size_t tb = (size_t)c->w.X * ny * c->w.Z * 4;
    if (!force) {
        size_t fr = 0, total = 0;
        HIP_TRY(c, hipMemGetInfo(&fr, &total));
        const size_t W = (size_t)c->cfg.width, H = (size_t)c->cfg.height;
        const size_t frame = (c->own_color_pitch + c->own_mv_pitch + c->own_depth_pitch) * H + W * H * 2;
        const size_t later = n_csdf(c) * 2 + c->gi_bytes + 2 * 32 * frame + 8 * W * H + ((size_t)1 << 30);
        if (tb + later > fr || tb > fr / 2) return RV_OK;
    }
    if (hipMalloc(&c->tex, tb) != hipSuccess) {
        c->tex = nullptr;
        (void)hipGetLastError();
        return RV_OK;
    }
    c->w.tex_ny = ny;
    launch_tex_table(c->stream, c->tex, c->w);
    LAUNCH_CHECK(c);
    c->w.tex = c->tex;
    return RV_OK;
}

// The sky exit of the frame traversal (World::ytop, rv_device.h trace): the highest solid voxel
// row + 2, and the sun exit of its shadow rays (World::horizon), recomputed after every write of the
// bits.  rv_config.exits_off & RV_EXIT_SKY turns all three exits off (ytop = Y, no horizon, no skip).
static rv_status world_top(rv_ctx* c) {
    c->w.ytop = (uint32_t)c->w.Y;
    uint32_t* hz = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->brick) + horizon_byte(c->w.coff));
    const size_t hzb = horizon_bytes(c->w.X, c->w.Z);
    HIP_TRY(c, hipMemsetAsync(hz, 0xFF, hzb, c->stream));   // no sun exit unless built below
    int* dt = reinterpret_cast<int*>(reinterpret_cast<char*>(c->brick) + dtop_byte(c->w.coff, c->w.X, c->w.Z));
    HIP_TRY(c, hipMemsetAsync(dt, 0x7F, dtop_bytes(c->w.X, c->w.Z), c->stream));   // no column skip unless built below
    const int off = c->cfg.exits_off;
    if (off & RV_EXIT_SKY) return RV_OK;
    if (!c->d_top) HIP_TRY(c, hipMalloc(&c->d_top, 4));
    HIP_TRY(c, hipMemsetAsync(c->d_top, 0, 4, c->stream));
    launch_world_top(c->stream, c->brick, current_world(c), c->d_top);
    LAUNCH_CHECK(c);
    uint32_t top = 0;
    HIP_TRY(c, hipMemcpyAsync(&top, c->d_top, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->w.ytop = std::min((uint32_t)c->w.Y, top + 1u);   // top = max solid y + 1
    // the column tops: the DDA's empty-column skip (dtop_at; RV_EXIT_COLUMN: off) and the sun horizon's input
    if (!c->coltop) HIP_TRY(c, hipMalloc(&c->coltop, hzb));
    HIP_TRY(c, hipMemsetAsync(c->coltop, 0, hzb, c->stream));
    launch_column_tops(c->stream, c->brick, current_world(c), c->coltop, dt);
    LAUNCH_CHECK(c);
    if (off & RV_EXIT_COLUMN) HIP_TRY(c, hipMemsetAsync(dt, 0x7F, dtop_bytes(c->w.X, c->w.Z), c->stream));
    // the sun exit of shadow rays (trace_sun): the horizon per brick column for the library's sun
    // (RV_EXIT_SUN: off)
    const f3 sun = sun_dir();
    const double hxz = std::sqrt((double)sun.x * sun.x + (double)sun.z * sun.z);
    if ((off & RV_EXIT_SUN) || !(sun.y > 0.0f) || hxz == 0.0) return RV_OK;
    // slope shaded 0.1 % low (a lower slope only raises the horizon: conservative)
    const float k = (float)((double)sun.y / hxz * (1.0 - 1e-3));
    launch_sun_horizon(c->stream, current_world(c), c->coltop, hz, (float)(sun.x / hxz), (float)(sun.z / hxz), k);
    LAUNCH_CHECK(c);
    return RV_OK;
}

rv_status rv_csdf_build(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    if (rv_status ws = wait_all_frames(c)) return ws;
    c->geom_ver++;
    uint64_t n = n_csdf(c);
    // Scratch of the three passes: plain allocations, freed after the build completed.  (Stream-
    // ordered hipMallocAsync scratch on the legacy stream was measured to overlap allocations of
    // later contexts' grouped-frame buffers in the same process: sporadically corrupted CSDF.)
    uint8_t *t0 = nullptr, *t1 = nullptr;
    HIP_TRY(c, hipMalloc((void**)&t0, n));
    HIP_TRY(c, hipMalloc((void**)&t1, n));
    launch_csdf(c->stream, c->brick, current_world(c), t0, t1);
    LAUNCH_CHECK(c);
    const hipError_t se = hipStreamSynchronize(c->stream);
    hipFree(t0);
    hipFree(t1);
    HIP_TRY(c, se);
    return mark_world(c);
}

rv_status rv_gi_init(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    if (rv_status ws = wait_all_frames(c)) return ws;
    launch_gi_init(c->stream, c->gi, current_world(c), sun_dir(),
                   c->cfg.gi_init_saturate ? RV_GI_LIT_SATURATE : RV_GI_LIT_REFERENCE, c->counters + ST_GI * NCNT);
    LAUNCH_CHECK(c);
    c->gi_frame = 0;
    c->gi_offset = 0;
    return mark_world(c);
}

rv_status rv_world_build(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    if (rv_status ws = wait_all_frames(c)) return ws;
    c->geom_ver++;
    launch_fill_bricks(c->stream, c->brick, current_world(c), c->cfg.seed_x, c->cfg.seed_z);
    LAUNCH_CHECK(c);
    if (rv_status ts = world_top(c)) return ts;
    if (rv_status ts = tex_table(c)) return ts;
    rv_status s = rv_csdf_build(c);
    if (s != RV_OK) return s;
    s = rv_gi_init(c);
    if (s != RV_OK) return s;
    c->world_ready = true;
    return RV_OK;
}

rv_status rv_world_import(rv_ctx* c, int32_t kind, const void* host, size_t bytes) {
    if (!c || !host) return RV_ERR_INVALID;
    if (rv_status ws = wait_all_frames(c)) return ws;
    if (kind != RV_WORLD_GI) c->geom_ver++;
    if (kind == RV_WORLD_BITS) {
        if (bytes != n_bits_words(c) * 4) return fail(c, RV_ERR_INVALID, "bits size mismatch");
        uint32_t* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, bytes));
        HIP_TRY(c, hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, c->stream));
        launch_bits_import(c->stream, d, c->brick, current_world(c), c->lx, c->ly);
        LAUNCH_CHECK(c);
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        hipFree(d);
        if (rv_status ts = world_top(c)) return ts;
        if (rv_status ts = tex_table(c)) return ts;
    } else if (kind == RV_WORLD_CSDF) {
        if (bytes != n_csdf(c)) return fail(c, RV_ERR_INVALID, "csdf size mismatch");
        uint8_t* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, bytes));
        HIP_TRY(c, hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, c->stream));
        launch_csdf_import(c->stream, d, c->brick, current_world(c));
        LAUNCH_CHECK(c);
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        hipFree(d);
    } else if (kind == RV_WORLD_GI) {
        if (bytes != c->gi_bytes) return fail(c, RV_ERR_INVALID, "gi size mismatch");
        HIP_TRY(c, hipMemcpyAsync(c->gi, host, bytes, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    } else {
        return fail(c, RV_ERR_INVALID, "bad world kind");
    }
    c->world_ready = true;
    return mark_world(c);
}

rv_status rv_world_export(rv_ctx* c, int32_t kind, void* host, size_t bytes) {
    if (!c || !host) return RV_ERR_INVALID;
    if (kind == RV_WORLD_BITS) {
        if (bytes != n_bits_words(c) * 4) return fail(c, RV_ERR_INVALID, "bits size mismatch");
        uint32_t* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, bytes));
        launch_bits_export(c->stream, c->brick, d, current_world(c), c->lx, c->ly);
        LAUNCH_CHECK(c);
        HIP_TRY(c, hipMemcpyAsync(host, d, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        hipFree(d);
    } else if (kind == RV_WORLD_CSDF) {
        if (bytes != n_csdf(c)) return fail(c, RV_ERR_INVALID, "csdf size mismatch");
        uint8_t* d = nullptr;
        HIP_TRY(c, hipMalloc(&d, bytes));
        launch_csdf_export(c->stream, c->brick, d, current_world(c));
        LAUNCH_CHECK(c);
        HIP_TRY(c, hipMemcpyAsync(host, d, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        hipFree(d);
    } else if (kind == RV_WORLD_GI) {
        if (bytes != c->gi_bytes) return fail(c, RV_ERR_INVALID, "gi size mismatch");
        HIP_TRY(c, hipMemcpyAsync(host, c->gi, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    } else {
        return fail(c, RV_ERR_INVALID, "bad world kind");
    }
    return RV_OK;
}

// One GI update over [first, first+count).  Serial: kernel + copy-back on
// `stream`.  Async (partial ranges only): the kernel runs on gi_stream after
// the last world/GI write and overlaps whatever `stream` has queued since
// (the previous frame's render, which reads `gi` only); `stream` waits for
// it before copying the range back, so every later reader sees the update.
static rv_status gi_update(rv_ctx* c, uint32_t frame, uint64_t first, uint64_t count, bool async,
                           hipEvent_t t0, hipEvent_t t1) {
    uint64_t n = n_gi(c);
    if (first >= n) return RV_OK;
    if (first + count > n) count = n - first;
    if (!c->gi_tmp) HIP_TRY(c, hipMalloc(&c->gi_tmp, c->gi_bytes));
    if (count == n) async = false;   // full sweep flips the double buffer instead
    hipStream_t ks = async ? c->gi_stream : c->stream;
    // the last world/GI write may have been issued on another stream
    if (async || c->world_stream != ks) HIP_TRY(c, hipStreamWaitEvent(ks, c->ev_world, 0));
    // gi_tmp is about to be written: frames in flight from before the last
    // flip of the double buffer still read it
    if (c->slots.size() > 1)
        for (const FrameSlot& sl : c->slots)
            if (sl.pending && sl.submitted < c->gi_swapped_at) HIP_TRY(c, hipStreamWaitEvent(ks, sl.done, 0));
    // a flow launch's GI part may still be writing gi_tmp (its cells for the next window)
    if (c->spec_rec && c->spec_stream != ks) HIP_TRY(c, hipStreamWaitEvent(ks, c->ev_spec, 0));
    if (t0) HIP_TRY(c, hipEventRecord(t0, ks));
    launch_gi_update(ks, c->gi, c->gi_tmp, current_world(c), sun_dir(), frame, first, count,
                     c->counters + ST_GI * NCNT, c->gi_stats);
    LAUNCH_CHECK(c);
    if (t1) HIP_TRY(c, hipEventRecord(t1, ks));
    if (async) {
        HIP_TRY(c, hipEventRecord(c->ev_gi_done, ks));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_gi_done, 0));
    }
    if (rv_status ws = wait_all_frames(c)) return ws;   // frames in flight still read `gi`
    if (count == n) {
        std::swap(c->gi, c->gi_tmp);   // full sweep: flip the double buffer
        c->gi_swapped_at = c->frame_seq;
    } else {
        launch_copy_u32(c->stream, c->gi + first, c->gi_tmp + first, count);
        LAUNCH_CHECK(c);
    }
    return mark_world(c);
}

rv_status rv_gi_update(rv_ctx* c, uint32_t frame, uint64_t first, uint64_t count) {
    if (!c) return RV_ERR_INVALID;
    return gi_update(c, frame, first, count, false, nullptr, nullptr);
}

rv_status rv_update_gi_data(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    uint64_t rays = c->cfg.gi_rays_per_frame, n = n_gi(c);
    const bool timed = c->timing_n < c->timing_cap;
    hipEvent_t* e = timed ? &c->ev[(size_t)EV_PER_FRAME * c->timing_n] : nullptr;
    c->upd_since_frame = true;
    const uint64_t count = c->gi_offset < n ? std::min(rays, n - c->gi_offset) : 0;
    rv_status s;
    if (c->spec_gi && c->spec_world == c->world_ver && c->spec_fr == c->gi_frame && c->spec_first == c->gi_offset &&
        c->spec_count == count && !c->gi_stats) {
        // computed ahead by the last flow launch (reads the same grid, same cells and frame number):
        // only its copy-back is left, after that launch
        c->spec_gi = false;
        if (c->spec_stream != c->stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_spec, 0));
        if (rv_status ws = wait_all_frames(c)) return ws;
        if (timed) HIP_TRY(c, hipEventRecord(e[NSTAGE], c->stream));
        launch_copy_u32(c->stream, c->gi + c->gi_offset, c->gi_tmp + c->gi_offset, count);
        LAUNCH_CHECK(c);
        if (timed) HIP_TRY(c, hipEventRecord(e[NSTAGE + 1], c->stream));
        s = mark_world(c);
    } else {
        c->spec_gi = false;
        s = gi_update(c, c->gi_frame, c->gi_offset, rays, c->gi_async, timed ? e[NSTAGE] : nullptr,
                      timed ? e[NSTAGE + 1] : nullptr);
    }
    if (s != RV_OK) return s;
    if (timed) c->gi_timed[c->timing_n] = 1;
    c->gi_frame++;
    if (c->gi_offset + rays >= n) c->gi_offset = 0;   // src/CoarseArray.cu:392-394
    else c->gi_offset += rays;
    return RV_OK;
}

static FrameParams make_params(rv_ctx* c, const rv_camera* cam, const float* vp, const float* pvp, float time,
                               float jx, float jy, int32_t flags) {
    FrameParams f{};
    f.pos = host_v(cam->pos[0], cam->pos[1], cam->pos[2]);
    f.fo = host_v(cam->forward[0], cam->forward[1], cam->forward[2]);
    f.ri = host_v(cam->right[0], cam->right[1], cam->right[2]);
    f.up = host_v(cam->up[0], cam->up[1], cam->up[2]);
    f.sun = sun_dir();
    f.time = time; f.jx = jx; f.jy = jy;
    cone_basis_scales(f.cone_k1, f.cone_k2);
    for (int i = 0; i < 16; i++) {
        f.vp[i] = vp ? vp[i] : (i % 5 == 0 ? 1.0f : 0.0f);
        f.pvp[i] = pvp ? pvp[i] : f.vp[i];
    }
    f.W = c->cfg.width; f.H = c->cfg.height; f.hw = f.W / 2; f.hh = f.H / 2;
    f.flags = flags;
    f.color = c->color; f.color_pitch = c->color_pitch;
    f.mv = c->mv; f.mv_pitch = c->mv_pitch;
    f.depth = c->depth; f.depth_pitch = c->depth_pitch;
    f.hdist = c->hdist; f.hshadow = c->hshadow;
    f.counters = c->counters;
    f.sched = c->sched;
    for (int g = 0; g < 2; g++) { f.chunk_order[g] = c->chunk_order[g]; f.chunk_cost[g] = c->chunk_cost[g]; }
    f.hpos = c->hpos; f.hinfo = c->hinfo; f.hsec = c->hsec; f.pphit = c->pphit;
    for (int q = 0; q < NQUEUE; q++) f.queue_wf[q] = c->wq[q];
    f.qcount = c->qcount;
    f.enq = c->enq;
    f.wtrace = c->wtrace;
    f.nbatch = 1;
    return f;
}

RV_HIDDEN FrameParams make_params_d(rv_ctx* c, const rv_frame_desc& d, int32_t flags) {
    return make_params(c, &d.cam, d.vp, d.prev_vp, d.time, d.jitter_x, d.jitter_y, flags);
}


static FrameCam frame_cam(const rv_frame_desc& d) {
    FrameCam fc{};
    fc.pos = host_v(d.cam.pos[0], d.cam.pos[1], d.cam.pos[2]);
    fc.fo = host_v(d.cam.forward[0], d.cam.forward[1], d.cam.forward[2]);
    fc.ri = host_v(d.cam.right[0], d.cam.right[1], d.cam.right[2]);
    fc.up = host_v(d.cam.up[0], d.cam.up[1], d.cam.up[2]);
    fc.time = d.time; fc.jx = d.jitter_x; fc.jy = d.jitter_y;
    for (int i = 0; i < 16; i++) { fc.vp[i] = d.vp[i]; fc.pvp[i] = d.prev_vp[i]; }
    return fc;
}

// Uploads the cameras of all frames of a sequence (batched launches index it
// from their first frame) on stream st; returns the device table.  The
// pinned staging buffer is reused only after its last upload has executed.
RV_HIDDEN rv_status upload_cams(rv_ctx* c, const Seq& q, hipStream_t st, const FrameCam** out,
                             const std::function<void(int, FrameCam&)>& fill) {
    const size_t n = (size_t)q.n;
    if (c->cam_pending) HIP_TRY(c, hipEventSynchronize(c->cam_ev));
    if (n > c->cam_cap) {
        HIP_TRY(c, hipDeviceSynchronize());   // kernels of earlier calls may still read the old table
        hipFree(c->cam_dev);
        if (c->cam_host) hipHostFree(c->cam_host);
        c->cam_dev = nullptr; c->cam_host = nullptr; c->cam_cap = 0;
        const size_t cap = std::max<size_t>(n, 256);
        HIP_TRY(c, hipMalloc(&c->cam_dev, cap * sizeof(FrameCam)));
        HIP_TRY(c, hipHostMalloc(&c->cam_host, cap * sizeof(FrameCam), hipHostMallocDefault));
        c->cam_cap = cap;
    }
    if (!c->cam_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->cam_ev, hipEventDisableTiming));
    for (size_t k = 0; k < n; k++) {
        c->cam_host[k] = frame_cam(q.at((int)k));
        if (fill) fill((int)k, c->cam_host[k]);
    }
    HIP_TRY(c, hipMemcpyAsync(c->cam_dev, c->cam_host, n * sizeof(FrameCam), hipMemcpyHostToDevice, st));
    HIP_TRY(c, hipEventRecord(c->cam_ev, st));
    c->cam_pending = true;
    *out = c->cam_dev;
    return RV_OK;
}


// Enqueue the frame's stages, recording a start event per stage when timing
// is on.  Each stage counts into its own counter block (rv_stats_stage).
// Per-XCD sub-queue capacities of this frame's producer grids (FrameParams
// ::qcap); grows the queue buffers when a tile list needs more room.
static rv_status ensure_queues(rv_ctx* c, FrameParams& f, bool tiles) {
    for (int q = 0; q < NQUEUE; q++) {
        uint32_t blocks = wf_producer_blocks(f, q, tiles);
        f.qcap[q] = (blocks + NXCD - 1) / NXCD * 256;
        size_t need = (size_t)NXCD * f.qcap[q];
        if (need > c->wq_cap[q]) {
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            hipFree(c->wq[q]);
            c->wq[q] = nullptr;
            c->wq_cap[q] = 0;
            if (hipMalloc(&c->wq[q], need * 4) != hipSuccess) return fail(c, RV_ERR_OOM, "wavefront queues");
            c->wq_cap[q] = need;
        }
        f.queue_wf[q] = c->wq[q];
    }
    return RV_OK;
}

// which: 1 = the pre-pass, 2 = the render (fused path), 3 = both.
RV_HIDDEN rv_status run_stages(rv_ctx* c, FrameParams f, bool tiles, int which) {
    if (!c->megakernel) {
        rv_status st = ensure_queues(c, f, tiles);
        if (st != RV_OK) return st;
    }
    // Stage timing: one event where a stage starts and one at the end of
    // the frame, on the stages that run (an event costs a few us of gap).
    const bool timed = c->timing_n < c->timing_cap;
    const size_t e0 = (size_t)EV_PER_FRAME * c->timing_n;
    int used = 0;
    auto mark = [&](int k) -> hipError_t {
        if (!timed) return hipSuccess;
        c->ev_stage[e0 + used] = (signed char)k;
        return hipEventRecord(c->ev[e0 + used++], c->stream);
    };
    World w = current_world(c);
    auto stage = [&](int k) { FrameParams g = f; g.counters = c->counters + (size_t)k * NCNT; return g; };
    const bool pre = (f.flags & RV_F_PREPASS) != 0;
    if (c->megakernel) {
        if (pre && (which & 1)) {
            HIP_TRY(c, mark(ST_PP_PRIMARY));
            if (tiles) launch_prepass_tiles(c->stream, w, stage(ST_PP_PRIMARY));
            else launch_prepass(c->stream, w, stage(ST_PP_PRIMARY));
            LAUNCH_CHECK(c);
        }
        if (which & 2) {
            HIP_TRY(c, mark(ST_PRIMARY));
            if (tiles) launch_render_tiles(c->stream, w, stage(ST_PRIMARY)); else launch_render(c->stream, w, stage(ST_PRIMARY));
            LAUNCH_CHECK(c);
        }
        HIP_TRY(c, mark(-1));
        if (!(which & 2)) {   // a pre-pass-only launch: orders are rebuilt after the renders
            if (timed) c->ev_used[c->timing_n] = used;
            if (timed) c->timing_n++;
            return RV_OK;
        }
        // SCHED_COST: re-order the chunks by the wave lifetimes (max over
        // the frames since the last ordering) every order_every frames; a
        // kernel boundary costs ~6 us, the ordering itself ~4 us (both grids' orderings in one launch).
        if (f.sched == SCHED_COST && ++c->frames_since_order >= (uint32_t)c->order_every) {
            c->frames_since_order = 0;
            if (tiles) {
                launch_chunk_order(c->stream, c->tile_cost, c->tile_order, (uint32_t)f.ntiles,
                                   ((uint32_t)f.ntiles + 7u) & ~7u);
            } else {
                launch_chunk_order(c->stream, pre ? c->chunk_cost[CG_PREPASS] : nullptr, c->chunk_order[CG_PREPASS],
                                   n_chunks(f.hw, f.hh), n_chunks_pad(f.hw, f.hh),
                                   c->chunk_cost[CG_RENDER], c->chunk_order[CG_RENDER], n_chunks(f.W, f.H),
                                   n_chunks_pad(f.W, f.H));
            }
            LAUNCH_CHECK(c);
        }
    } else {
        HIP_TRY(c, hipMemsetAsync(c->qcount, 0, QCOUNT_BYTES, c->stream));
        if (pre) {
            HIP_TRY(c, mark(ST_PP_PRIMARY));
            launch_wf_pp_primary(c->stream, w, stage(ST_PP_PRIMARY), tiles);
            LAUNCH_CHECK(c);
            HIP_TRY(c, mark(ST_PP_SHADOW));
            launch_wf_pp_shadow(c->stream, w, stage(ST_PP_SHADOW));
            LAUNCH_CHECK(c);
        }
        HIP_TRY(c, mark(ST_PRIMARY));
        launch_wf_primary(c->stream, w, stage(ST_PRIMARY), tiles);
        LAUNCH_CHECK(c);
        if (!pre && (f.flags & RV_F_SHADOW)) {
            HIP_TRY(c, mark(ST_SHADOW));
            launch_wf_shadow(c->stream, w, stage(ST_SHADOW));
            LAUNCH_CHECK(c);
        }
        if (f.flags & RV_F_WATER) {
            HIP_TRY(c, mark(ST_WATER));
            launch_wf_water(c->stream, w, stage(ST_WATER));
            LAUNCH_CHECK(c);
        }
        if (f.flags & RV_F_GI) {
            HIP_TRY(c, mark(ST_CONES));
            launch_wf_cones(c->stream, w, stage(ST_CONES));
            LAUNCH_CHECK(c);
        }
        HIP_TRY(c, mark(ST_SHADE));
        launch_wf_shade(c->stream, w, stage(ST_SHADE), tiles);
        LAUNCH_CHECK(c);
        HIP_TRY(c, mark(-1));
    }
    if (timed) c->ev_used[c->timing_n] = used;
    if (timed) c->timing_n++;
    return RV_OK;
}

// Flow frame (rv_set_flow, default on): the drop-in drawCUDA of a frame with the pre-pass as one
// k_ref_flow launch on `stream` -- pre-pass k | the next UpdateGIData's cells | render k, the render
// waves waiting per half-res tile for the pre-pass waves of the same launch (rv_kernels.hip), so the
// pre-pass's long camera + shadow rays overlap the render instead of forming a launch of their own.
// The GI part runs only while the caller updates the grid before every frame (renderLoop's
// UpdateGIData -> drawCUDA, src/main.cpp:119-132): its window is the one rv_update_gi_data will
// apply next, read from the grid this frame renders with; that call then only copies it back.
// The render part reads its 8 half-res taps per pixel from an 8x8-texel LDS window (rv_frame.h HalfWin) that
// holds every tap only when the half-res images are W/2 x H/2 (Appendix R6); a tap outside it would read the
// global image, which the same launch's pre-pass writes without ordering -- so the flow launch requires that
// shape (make_params always sets it; the check keeps any other resolution on the two-launch path).
static bool flow_eligible(const rv_ctx* c, const FrameParams& f) {
    return c->flow && c->megakernel && c->slots.size() == 1 && (f.flags & RV_F_PREPASS) != 0 && f.hw > 0 && f.hh > 0 &&
           f.hw == f.W / 2 && f.hh == f.H / 2;
}

static rv_status flow_frame(rv_ctx* c, FrameParams f) {
    const uint32_t ntx = (uint32_t)(f.hw + 7) / 8, nty = (uint32_t)(f.hh + 7) / 8;
    const size_t ntiles = (size_t)ntx * nty;
    if (c->flow_tiles != ntiles || !c->flow_half) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        hipFree(c->flow_half);
        c->flow_half = nullptr; c->flow_tiles = 0;
        HIP_TRY(c, hipMalloc(&c->flow_half, ntiles * 64 * 8));
        HIP_TRY(c, hipMemset(c->flow_half, 0, ntiles * 64 * 8));   // tag 0: no launch's
        c->flow_tiles = ntiles;
        c->flow_epoch = 0;
    }
    if (!c->flow_fb) {
        HIP_TRY(c, hipMalloc(&c->flow_fb, 8));
        HIP_TRY(c, hipMemset(c->flow_fb, 0, 8));
    }
    if (++c->flow_epoch > 0x3FFFFFFFu) {   // 30-bit epochs (tag = epoch << 1 | phase): restart them from a zeroed buffer
        HIP_TRY(c, hipMemsetAsync(c->flow_half, 0, ntiles * 64 * 8, c->stream));
        c->flow_epoch = 1;
    }
    const bool stats = (f.flags & RV_F_STATS) != 0;
    const uint64_t n = n_gi(c), rays = c->cfg.gi_rays_per_frame;
    const uint64_t first = c->gi_offset, count = first < n ? std::min(rays, n - first) : 0;
    const bool spec_valid = c->spec_gi && c->spec_world == c->world_ver && c->spec_fr == c->gi_frame &&
                            c->spec_first == first && c->spec_count == count;
    // a full sweep flips the double buffer instead (gi_update); stats frames keep their counters clean
    const bool spec = c->upd_since_frame && !spec_valid && !stats && !c->gi_stats && count > 0 && count < n;
    if (spec && !c->gi_tmp) HIP_TRY(c, hipMalloc(&c->gi_tmp, c->gi_bytes));
    PipeParams p{};
    p.gi_prev = c->gi;
    if (spec) {
        p.gi_frame = c->gi_frame; p.gi_first = first; p.gi_count = count;
        p.gi_next = c->gi_tmp + first;
        c->carry_gi = false;   // the pipelined loop's kept update shares gi_tmp
    }
    p.pp_counters = c->counters + (size_t)ST_PP_PRIMARY * NCNT;
    p.gi_counters = c->counters + (size_t)ST_GI * NCNT;
    f.counters = c->counters + (size_t)ST_PRIMARY * NCNT;
    p.part[0] = PIPE_PP; p.part[1] = PIPE_GI; p.part[2] = PIPE_RENDER;
    if (RV_PIPE_DIAG)   // diagnostics builds only (tools/flow_waves.py): the pre-pass alone, one tile's waves
        if (const char* e = getenv("RV_FLOW_OPTS")) p.flow_opts = (uint32_t)atoi(e);
    // pre-pass workgroups: 16 per render chunk slot in the render's order
    p.len[0] = n_chunks_pad(f.W, f.H) * 16u;
    p.len[2] = pipe_len(f, PIPE_RENDER, 0);
    p.gi_pairs = c->gi_pairs > 0 && pipe_latency_variant(f, p.len[2]) ? 1u : 0u;   // whole frames: off unless forced
    p.len[1] = spec ? pipe_len(f, PIPE_GI, p.gi_pairs ? 2 * count : count) : 0u;
    p.flow_half = c->flow_half;
    p.flow_epoch = c->flow_epoch; p.flow_ntx = ntx;
    p.flow_expect = c->flow_force_fallback ? c->flow_epoch ^ 0x20000000u : c->flow_epoch;
    p.flow_spin = c->flow_spin;
    p.flow_fallback = c->flow_fb;
    if (RV_PIPE_DIAG && getenv("RV_FLOW_WAVE_TRACE")) {   // diagnostics: this launch's per-wave records
        const uint32_t nb = p.len[0] + p.len[1] + p.len[2];
        if (nb > c->flow_wtrace_n) {
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            hipFree(c->flow_wtrace);
            c->flow_wtrace = nullptr;
            HIP_TRY(c, hipMalloc(&c->flow_wtrace, (size_t)nb * 16));
        }
        c->flow_wtrace_n = nb;
        c->flow_wlen[0] = p.len[0]; c->flow_wlen[1] = p.len[1]; c->flow_wlen[2] = p.len[2];
        HIP_TRY(c, hipMemsetAsync(c->flow_wtrace, 0xFF, (size_t)nb * 16, c->stream));
        p.wave_max = c->flow_wtrace;
    }
    const bool timed = c->timing_n < c->timing_cap;
    const size_t e0 = (size_t)EV_PER_FRAME * c->timing_n;
    if (timed) { c->ev_stage[e0] = ST_PRIMARY; HIP_TRY(c, hipEventRecord(c->ev[e0], c->stream)); }
    launch_ref_flow(c->stream, current_world(c), f, p);
    LAUNCH_CHECK(c);
    c->flow_launches++;
    if (!c->ev_flow) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_flow, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(c->ev_flow, c->stream));
    if (timed) {
        c->ev_stage[e0 + 1] = -1;
        HIP_TRY(c, hipEventRecord(c->ev[e0 + 1], c->stream));
        c->ev_used[c->timing_n] = 2;
        c->timing_n++;
    }
    if (spec) {
        if (!c->ev_spec) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_spec, hipEventDisableTiming));
        HIP_TRY(c, hipEventRecord(c->ev_spec, c->stream));
        c->spec_stream = c->stream;
        c->spec_rec = true;
        c->spec_gi = true;
        c->spec_fr = c->gi_frame; c->spec_first = first; c->spec_count = count; c->spec_world = c->world_ver;
    }
    if (f.sched == SCHED_COST && ++c->frames_since_order >= (uint32_t)c->order_every) {
        c->frames_since_order = 0;
        launch_chunk_order(c->stream, c->chunk_cost[CG_PREPASS], c->chunk_order[CG_PREPASS], n_chunks(f.hw, f.hh),
                           n_chunks_pad(f.hw, f.hh), c->chunk_cost[CG_RENDER],
                           c->chunk_order[CG_RENDER], n_chunks(f.W, f.H), n_chunks_pad(f.W, f.H));
        LAUNCH_CHECK(c);
    }
    return RV_OK;
}

rv_status rv_frame(rv_ctx* c, const rv_camera* cam, const float* vp16, const float* pvp16, float time,
                   float jx, float jy, int32_t flags) {
    if (!c || !cam) return RV_ERR_INVALID;
    if (!c->world_ready) return fail(c, RV_ERR_STATE, "rv_frame before rv_world_build/import");
    if (rv_status bs = begin_frame(c)) return bs;
    FrameParams f = make_params(c, cam, vp16, pvp16, time, jx, jy, flags);
    const bool upd = c->upd_since_frame;
    c->upd_since_frame = false;
    if (flow_eligible(c, f)) {
        c->upd_since_frame = upd;   // flow_frame reads it
        rv_status fs = flow_frame(c, f);
        c->upd_since_frame = false;
        if (fs != RV_OK) return fs;
    } else if (rv_status rs = run_stages(c, f, false)) {
        return rs;
    }
    return end_frame(c);
}

rv_status rv_draw_cuda(rv_ctx* c, const float pos[3], const float fo[3], const float up[3], const float ri[3],
                       const float* vp16, const float* pvp16, float jitter_x, float jitter_y) {
    if (!c || !pos || !fo || !up || !ri) return RV_ERR_INVALID;
    rv_camera cam{};
    for (int i = 0; i < 3; i++) { cam.pos[i] = pos[i]; cam.forward[i] = fo[i]; cam.up[i] = up[i]; cam.right[i] = ri[i]; }
    float time, jx, jy;
    if (c->cfg.ref_compat) {
        // c_time = c_cam[17] = host jitterY; c_jitterX = c_cam[18] (never
        // written, 0); c_jitterY = c_cam[19] (4 B past the symbol).
        time = jitter_y; jx = 0.0f; jy = c->cfg.ref_oob_jy;
        return rv_frame(c, &cam, vp16, pvp16, time, jx, jy, c->cfg.flags | RV_F_REF_FETCH);
    } else {
        long long ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                           std::chrono::system_clock::now().time_since_epoch()).count();
        time = (float)(ms % 1000000) * 0.001f;
        jx = jitter_x; jy = jitter_y;
    }
    return rv_frame(c, &cam, vp16, pvp16, time, jx, jy, c->cfg.flags);
}

// Device tile list (uploaded when it changes) and the active slot's
// SCHED_COST order/cost arrays for it (identity order, zero costs whenever
// the slot has not rendered this list yet).
RV_HIDDEN rv_status tile_list(rv_ctx* c, const int32_t* tile_ids, int32_t ntiles, int32_t tile_px) {
    bool changed = false;
    rv_status us = upload_ids(c, c->tiles, tile_ids, ntiles, &changed);
    if (us != RV_OK) return us;
    if (changed) c->tiles_ver++;
    if (c->tiles_seen != c->tiles_ver || tile_px != c->tiles_px) {
        const size_t npad = ((size_t)ntiles + 7) & ~(size_t)7;
        if (npad > c->tile_ord_cap) {
            HIP_TRY(c, c->slots.size() > 1 ? hipDeviceSynchronize() : hipStreamSynchronize(c->stream));
            hipFree(c->tile_order); hipFree(c->tile_cost);
            c->tile_order = nullptr; c->tile_cost = nullptr; c->tile_ord_cap = 0;
            HIP_TRY(c, hipMalloc(&c->tile_order, npad * 4));
            HIP_TRY(c, hipMalloc(&c->tile_cost, npad * 4));
            c->tile_ord_cap = npad;
        }
        c->tile_ident.resize(npad);
        for (size_t i = 0; i < npad; i++) c->tile_ident[i] = (int)i;
        if (npad) {
            HIP_TRY(c, hipMemcpyAsync(c->tile_order, c->tile_ident.data(), npad * 4, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemsetAsync(c->tile_cost, 0, npad * 4, c->stream));
        }
        c->tiles_px = tile_px;
        c->tiles_seen = c->tiles_ver;
        c->frames_since_order = 0;
    }
    return RV_OK;
}

rv_status rv_frame_tiles(rv_ctx* c, const rv_camera* cam, const float* vp16, const float* pvp16, float time,
                         float jx, float jy, int32_t flags, const int32_t* tile_ids, int32_t ntiles,
                         int32_t tile_px) {
    if (!c || !cam || (ntiles > 0 && !tile_ids) || ntiles < 0) return RV_ERR_INVALID;
    if (tile_px < 16 || (tile_px & 15)) return fail(c, RV_ERR_INVALID, "tile_px must be a multiple of 16");
    if (!c->world_ready) return fail(c, RV_ERR_STATE, "rv_frame_tiles before world");
    int tiles_x = (c->cfg.width + tile_px - 1) / tile_px;
    int tiles_y = (c->cfg.height + tile_px - 1) / tile_px;
    for (int i = 0; i < ntiles; i++)
        if (tile_ids[i] < 0 || tile_ids[i] >= tiles_x * tiles_y) return fail(c, RV_ERR_INVALID, "tile id out of range");
    size_t need = (size_t)ntiles * tile_px * tile_px * 4;
    if (!c->ext_tilebuf && need > c->tilebuf_bytes) {
        hipFree(c->tilebuf);
        c->tilebuf = nullptr;
        HIP_TRY(c, hipMalloc(&c->tilebuf, need));
        c->tilebuf_bytes = need;
    }
    if (c->ext_tilebuf && need > c->ext_tilebuf_bytes) return fail(c, RV_ERR_INVALID, "bound tile buffer too small");
    if (rv_status bs = begin_frame(c)) return bs;
    if (rv_status ts = tile_list(c, tile_ids, ntiles, tile_px)) return ts;
    FrameParams f = make_params(c, cam, vp16, pvp16, time, jx, jy, flags);
    f.tiles = c->tiles.d; f.ntiles = ntiles; f.tile_px = tile_px; f.tiles_x = tiles_x;
    f.tilebuf = c->ext_tilebuf ? c->ext_tilebuf : c->tilebuf;
    f.chunk_order[CG_RENDER] = c->tile_order; f.chunk_cost[CG_RENDER] = c->tile_cost;
    if (rv_status rs = run_stages(c, f, true)) return rs;
    return end_frame(c);
}

rv_status rv_tile_buffer(rv_ctx* c, void** p, size_t* bytes) {
    if (!c || !p) return RV_ERR_INVALID;
    *p = c->ext_tilebuf ? c->ext_tilebuf : c->tilebuf;
    if (bytes) *bytes = c->ext_tilebuf ? c->ext_tilebuf_bytes : c->tilebuf_bytes;
    return RV_OK;
}

rv_status rv_bind_tile_buffer(rv_ctx* c, void* p, size_t bytes) {
    if (!c) return RV_ERR_INVALID;
    c->ext_tilebuf = (uint32_t*)p;
    c->ext_tilebuf_bytes = p ? bytes : 0;
    return RV_OK;
}

rv_status rv_timing_enable(rv_ctx* c, int32_t max_frames) {
    if (!c || max_frames < 0) return RV_ERR_INVALID;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (hipEvent_t e : c->ev) hipEventDestroy(e);
    c->ev.clear();
    c->timing_cap = 0; c->timing_n = 0;
    c->ev.resize((size_t)max_frames * EV_PER_FRAME);
    c->gi_timed.assign((size_t)max_frames, 0);
    c->ev_stage.assign((size_t)max_frames * EV_PER_FRAME, -1);
    c->ev_used.assign((size_t)max_frames, 0);
    for (auto& e : c->ev) HIP_TRY(c, hipEventCreate(&e));
    c->timing_cap = max_frames;
    return RV_OK;
}

rv_status rv_timing_stages(rv_ctx* c, double* ms, int32_t n, int32_t* frames) {
    if (!c || !ms || n < 0) return RV_ERR_INVALID;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < n; k++) ms[k] = 0.0;
    for (int i = 0; i < c->timing_n; i++) {
        const size_t e0 = (size_t)EV_PER_FRAME * i;
        hipEvent_t* e = &c->ev[e0];
        for (int j = 0; j + 1 < c->ev_used[i]; j++) {
            const int k = c->ev_stage[e0 + j];
            float t = 0.0f;
            HIP_TRY(c, hipEventElapsedTime(&t, e[j], e[j + 1]));
            if (k >= 0 && k < n) ms[k] += t;
        }
        if (c->gi_timed[i] && ST_GI < n) {
            float t = 0.0f;
            HIP_TRY(c, hipEventElapsedTime(&t, e[NSTAGE], e[NSTAGE + 1]));
            ms[ST_GI] += t;
        }
    }
    if (frames) *frames = c->timing_n;
    return RV_OK;
}

rv_status rv_timing_launches(rv_ctx* c, int32_t* counts, int32_t n) {
    if (!c || !counts || n < 0) return RV_ERR_INVALID;
    for (int k = 0; k < n; k++) counts[k] = 0;
    for (int i = 0; i < c->timing_n; i++) {
        const size_t e0 = (size_t)EV_PER_FRAME * i;
        for (int j = 0; j + 1 < c->ev_used[i]; j++) {
            const int k = c->ev_stage[e0 + j];
            if (k >= 0 && k < n) counts[k]++;
        }
        if (c->gi_timed[i] && ST_GI < n) counts[ST_GI]++;
    }
    return RV_OK;
}

rv_status rv_timing_get(rv_ctx* c, double ms[3], int32_t* frames) {
    if (!c || !ms) return RV_ERR_INVALID;
    double st[NSTAGE];
    rv_status s = rv_timing_stages(c, st, NSTAGE, frames);
    if (s != RV_OK) return s;
    ms[0] = st[ST_GI];
    ms[1] = st[ST_PP_PRIMARY] + st[ST_PP_SHADOW];
    ms[2] = st[ST_PRIMARY] + st[ST_SHADOW] + st[ST_WATER] + st[ST_CONES] + st[ST_SHADE];
    return RV_OK;
}

rv_status rv_untile(rv_ctx* c, const void* dev_tiles, const int32_t* tile_ids, int32_t ntiles, int32_t tile_px) {
    if (!c || (ntiles > 0 && (!dev_tiles || !tile_ids)) || tile_px <= 0 || ntiles < 0) return RV_ERR_INVALID;
    int tiles_x = (c->cfg.width + tile_px - 1) / tile_px;
    int tiles_y = (c->cfg.height + tile_px - 1) / tile_px;
    for (int i = 0; i < ntiles; i++)
        if (tile_ids[i] < -1 || tile_ids[i] >= tiles_x * tiles_y) return fail(c, RV_ERR_INVALID, "tile id out of range");
    rv_status us = upload_ids(c, c->untile_ids, tile_ids, ntiles, nullptr);
    if (us != RV_OK) return us;
    launch_untile(c->stream, (const uint32_t*)dev_tiles, c->untile_ids.d, ntiles, tile_px, tiles_x, c->cfg.width,
                  c->cfg.height, c->color, c->color_pitch);
    LAUNCH_CHECK(c);
    return end_frame(c);   // the assembled frame is part of this slot's work
}

rv_status rv_bind_output(rv_ctx* c, int32_t kind, void* p, size_t pitch) {
    if (!c) return RV_ERR_INVALID;
    size_t W = (size_t)c->cfg.width;
    // the frame kernels address an image with a 32-bit byte offset from its base
    if (p && (uint64_t)pitch * (uint64_t)c->cfg.height >= (1ull << 32))
        return fail(c, RV_ERR_INVALID, "image larger than 4 GiB (pitch x height)");
    switch (kind) {
    case RV_IMAGE_COLOR:
        if (p && pitch < W * 4) return fail(c, RV_ERR_INVALID, "pitch too small");
        c->color = p ? (uint32_t*)p : c->own_color;
        c->color_pitch = p ? pitch : c->own_color_pitch;
        c->color_ext = p != nullptr;
        return RV_OK;
    case RV_IMAGE_MOTION:
        if (p && pitch < W * 4) return fail(c, RV_ERR_INVALID, "pitch too small");
        c->mv = p ? (uint32_t*)p : c->own_mv;
        c->mv_pitch = p ? pitch : c->own_mv_pitch;
        c->mv_ext = p != nullptr;
        return RV_OK;
    case RV_IMAGE_DEPTH:
        if (p && pitch < W * 2) return fail(c, RV_ERR_INVALID, "pitch too small");
        c->depth = p ? (uint16_t*)p : c->own_depth;
        c->depth_pitch = p ? pitch : c->own_depth_pitch;
        c->depth_ext = p != nullptr;
        return RV_OK;
    default:
        return fail(c, RV_ERR_INVALID, "bad image kind");
    }
}

static rv_status image_desc(rv_ctx* c, int32_t kind, void** p, size_t* pitch, size_t* row_bytes, int* rows) {
    int W = c->cfg.width, H = c->cfg.height;
    switch (kind) {
    case RV_IMAGE_COLOR: *p = c->color; *pitch = c->color_pitch; *row_bytes = (size_t)W * 4; *rows = H; return RV_OK;
    case RV_IMAGE_MOTION: *p = c->mv; *pitch = c->mv_pitch; *row_bytes = (size_t)W * 4; *rows = H; return RV_OK;
    case RV_IMAGE_DEPTH: *p = c->depth; *pitch = c->depth_pitch; *row_bytes = (size_t)W * 2; *rows = H; return RV_OK;
    case RV_IMAGE_HALF_DIST:
        *p = c->hdist; *pitch = (size_t)(W / 2) * 4; *row_bytes = *pitch; *rows = H / 2; return RV_OK;
    case RV_IMAGE_HALF_SHADOW:
        *p = c->hshadow; *pitch = (size_t)(W / 2) * 4; *row_bytes = *pitch; *rows = H / 2; return RV_OK;
    default: return fail(c, RV_ERR_INVALID, "bad image kind");
    }
}

rv_status rv_image_ptr(rv_ctx* c, int32_t kind, void** p, size_t* pitch) {
    if (!c || !p) return RV_ERR_INVALID;
    size_t pt, rb; int rows;
    rv_status s = image_desc(c, kind, p, &pt, &rb, &rows);
    if (pitch) *pitch = pt;
    return s;
}

rv_status rv_readback(rv_ctx* c, int32_t kind, void* host, size_t pitch) {
    if (!c || !host) return RV_ERR_INVALID;
    void* p; size_t dp, rb; int rows;
    rv_status s = image_desc(c, kind, &p, &dp, &rb, &rows);
    if (s != RV_OK) return s;
    if (pitch == 0) pitch = rb;
    if (pitch < rb) return fail(c, RV_ERR_INVALID, "host pitch too small");
    if (c->slots.size() > 1 && c->slots[c->cur_slot].pending)   // the last frame's slot
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->slots[c->cur_slot].done, 0));
    HIP_TRY(c, hipMemcpy2DAsync(host, pitch, p, dp, rb, rows, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return RV_OK;
}

rv_status rv_trace_rays(rv_ctx* c, const float* org, const float* dir, const float* dist, int64_t n, rv_hit* out) {
    if (!c || n < 0 || (n > 0 && (!org || !dir || !dist || !out))) return RV_ERR_INVALID;
    if (n == 0) return RV_OK;
    float *d_o = nullptr, *d_d = nullptr, *d_t = nullptr;
    RvHitDev* d_h = nullptr;
    HIP_TRY(c, hipMalloc(&d_o, (size_t)n * 12));
    HIP_TRY(c, hipMalloc(&d_d, (size_t)n * 12));
    HIP_TRY(c, hipMalloc(&d_t, (size_t)n * 4));
    HIP_TRY(c, hipMalloc(&d_h, (size_t)n * sizeof(RvHitDev)));
    HIP_TRY(c, hipMemcpyAsync(d_o, org, (size_t)n * 12, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(d_d, dir, (size_t)n * 12, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(d_t, dist, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    World tw = current_world(c);
    tw.ytop = (uint32_t)tw.Y;   // rv_trace_rays reports the reference's step counts: no sky exit (and it
                                // traces no sun rays through trace_sun)
    launch_trace_rays(c->stream, tw, d_o, d_d, d_t, n, d_h);
    LAUNCH_CHECK(c);
    HIP_TRY(c, hipMemcpyAsync(out, d_h, (size_t)n * sizeof(RvHitDev), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    hipFree(d_o); hipFree(d_d); hipFree(d_t); hipFree(d_h);
    return RV_OK;
}

// Character::Update camera math (src/Character.cpp:18-126) for a static pose.
static f3 glm_norm(f3 v) {
    float d = v.x * v.x + v.y * v.y + v.z * v.z;
    float inv = 1.0f / sqrtf(d);
    return host_v(v.x * inv, v.y * inv, v.z * inv);
}
static f3 h_cross(f3 a, f3 b) {
    return host_v(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

rv_status rv_camera_from_pose(float px, float py, float pz, float yaw, float pitch, int32_t width, int32_t height,
                              rv_camera* cam, float* vp16) {
    if (!cam || width <= 0 || height <= 0) return RV_ERR_INVALID;
    const float pih = 3.14159265358979323846f * 0.5f;
    float s0 = sinf((float)(double)yaw), s1 = sinf((float)((double)yaw + (double)pih));
    float s2 = sinf((float)(double)pitch), s3 = sinf((float)((double)pitch + (double)pih));
    f3 dir = glm_norm(host_v(-s0 * -s3, -s2, -s1 * s3));
    f3 right = glm_norm(h_cross(dir, host_v(0.0f, 1.0f, 0.0f)));
    f3 up = glm_norm(h_cross(dir, right));
    std::memset(cam, 0, sizeof(*cam));
    cam->pos[0] = px; cam->pos[1] = py; cam->pos[2] = pz;
    cam->forward[0] = dir.x; cam->forward[1] = dir.y; cam->forward[2] = dir.z;
    cam->right[0] = right.x; cam->right[1] = right.y; cam->right[2] = right.z;
    cam->up[0] = up.x; cam->up[1] = up.y; cam->up[2] = up.z;
    float fov_factor = (float)tan(60.0f * 3.14159265358979323846 / 180.0);
    float aspect = (float)width / (float)height;
    cam->add[0] = aspect * -fov_factor; cam->add[1] = 1.0f * -fov_factor;
    cam->mul[0] = fov_factor * aspect * (2.0f / (float)width);
    cam->mul[1] = fov_factor * 1.0f * (2.0f / (float)height);
    if (vp16) {
        f3 eye = host_v(px, py, pz);
        f3 ctr = host_v(eye.x + dir.x, eye.y + dir.y, eye.z + dir.z);
        f3 f = glm_norm(host_v(ctr.x - eye.x, ctr.y - eye.y, ctr.z - eye.z));
        f3 s = glm_norm(h_cross(f, host_v(0.0f, 1.0f, 0.0f)));
        f3 u = h_cross(s, f);
        float view[16] = {0};
        view[0] = s.x; view[4] = s.y; view[8] = s.z;
        view[1] = u.x; view[5] = u.y; view[9] = u.z;
        view[2] = -f.x; view[6] = -f.y; view[10] = -f.z;
        view[12] = -(s.x * eye.x + s.y * eye.y + s.z * eye.z);
        view[13] = -(u.x * eye.x + u.y * eye.y + u.z * eye.z);
        view[14] = f.x * eye.x + f.y * eye.y + f.z * eye.z;
        view[15] = 1.0f;
        float fovy = 60.0f * 0.01745329251994329576923690768489f;
        float zn = 0.1f, zf = 50000.0f;
        float th = tanf(fovy / 2.0f);
        float proj[16] = {0};
        proj[0] = 1.0f / (aspect * th);
        proj[5] = 1.0f / th;
        proj[10] = -(zf + zn) / (zf - zn);
        proj[11] = -1.0f;
        proj[14] = -(2.0f * zf * zn) / (zf - zn);
        for (int col = 0; col < 4; col++)
            for (int r = 0; r < 4; r++)
                vp16[col * 4 + r] = proj[0 * 4 + r] * view[col * 4 + 0] + proj[1 * 4 + r] * view[col * 4 + 1] +
                                    proj[2 * 4 + r] * view[col * 4 + 2] + proj[3 * 4 + r] * view[col * 4 + 3];
    }
    return RV_OK;
}

// counters: one block of NCNT per frame stage (ST_*), -1 = their sum
rv_status rv_stats_stage(rv_ctx* c, int32_t stage, rv_stats* out) {
    if (!c || !out || stage < -1 || stage >= NSTAGE) return RV_ERR_INVALID;
    std::vector<unsigned long long> h((size_t)NSTAGE * NCNT);
    HIP_TRY(c, hipMemcpyAsync(h.data(), c->counters, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    static_assert(sizeof(rv_stats) == NCNT * 8, "rv_stats layout");
    unsigned long long r[NCNT] = {};
    for (int s = 0; s < NSTAGE; s++)
        if (stage < 0 || s == stage)
            for (int k = 0; k < NCNT; k++) r[k] += h[(size_t)s * NCNT + k];
    std::memcpy(out, r, sizeof(r));
    return RV_OK;
}

rv_status rv_stats_get(rv_ctx* c, rv_stats* out) { return rv_stats_stage(c, -1, out); }

rv_status rv_stats_reset(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    HIP_TRY(c, hipMemsetAsync(c->counters, 0, NSTAGE * NCNT * sizeof(unsigned long long), c->stream));
    return RV_OK;
}

}  // extern "C"
