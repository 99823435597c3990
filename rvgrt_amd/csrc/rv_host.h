// rv_host.h -- internal to librvgrt_hip.so (not installed): the context (rv_ctx), the communicator and
// the host helpers shared by the three parts of the C ABI declared in include/rvgrt.h --
//   rv_abi.cpp    contexts, world build / import / export, the GI update, single frames (flow frames,
//                 drawCUDA), readback, stats;
//   rv_loops.cpp  the native frame loops (batched, pipelined, grouped), tile shards;
//   rv_comm.cpp   the transport: RCCL resolved at run time, or the in-process loopback group.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types only: RCCL is resolved at run time (rccl_load)

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <tuple>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rvgrt/rv_frame.h"
#ifndef RV_PIPE_DIAG
#define RV_PIPE_DIAG 0   // per-wave diagnostics of the pipelined and flow launches (tools/pipe_waves.py, tools/flow_waves.py)
#endif

using namespace rv;


// Device copy of a host id list, uploaded only when the list changes.
struct DevIds {
    int* d = nullptr;
    size_t cap = 0;
    std::vector<int32_t> h;
};

// Per-frame resources of one frame in flight (rv_set_frames_in_flight): the
// library-owned output images, the half-res pre-pass images and the
// SCHED_COST order/cost arrays.  The active slot's pointers live in rv_ctx's
// own fields (slot_load/slot_save swap them), so single-slot code paths read
// exactly what they did before.
struct FrameSlot {
    uint32_t* own_color = nullptr; uint32_t* own_mv = nullptr; uint16_t* own_depth = nullptr;
    float* hdist = nullptr; float* hshadow = nullptr;
    int* chunk_order[2] = {nullptr, nullptr}; uint32_t* chunk_cost[2] = {nullptr, nullptr};
    int* tile_order = nullptr; uint32_t* tile_cost = nullptr; size_t tile_ord_cap = 0;
    int tiles_px = 0; uint32_t frames_since_order = 0;
    uint64_t tiles_seen = ~0ull;
    hipEvent_t done = nullptr;    // recorded after the slot's last frame work
    bool pending = false;         // `done` has been recorded at least once
    hipStream_t last_stream = nullptr;   // stream of the slot's last frame
    uint64_t submitted = 0;       // frame_seq of the slot's last frame
    uint64_t world_seen = 0;      // world version the slot's last frame waited for
    // rv_render_frames with a tile shard: packed tiles, rank-0 gather buffer
    uint32_t* tbuf = nullptr; size_t tbytes = 0;
    uint32_t* gbuf = nullptr; size_t gbytes = 0;
    hipEvent_t gathered = nullptr;      // recorded on the comm stream after the slot's gather
};

// rv_render_frames batches: B frames per launch, two sets in ping-pong (set
// j & 1 also uses frame slot j & 1's scheduling state).
struct BatchSet {
    uint32_t* color = nullptr; uint32_t* mv = nullptr; uint16_t* depth = nullptr;
    float* hdist = nullptr; float* hshadow = nullptr;
    uint32_t* tbuf = nullptr; uint32_t* gbuf = nullptr;
    int nb = 0; size_t slice = 0, gbytes = 0;   // allocated for
    hipEvent_t rendered = nullptr, gathered = nullptr;
    bool pending = false;
};

struct rv_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    rv_config cfg{};
    int lx = 0, ly = 0, lz = 0;
    World w{};
    uint32_t* d_top = nullptr;     // world_top scratch (one dword)
    uint32_t* coltop = nullptr;    // sun horizon: highest solid row + 1 per brick column
    uint32_t* brick = nullptr;
    size_t brick_bytes = 0;
    uint32_t* gi = nullptr;       // current grid
    uint32_t* gi_tmp = nullptr;   // update target (double buffer)
    size_t gi_bytes = 0;
    uint32_t* atlas = nullptr;
    uint32_t* tex = nullptr;      // sampleTexture's tile table (World::tex), or null
    bool tex_tried = false;       // tex_table() ran (the table is built once per context)
    // frame images (library-owned unless bound)
    uint32_t* color = nullptr; size_t color_pitch = 0; bool color_ext = false;
    uint32_t* mv = nullptr; size_t mv_pitch = 0; bool mv_ext = false;
    uint16_t* depth = nullptr; size_t depth_pitch = 0; bool depth_ext = false;
    uint32_t* own_color = nullptr; uint32_t* own_mv = nullptr; uint16_t* own_depth = nullptr;
    size_t own_color_pitch = 0, own_mv_pitch = 0, own_depth_pitch = 0;
    float* hdist = nullptr;
    float* hshadow = nullptr;
    unsigned long long* counters = nullptr;
    DevIds tiles;                 // rv_frame_tiles list (device copy, re-uploaded on change)
    DevIds untile_ids;            // rv_untile list
    int tiles_px = 0;             // tile size of the cached list (active slot)
    uint64_t tiles_ver = 0;       // bumped when the device tile list changes
    uint64_t tiles_seen = ~0ull;  // list version the active slot's order arrays are for
    std::vector<int> tile_ident;
    int* tile_order = nullptr; uint32_t* tile_cost = nullptr; size_t tile_ord_cap = 0;   // SCHED_COST per tile slot
    uint32_t* tilebuf = nullptr; size_t tilebuf_bytes = 0;
    uint32_t* ext_tilebuf = nullptr; size_t ext_tilebuf_bytes = 0;
    // stage timing (rv_timing_enable): EV_PER_FRAME events per frame
    int timing_cap = 0, timing_n = 0;
    std::vector<hipEvent_t> ev;
    std::vector<char> gi_timed;
    std::vector<signed char> ev_stage;   // stage of each frame event slot (-1: end of frame)
    std::vector<int> ev_used;            // frame event slots used per frame
    bool megakernel = true;       // RV_PATH_FUSED (k_prepass/k_render); false: wavefront stages
    // asynchronous GI update (rv_set_gi_async): kernel on gi_stream, copy-back on stream
    bool gi_async = true;
    hipStream_t gi_stream = nullptr;
    int prio_lo = 0, prio_hi = 0;  // stream priority range (numerically: lo = least urgent)
    int gi_low_prio = 1;           // 1 = GI stream at the lowest priority (fills the frame's gaps)
    hipEvent_t ev_world = nullptr;    // recorded on `stream` after the last world/GI write
    hipEvent_t ev_gi_done = nullptr;  // recorded on gi_stream after a GI kernel
    int enq = 1;                  // wavefront path: queue append granularity (FrameParams::enq)
    // wavefront buffers
    float4* hpos = nullptr; uint32_t* hinfo = nullptr; float4* hsec = nullptr; float4* pphit = nullptr;
    int* wq[NQUEUE] = {nullptr, nullptr, nullptr, nullptr};
    size_t wq_cap[NQUEUE] = {0, 0, 0, 0};   // items allocated per queue (all sub-queues)
    unsigned* qcount = nullptr;
    uint32_t* wtrace = nullptr;   // RV_WAVE_TRACE builds: per-wave records of the last k_render
    size_t wtrace_bytes = 0;
    uint32_t gi_frame = 0;
    uint64_t gi_offset = 0;
    bool world_ready = false;
    int sched = SCHED_COST;
    int order_every = 4;          // frames between chunk re-orderings
    int pipe = 1;                 // rv_set_pipeline: pipelined reference frames
    uint32_t pipe_order = 0x102;  // RV_OPT_PIPE_ORDER: dispatch order, hex digits PIPE_* (first = high): pre-pass, GI, render
    float* pipe_half[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};   // [k & 1] {dist, shadow}
    bool gi_stats = false;        // rv_set_gi_stats
    // pipelined tile loop: packed tiles / rank-0 gather buffers per frame parity, GI shard staging
    uint32_t* pipe_tbuf[2] = {nullptr, nullptr}; uint32_t* pipe_gbuf[2] = {nullptr, nullptr};
    size_t pipe_slice = 0, pipe_gbytes = 0;
    uint32_t* pipe_gi_stage = nullptr; uint32_t* pipe_gi_all = nullptr;
    uint64_t pipe_chunk = 0; int pipe_chunk_n = 0;
    hipEvent_t pipe_ev[4] = {nullptr, nullptr, nullptr, nullptr};   // rendered, all-gathered, gathered[2]
    uint32_t* pipe_wstat = nullptr;   // env RV_PIPE_WAVE_STATS: per-wave records of the first launches
    // env RV_FLOW_WAVE_TRACE=<file> (RV_PIPE_DIAG builds): the last flow launch's per-wave records, dumped at
    // rv_destroy (tools/flow_waves.py)
    uint32_t* flow_wtrace = nullptr; uint32_t flow_wtrace_n = 0, flow_wlen[3] = {0, 0, 0};
    uint32_t pipe_launches = 0;
    uint32_t pipe_wnb[64] = {};       // workgroups of each recorded launch
    int gather_bpp = 3;           // rv_set_gather_bpp: packed pixel bytes of rv_render_frames' tile gather (3 or 4)
    uint32_t frames_since_order = 0;
    int* chunk_order[2] = {nullptr, nullptr};      // SCHED_COST feedback per grid (CG_*)
    uint32_t* chunk_cost[2] = {nullptr, nullptr};
    std::vector<FrameSlot> slots;  // frames in flight; slots[cur_slot] mirrors the fields above
    std::vector<hipStream_t> fstreams;   // rv_render_frames: streams of slots 1..n-1 (slot 0: `stream`)
    int fstream_prio = 0;
    hipStream_t comm_stream = nullptr;   // rv_render_frames: RCCL gathers, in frame order
    hipEvent_t ev_loop = nullptr;        // scratch event of rv_render_frames
    BatchSet bsets[2];
    int batch_streams = 1;               // RV_OPT_BATCH_STREAMS: streams rv_render_frames' groups alternate over
    // rv_set_tile_shard: this rank's tiles and the gathered layout (rank 0)
    int shard_px = 0, shard_rank = 0, shard_n = 0, shard_max = 0;
    std::vector<int32_t> shard_ids, shard_all;
    uint64_t world_ver = 1;        // bumped by every world/GI write (mark_world)
    uint64_t geom_ver = 1;         // bumped by every voxel-bits / CSDF write (what the pre-pass reads)
    // Pipelined loop: the next frame's GI update and pre-pass computed by the last launch of a call and
    // kept for the next call (rv_render_frame_seq).  gi: update `carry_fr` of [carry_first, +count) in
    // gi_tmp (or this rank's shard in pipe_gi_stage), not yet copied back; pp: pre-pass of the camera
    // `carry_key` in pipe_half[carry_half].
    bool carry_gi = false, carry_pp = false;
    uint32_t carry_fr = 0; uint64_t carry_first = 0, carry_count = 0, carry_world = 0, carry_geom = 0;
    uint64_t carry_chunk = 0; int carry_n = 0, carry_r = 0, carry_half = 0;
    float carry_key[24] = {};
    int pipe_carry = 1;            // the next frame's GI update and pre-pass are kept between calls
    // Flow frames (rv_set_flow; rv_frame / rv_draw_cuda of a frame with the pre-pass): one k_ref_flow
    // launch per frame.  Tile-major half-res hand-off buffer, per-tile flags, the launch epoch and the
    // count of render waves that fell back to evaluating their window.
    int flow = 1;
    unsigned long long* flow_half = nullptr; size_t flow_tiles = 0;
    uint32_t flow_epoch = 0;
    unsigned long long* flow_fb = nullptr;
    hipEvent_t ev_flow = nullptr;   // recorded after every flow launch, on the stream it ran on
    uint64_t flow_launches = 0;
    // RV_OPT_GI_PAIRS: latency-variant launches trace a GI cell's two rays on a lane pair (1 all, 0 none);
    // default -1: a rank's tile share only -- its GI part is 1/N of the cells and its longest GI waves
    // were the launch's floor (8-rank C4 share 137.4 -> 132.8 us/frame, GI longest wave 127.5 -> 98.9 us),
    // while a whole C3 frame's GI waves double for no gain (0.204 -> 0.240 ms; profiles/r04/gi_pairs_ab.txt)
    int gi_pairs = -1;
    uint32_t flow_spin = 16384;      // RV_OPT_FLOW_SPIN: polls before a render wave evaluates its window
    bool flow_force_fallback = false;   // RV_OPT_FLOW_FORCE_FALLBACK (tests): no wave waits, all evaluate
    bool gi_shard_probe = false;     // RV_OPT_GI_SHARD_PROBE: a sharded loop without a communicator runs its 1/N GI share
    // The next UpdateGIData computed ahead by a flow launch (camera-independent): update `spec_fr` of
    // [spec_first, + spec_count) in gi_tmp, valid while the world/GI version is spec_world; recorded
    // on the launch's stream (ev_spec).  upd_since_frame: an UpdateGIData came since the last frame
    // (the caller runs renderLoop's per-frame update, so the next one is worth computing ahead).
    bool spec_gi = false;
    uint32_t spec_fr = 0; uint64_t spec_first = 0, spec_count = 0, spec_world = 0;
    hipEvent_t ev_spec = nullptr; hipStream_t spec_stream = nullptr; bool spec_rec = false;
    bool upd_since_frame = false;
    // grouped reference frames (rv_set_frame_group): frame sets per group parity, phase-A records
    // (this rank's stage slots and the all-gathered ones, 3 groups each), the update ring, the
    // phase-B stream and the loop's events
    int group = 0;
    BatchSet gsets[2];
    uint2* grec_stage = nullptr; uint2* grec_all = nullptr; size_t grec_stage_n = 0, grec_all_n = 0;
    uint32_t* gring = nullptr; size_t gring_n = 0;
    hipStream_t grp_stream = nullptr;
    hipEvent_t gev[8] = {};
    rv_comm* comm_attached = nullptr;   // the communicator of the last rv_render_frame_seq (bounded rv_sync)
    float shard_w0 = 1.0f;              // rank 0's tile weight of the shard (rv_set_tile_shard_weighted)
    // per-frame camera table of batched launches (rv_render_frame_seq): device copy, pinned staging
    FrameCam* cam_dev = nullptr; FrameCam* cam_host = nullptr; size_t cam_cap = 0;
    hipEvent_t cam_ev = nullptr; bool cam_pending = false;
    uint64_t gi_swapped_at = 0;    // frame_seq at the last GI buffer flip: older frames read gi_tmp
    hipStream_t world_stream = nullptr;   // stream ev_world was recorded on
    int cur_slot = 0;
    uint64_t frame_seq = 0;
    std::string err;
};

// ---------------------------------------------------------------- transport
// Everything the loops exchange goes through four operations on a
// communicator: an all-gather (the GI update's cells) and grouped
// send/recv (packed tiles to rank 0).  Two backends:
//   RCCL     -- one process per GPU over xGMI (ncclAllGather / ncclSend /
//               ncclRecv inside ncclGroupStart/End);
//   loopback -- N contexts of one process (one GPU): each rank's host thread
//               posts its side of an operation, the group meets at a host
//               barrier, and every rank enqueues on its own stream the
//               device-to-device copies that fetch what it receives, after
//               the senders' ready events; a second barrier lets every rank
//               wait for the copies that read its buffers.  It runs the real
//               multi-rank code paths (shard slices, padded deals, RGB24
//               packing, GI all-gather) without N GPUs.
// Waits are bounded (rv_comm_wait): a dead or diverged peer is an error
// after a timeout, the communicator is aborted.
struct LoopGroup {
    struct Post {
        int kind = 0;                   // 1 all-gather, 2 grouped send/recv
        const void* send = nullptr; void* recv = nullptr; size_t bytes = 0;
        std::vector<std::tuple<int, int, const void*, void*, size_t>> p2p;   // (is_send, peer, sbuf, rbuf, bytes)
        hipEvent_t ready = nullptr, done = nullptr;
    };
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    uint64_t gen = 0;                   // barrier generation
    int arrived = 0;
    bool aborted = false;
    std::vector<Post> post;
    double timeout_s = 60.0;
    // the barrier all ranks of a round pass twice; false on timeout or abort
    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::duration<double>(timeout_s),
                                    [&] { return gen != g || aborted; });
        if (!ok || aborted) { aborted = true; cv.notify_all(); return false; }
        return true;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
};

struct rv_comm {
    ncclComm_t comm = nullptr;   // RCCL backend
    LoopGroup* loop = nullptr;   // loopback backend (not owned)
    int rank = 0, nranks = 1, device = 0;
    rv_ctx* ctx = nullptr;       // the context it was created with (bounded waits, rv_comm_destroy)
    bool in_group = false;
    LoopGroup::Post pending;     // loopback: the ops of the open group
    hipEvent_t ready = nullptr, done = nullptr;
    uint64_t verified = 0;       // config record the ranks last agreed on (shard / bpp)
    bool aborted = false;
    // verify_ranks' exchange buffers, allocated on first use and kept: (nranks + 1) x 8 B on the device
    // (the all-gather's output, then this rank's hash), nranks x 8 B pinned on the host
    uint64_t* vdev = nullptr;
    uint64_t* vhost = nullptr;
};


// ---------------------------------------------------------------- helpers

inline int gi_prio(const rv_ctx* c) { return c->gi_low_prio ? c->prio_lo : c->prio_hi; }

inline rv_status fail(rv_ctx* c, rv_status s, const std::string& msg) {
    if (c) c->err = msg;
    return s;
}

#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail((ctx), e_ == hipErrorOutOfMemory ? RV_ERR_OOM : RV_ERR_HIP,          \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                  \
    } while (0)

#define LAUNCH_CHECK(ctx) HIP_TRY(ctx, hipGetLastError())

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

inline void slot_save(rv_ctx* c) {
    FrameSlot& sl = c->slots[c->cur_slot];
    sl.own_color = c->own_color; sl.own_mv = c->own_mv; sl.own_depth = c->own_depth;
    sl.hdist = c->hdist; sl.hshadow = c->hshadow;
    for (int g = 0; g < 2; g++) { sl.chunk_order[g] = c->chunk_order[g]; sl.chunk_cost[g] = c->chunk_cost[g]; }
    sl.tile_order = c->tile_order; sl.tile_cost = c->tile_cost; sl.tile_ord_cap = c->tile_ord_cap;
    sl.tiles_px = c->tiles_px; sl.frames_since_order = c->frames_since_order;
    sl.tiles_seen = c->tiles_seen;
}

inline void slot_load(rv_ctx* c, int s) {
    const FrameSlot& sl = c->slots[s];
    c->cur_slot = s;
    c->own_color = sl.own_color; c->own_mv = sl.own_mv; c->own_depth = sl.own_depth;
    if (!c->color_ext) c->color = sl.own_color;
    if (!c->mv_ext) c->mv = sl.own_mv;
    if (!c->depth_ext) c->depth = sl.own_depth;
    c->hdist = sl.hdist; c->hshadow = sl.hshadow;
    for (int g = 0; g < 2; g++) { c->chunk_order[g] = sl.chunk_order[g]; c->chunk_cost[g] = sl.chunk_cost[g]; }
    c->tile_order = sl.tile_order; c->tile_cost = sl.tile_cost; c->tile_ord_cap = sl.tile_ord_cap;
    c->tiles_px = sl.tiles_px; c->frames_since_order = sl.frames_since_order;
    c->tiles_seen = sl.tiles_seen;
}

// Images (rows padded to 256 B like a D3D12 placed footprint), half-res
// pre-pass images, identity chunk orders and zero costs of one slot.
inline bool slot_alloc(rv_ctx* c, FrameSlot& sl) {
    const int W = c->cfg.width, H = c->cfg.height;
    const size_t hbytes = (size_t)(W / 2) * (H / 2) * 4;
    if (hipMalloc(&sl.own_color, c->own_color_pitch * H) != hipSuccess ||
        hipMalloc(&sl.own_mv, c->own_mv_pitch * H) != hipSuccess ||
        hipMalloc(&sl.own_depth, c->own_depth_pitch * H) != hipSuccess ||
        hipMalloc(&sl.hdist, hbytes) != hipSuccess || hipMalloc(&sl.hshadow, hbytes) != hipSuccess)
        return false;
    hipMemset(sl.own_color, 0, c->own_color_pitch * H);
    hipMemset(sl.own_mv, 0, c->own_mv_pitch * H);
    hipMemset(sl.own_depth, 0, c->own_depth_pitch * H);
    hipMemset(sl.hdist, 0, hbytes);
    hipMemset(sl.hshadow, 0, hbytes);
    const uint32_t nb[2][2] = {{(uint32_t)(W / 2), (uint32_t)(H / 2)}, {(uint32_t)W, (uint32_t)H}};
    for (int g = 0; g < 2; g++) {
        uint32_t npad = n_chunks_pad(nb[g][0], nb[g][1]);
        std::vector<int> id(npad);
        for (uint32_t i = 0; i < npad; i++) id[i] = (int)i;
        if (hipMalloc(&sl.chunk_order[g], npad * 4) != hipSuccess || hipMalloc(&sl.chunk_cost[g], npad * 4) != hipSuccess)
            return false;
        hipMemcpy(sl.chunk_order[g], id.data(), npad * 4, hipMemcpyHostToDevice);
        hipMemset(sl.chunk_cost[g], 0, npad * 4);
    }
    return hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&sl.gathered, hipEventDisableTiming) == hipSuccess;
}

inline void slot_free(FrameSlot& sl) {
    hipFree(sl.own_color); hipFree(sl.own_mv); hipFree(sl.own_depth);
    hipFree(sl.hdist); hipFree(sl.hshadow);
    for (int g = 0; g < 2; g++) { hipFree(sl.chunk_order[g]); hipFree(sl.chunk_cost[g]); }
    hipFree(sl.tile_order); hipFree(sl.tile_cost);
    hipFree(sl.tbuf); hipFree(sl.gbuf);
    if (sl.done) hipEventDestroy(sl.done);
    if (sl.gathered) hipEventDestroy(sl.gathered);
    sl = FrameSlot{};
}

// per frame: [0, NSTAGE-1) start of each frame stage, [NSTAGE-1] end of the
// frame, [NSTAGE] / [NSTAGE+1] start / end of the GI update before it
constexpr int EV_PER_FRAME = NSTAGE + 2;

inline uint64_t n_gi(const rv_ctx* c) { return (uint64_t)c->w.GX * c->w.GY * c->w.GZ; }
inline uint64_t n_csdf(const rv_ctx* c) { return (uint64_t)c->w.SX * c->w.SY * c->w.SZ; }
inline uint64_t n_bits_words(const rv_ctx* c) { return ((uint64_t)c->w.X * c->w.Y * c->w.Z) >> 5; }

inline f3 host_v(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }

// glm::normalize(vec3(10,5,-4)) (src/StateRender.cu:299, src/CoarseArray.cu:359)
inline f3 sun_dir() {
    float d = 10.0f * 10.0f + 5.0f * 5.0f + (-4.0f) * (-4.0f);
    float inv = 1.0f / sqrtf(d);
    return host_v(10.0f * inv, 5.0f * inv, -4.0f * inv);
}

inline World current_world(const rv_ctx* c) {
    World w = c->w;
    world_set_brick(w, c->brick);
    w.gi = c->gi;
    w.atlas = c->atlas;
    return w;
}



// A frame sequence: desc k = d[k * stride] (stride 0: one camera for every
// frame); after() = the frame that follows the sequence.
struct Seq {
    const rv_frame_desc* d = nullptr;
    int stride = 0, n = 0;
    const rv_frame_desc* next = nullptr;
    const rv_frame_desc& at(int k) const { return d[(size_t)k * stride]; }
    const rv_frame_desc& after() const { return next ? *next : at(n - 1); }
    bool uniform(int k0, int k1) const {   // frames [k0, k1) share one camera
        if (stride == 0) return true;
        for (int k = k0 + 1; k < k1; k++)
            if (std::memcmp(&at(k), &at(k0), sizeof(rv_frame_desc)) != 0) return false;
        return true;
    }
};


// ---------------------------------------------------------------- shared between the parts
// Not exported from the library (hidden visibility).
#define RV_HIDDEN __attribute__((visibility("hidden")))

// rv_abi.cpp (C linkage: defined inside its extern "C" block)
extern "C" {
RV_HIDDEN rv_status end_frame(rv_ctx* c);
RV_HIDDEN rv_status wait_all_frames(rv_ctx* c);   // every frame in flight and the last world/GI write
RV_HIDDEN rv_status mark_world(rv_ctx* c);        // a world/GI write: versions bumped, ev_world recorded
RV_HIDDEN rv_status upload_ids(rv_ctx* c, DevIds& ids, const int32_t* src, int n, bool* changed);
RV_HIDDEN FrameParams make_params_d(rv_ctx* c, const rv_frame_desc& d, int32_t flags);
RV_HIDDEN rv_status upload_cams(rv_ctx* c, const Seq& q, hipStream_t st, const FrameCam** out,
                                const std::function<void(int, FrameCam&)>& fill = nullptr);
RV_HIDDEN rv_status run_stages(rv_ctx* c, FrameParams f, bool tiles, int which = 3);
RV_HIDDEN rv_status tile_list(rv_ctx* c, const int32_t* tile_ids, int32_t ntiles, int32_t tile_px);
}

// rv_comm.cpp: the four exchange operations of the loops and the bounded wait
RV_HIDDEN double comm_timeout_s();
RV_HIDDEN void comm_detach(rv_comm* m);
RV_HIDDEN rv_status comm_wait_bounded(rv_ctx* c, rv_comm* m, double timeout_s);
RV_HIDDEN rv_status comm_all_gather(rv_ctx* c, rv_comm* m, const void* send, void* recv, size_t bytes, hipStream_t s);
RV_HIDDEN rv_status comm_group_start(rv_ctx* c, rv_comm* m);
RV_HIDDEN rv_status comm_send(rv_ctx* c, rv_comm* m, const void* buf, size_t bytes, int peer, hipStream_t s);
RV_HIDDEN rv_status comm_recv(rv_ctx* c, rv_comm* m, void* buf, size_t bytes, int peer, hipStream_t s);
RV_HIDDEN rv_status comm_group_end(rv_ctx* c, rv_comm* m, hipStream_t s);
