// rv_abi.cpp -- host side of librvgrt_hip.so: the C ABI declared in
// include/rvgrt.h.  Owns device memory, the HIP stream and the GI update
// state; every entry point converts failures into rv_status + message.
#include <dlfcn.h>
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

static rv_status comm_wait_bounded(rv_ctx* c, rv_comm* m, double timeout_s);
static double comm_timeout_s();
static void comm_detach(rv_comm* m);

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
    int gi_low_prio = 1;           // RV_GI_PRIO: 1 = GI stream at the lowest priority (fills the frame's gaps)
    hipEvent_t ev_world = nullptr;    // recorded on `stream` after the last world/GI write
    hipEvent_t ev_gi_done = nullptr;  // recorded on gi_stream after a GI kernel
    int enq = 1;                  // RV_WF_ENQ: queue append granularity (FrameParams::enq)
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
    int order_every = 4;          // RV_ORDER_EVERY: frames between chunk re-orderings
    int pipe = 1;                 // rv_set_pipeline / RV_PIPE: pipelined reference frames
    uint32_t pipe_order = 0x102;  // RV_PIPE_ORDER: dispatch order, hex digits PIPE_* (first = high): pre-pass, GI, render
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
    int gather_bpp = 3;           // RV_GATHER_BPP: packed pixel bytes of rv_render_frames' tile gather (3 or 4)
    uint32_t frames_since_order = 0;
    int* chunk_order[2] = {nullptr, nullptr};      // SCHED_COST feedback per grid (CG_*)
    uint32_t* chunk_cost[2] = {nullptr, nullptr};
    std::vector<FrameSlot> slots;  // frames in flight; slots[cur_slot] mirrors the fields above
    std::vector<hipStream_t> fstreams;   // rv_render_frames: streams of slots 1..n-1 (slot 0: `stream`)
    int fstream_prio = 0;
    hipStream_t comm_stream = nullptr;   // rv_render_frames: RCCL gathers, in frame order
    hipEvent_t ev_loop = nullptr;        // scratch event of rv_render_frames
    BatchSet bsets[2];
    int batch_streams = 1;               // RV_BATCH_STREAMS: streams rv_render_frames' groups alternate over
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
    int pipe_carry = 1;            // RV_PIPE_CARRY
    // Flow frames (rv_set_flow; rv_frame / rv_draw_cuda of a frame with the pre-pass): one k_ref_flow
    // launch per frame.  Tile-major half-res hand-off buffer, per-tile flags, the launch epoch and the
    // count of render waves that fell back to evaluating their window.
    int flow = 1;
    unsigned long long* flow_half = nullptr; size_t flow_tiles = 0;
    uint32_t flow_epoch = 0;
    unsigned long long* flow_fb = nullptr;
    hipEvent_t ev_flow = nullptr;   // recorded after every flow launch, on the stream it ran on
    uint64_t flow_launches = 0;
    // env RV_GI_PAIRS: latency-variant launches trace a GI cell's two rays on a lane pair (1 all, 0 none);
    // default -1: a rank's tile share only -- its GI part is 1/N of the cells and its longest GI waves
    // were the launch's floor (8-rank C4 share 137.4 -> 132.8 us/frame, GI longest wave 127.5 -> 98.9 us),
    // while a whole C3 frame's GI waves double for no gain (0.204 -> 0.240 ms; profiles/r04/gi_pairs_ab.txt)
    int gi_pairs = -1;
    uint32_t prio_blocks = 0;        // env RV_PRIO_BLOCKS: leading pipelined-launch workgroups per part at high issue priority
    uint32_t flow_spin = 16384;      // env RV_FLOW_SPIN: polls before a render wave evaluates its window
    bool flow_force_fallback = false;   // env RV_FLOW_FORCE_FALLBACK=1 (tests): no wave waits, all evaluate
    // env RV_FLOW_PP_ORDER: 1 (default) pre-pass tiles in the render's chunk order, so the tiles the first
    // render waves read are published first (C3 -2 %, C4 -0.2 %, render waves finding a tile unpublished
    // on arrival 330 -> 130 per C4 frame: profiles/r04/flow_ab.txt); 0 the pre-pass's own cost order
    uint32_t flow_pp_order = 1;
    // env RV_FLOW_GI_SIDE=1: the next UpdateGIData's cells of a flow frame run as their own GI kernel on the
    // low-priority GI stream beside the flow launch (which then holds pre-pass + render only) instead of as
    // the flow launch's GI part; same cells, same kernel body, consumed the same way (ev_spec)
    bool flow_gi_side = false;
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

namespace {

int gi_prio(const rv_ctx* c) { return c->gi_low_prio ? c->prio_lo : c->prio_hi; }

rv_status fail(rv_ctx* c, rv_status s, const std::string& msg) {
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

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

void slot_save(rv_ctx* c) {
    FrameSlot& sl = c->slots[c->cur_slot];
    sl.own_color = c->own_color; sl.own_mv = c->own_mv; sl.own_depth = c->own_depth;
    sl.hdist = c->hdist; sl.hshadow = c->hshadow;
    for (int g = 0; g < 2; g++) { sl.chunk_order[g] = c->chunk_order[g]; sl.chunk_cost[g] = c->chunk_cost[g]; }
    sl.tile_order = c->tile_order; sl.tile_cost = c->tile_cost; sl.tile_ord_cap = c->tile_ord_cap;
    sl.tiles_px = c->tiles_px; sl.frames_since_order = c->frames_since_order;
    sl.tiles_seen = c->tiles_seen;
}

void slot_load(rv_ctx* c, int s) {
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
bool slot_alloc(rv_ctx* c, FrameSlot& sl) {
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

void slot_free(FrameSlot& sl) {
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

uint64_t n_gi(const rv_ctx* c) { return (uint64_t)c->w.GX * c->w.GY * c->w.GZ; }
uint64_t n_csdf(const rv_ctx* c) { return (uint64_t)c->w.SX * c->w.SY * c->w.SZ; }
uint64_t n_bits_words(const rv_ctx* c) { return ((uint64_t)c->w.X * c->w.Y * c->w.Z) >> 5; }

f3 host_v(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }

// glm::normalize(vec3(10,5,-4)) (src/StateRender.cu:299, src/CoarseArray.cu:359)
f3 sun_dir() {
    float d = 10.0f * 10.0f + 5.0f * 5.0f + (-4.0f) * (-4.0f);
    float inv = 1.0f / sqrtf(d);
    return host_v(10.0f * inv, 5.0f * inv, -4.0f * inv);
}

World current_world(const rv_ctx* c) {
    World w = c->w;
    world_set_brick(w, c->brick);
    w.gi = c->gi;
    w.atlas = c->atlas;
    return w;
}

}  // namespace

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
    if (cfg->width < 2 || cfg->height < 2 || (cfg->width & 1) || (cfg->height & 1)) return RV_ERR_INVALID;
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
    if (const char* e = getenv("RV_SCHED")) c->sched = atoi(e);
    if (const char* e = getenv("RV_BATCH_STREAMS")) c->batch_streams = atoi(e);
    if (const char* e = getenv("RV_GI_PRIO")) c->gi_low_prio = atoi(e);
    if (const char* e = getenv("RV_ORDER_EVERY")) c->order_every = atoi(e) > 0 ? atoi(e) : 1;
    if (const char* e = getenv("RV_PIPE")) c->pipe = atoi(e);
    if (const char* e = getenv("RV_PIPE_CARRY")) c->pipe_carry = atoi(e);
    if (const char* e = getenv("RV_FLOW")) c->flow = atoi(e);
    if (const char* e = getenv("RV_GI_PAIRS")) c->gi_pairs = atoi(e);
    if (const char* e = getenv("RV_PRIO_BLOCKS")) c->prio_blocks = (uint32_t)std::max(0, atoi(e));
    if (const char* e = getenv("RV_FLOW_SPIN")) c->flow_spin = (uint32_t)std::max(0, atoi(e));
    if (const char* e = getenv("RV_FLOW_FORCE_FALLBACK")) c->flow_force_fallback = atoi(e) != 0;
    if (const char* e = getenv("RV_FLOW_PP_ORDER")) c->flow_pp_order = (uint32_t)(atoi(e) != 0);
    if (const char* e = getenv("RV_FLOW_GI_SIDE")) c->flow_gi_side = atoi(e) != 0;
    if (const char* e = getenv("RV_GROUP")) c->group = std::min(32, std::max(0, atoi(e)));
    if (const char* e = getenv("RV_GATHER_BPP")) {   // 3 or 4; anything else is an error, not a silent default
        if (strcmp(e, "3") != 0 && strcmp(e, "4") != 0) return cleanup_fail(RV_ERR_INVALID, "RV_GATHER_BPP");
        c->gather_bpp = atoi(e);
    }
    if (const char* e = getenv("RV_PIPE_ORDER")) {   // a permutation of the parts, else the default
        const uint32_t o = (uint32_t)strtoul(e, nullptr, 16);
        const uint32_t a = o >> 8 & 0xF, b = o >> 4 & 0xF, d = o & 0xF;
        if (o <= 0x210 && a < 3 && b < 3 && d < 3 && a != b && b != d && a != d) c->pipe_order = o;
    }
    if (hipMalloc(&c->counters, NSTAGE * NCNT * sizeof(unsigned long long)) != hipSuccess)
        return cleanup_fail(RV_ERR_OOM, "counters");
    hipMemset(c->counters, 0, NSTAGE * NCNT * sizeof(unsigned long long));
    if (const char* e = getenv("RV_MEGAKERNEL")) c->megakernel = atoi(e) != 0;
    if (const char* e = getenv("RV_WF_ENQ")) c->enq = atoi(e);
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

static rv_status end_frame(rv_ctx* c) {
    if (c->slots.size() > 1) {
        FrameSlot& sl = c->slots[c->cur_slot];
        HIP_TRY(c, hipEventRecord(sl.done, c->stream));
        sl.pending = true;
    }
    return RV_OK;
}

// Before anything that rewrites state frames read (world, GI grid, device
// tile lists): `stream` waits for every frame still in flight.
static rv_status wait_all_frames(rv_ctx* c) {
    if (c->world_stream != c->stream) HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_world, 0));   // write after write
    if (c->slots.size() > 1)
        for (const FrameSlot& sl : c->slots)
            if (sl.pending) HIP_TRY(c, hipStreamWaitEvent(c->stream, sl.done, 0));
    return RV_OK;
}

// Everything that writes the world or the GI grid runs on `stream`; the GI
// side stream waits on this mark before it reads them.
static rv_status mark_world(rv_ctx* c) {
    HIP_TRY(c, hipEventRecord(c->ev_world, c->stream));
    c->world_ver++;
    c->world_stream = c->stream;
    return RV_OK;
}

// Uploads `src` to ids unless it equals the cached list; *changed tells.
static rv_status upload_ids(rv_ctx* c, DevIds& ids, const int32_t* src, int n, bool* changed) {
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
    if (bytes) *bytes = c->tex ? (uint64_t)c->w.X * c->w.Y * c->w.Z * 4 : 0;
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

// sampleTexture's tile table (World::tex, rv_device.h tex_index): 4 B per voxel, a function of the voxel
// coordinates only, so it is built once, at the first world build or import (bench.py's world_build_s
// includes it) and kept through rebuilds.  It is optional -- a context without it evaluates the noise in
// the kernels, with identical tiles -- so it is only allocated when it leaves room: the memory this
// context may still allocate (CSDF build scratch, the GI scratch grid, two grouped-frame sets of 32
// frames, the pipelined loop's buffers) plus 1 GiB, and at most half the device's free memory (other
// contexts on the GPU).  Env RV_TEX_TABLE=0: never; =1: whenever the allocation succeeds.
static rv_status tex_table(rv_ctx* c) {
    if (c->tex_tried) return RV_OK;
    c->tex_tried = true;
    const char* te = getenv("RV_TEX_TABLE");
    if (te && te[0] == '0') return RV_OK;
    const bool force = te && te[0] == '1';
    const size_t tb = (size_t)c->w.X * c->w.Y * c->w.Z * 4;
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
    launch_tex_table(c->stream, c->tex, c->w);
    LAUNCH_CHECK(c);
    c->w.tex = c->tex;
    return RV_OK;
}

// The sky exit of the frame traversal (World::ytop, rv_device.h trace): the highest solid voxel
// row + 2, and the sun exit of its shadow rays (World::horizon), recomputed after every write of the
// bits.  Env RV_SKY_EXIT=0 turns both off (ytop = Y, no horizon).
static rv_status world_top(rv_ctx* c) {
    c->w.ytop = (uint32_t)c->w.Y;
    uint32_t* hz = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(c->brick) + horizon_byte(c->w.coff));
    const size_t hzb = horizon_bytes(c->w.X, c->w.Z);
    HIP_TRY(c, hipMemsetAsync(hz, 0xFF, hzb, c->stream));   // no sun exit unless built below
    int* dt = reinterpret_cast<int*>(reinterpret_cast<char*>(c->brick) + dtop_byte(c->w.coff, c->w.X, c->w.Z));
    HIP_TRY(c, hipMemsetAsync(dt, 0x7F, dtop_bytes(c->w.X, c->w.Z), c->stream));   // no column skip unless built below
    const char* e = getenv("RV_SKY_EXIT");
    if (e && e[0] == '0') return RV_OK;
    if (!c->d_top) HIP_TRY(c, hipMalloc(&c->d_top, 4));
    HIP_TRY(c, hipMemsetAsync(c->d_top, 0, 4, c->stream));
    launch_world_top(c->stream, c->brick, current_world(c), c->d_top);
    LAUNCH_CHECK(c);
    uint32_t top = 0;
    HIP_TRY(c, hipMemcpyAsync(&top, c->d_top, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->w.ytop = std::min((uint32_t)c->w.Y, top + 1u);   // top = max solid y + 1
    // the column tops: the DDA's empty-column skip (dtop_at; env RV_COL_SKIP=0: off) and the sun horizon's input
    if (!c->coltop) HIP_TRY(c, hipMalloc(&c->coltop, hzb));
    HIP_TRY(c, hipMemsetAsync(c->coltop, 0, hzb, c->stream));
    const char* cs = getenv("RV_COL_SKIP");
    launch_column_tops(c->stream, c->brick, current_world(c), c->coltop, dt);
    LAUNCH_CHECK(c);
    if (cs && cs[0] == '0') HIP_TRY(c, hipMemsetAsync(dt, 0x7F, dtop_bytes(c->w.X, c->w.Z), c->stream));
    // the sun exit of shadow rays (trace_sun): the horizon per brick column for the library's sun
    // (env RV_SUN_EXIT=0: off)
    const char* se = getenv("RV_SUN_EXIT");
    const f3 sun = sun_dir();
    const double hxz = std::sqrt((double)sun.x * sun.x + (double)sun.z * sun.z);
    if ((se && se[0] == '0') || !(sun.y > 0.0f) || hxz == 0.0) return RV_OK;
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
    launch_gi_init(c->stream, c->gi, current_world(c), sun_dir(), c->counters + ST_GI * NCNT);
    LAUNCH_CHECK(c);
    c->gi_frame = 0;
    c->gi_offset = 0;
    return mark_world(c);
}

rv_status rv_world_build(rv_ctx* c) {
    if (!c) return RV_ERR_INVALID;
    if (rv_status ws = wait_all_frames(c)) return ws;
    c->geom_ver++;
    if (rv_status ts = tex_table(c)) return ts;
    launch_fill_bricks(c->stream, c->brick, current_world(c), c->cfg.seed_x, c->cfg.seed_z);
    LAUNCH_CHECK(c);
    if (rv_status ts = world_top(c)) return ts;
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
    if (rv_status ts = tex_table(c)) return ts;
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
        HIP_TRY(c, hipMemcpyAsync(c->gi + first, c->gi_tmp + first, count * 4, hipMemcpyDeviceToDevice,
                                  c->stream));
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
        HIP_TRY(c, hipMemcpyAsync(c->gi + c->gi_offset, c->gi_tmp + c->gi_offset, count * 4, hipMemcpyDeviceToDevice,
                                  c->stream));
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

static FrameParams make_params_d(rv_ctx* c, const rv_frame_desc& d, int32_t flags) {
    return make_params(c, &d.cam, d.vp, d.prev_vp, d.time, d.jitter_x, d.jitter_y, flags);
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
static rv_status upload_cams(rv_ctx* c, const Seq& q, hipStream_t st, const FrameCam** out,
                             const std::function<void(int, FrameCam&)>& fill = nullptr) {
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
static rv_status run_stages(rv_ctx* c, FrameParams f, bool tiles, int which = 3) {
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
        // kernel boundary costs ~6 us, the ordering itself ~4 us.
        if (f.sched == SCHED_COST && ++c->frames_since_order >= (uint32_t)c->order_every) {
            c->frames_since_order = 0;
            if (tiles) {
                launch_chunk_order(c->stream, c->tile_cost, c->tile_order, (uint32_t)f.ntiles,
                                   ((uint32_t)f.ntiles + 7u) & ~7u);
            } else {
                if (pre) launch_chunk_order(c->stream, c->chunk_cost[CG_PREPASS], c->chunk_order[CG_PREPASS],
                                            n_chunks(f.hw, f.hh), n_chunks_pad(f.hw, f.hh));
                launch_chunk_order(c->stream, c->chunk_cost[CG_RENDER], c->chunk_order[CG_RENDER],
                                   n_chunks(f.W, f.H), n_chunks_pad(f.W, f.H));
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
    p.flow_pp_by_render = c->flow_pp_order;
    if (const char* e = getenv("RV_FLOW_OPTS")) p.flow_opts = (uint32_t)atoi(e);   // A/B experiments
    // pre-pass workgroups: 16 per render chunk slot in the render's order, or the pre-pass's own grid
    p.len[0] = c->flow_pp_order ? n_chunks_pad(f.W, f.H) * 16u : pipe_len(f, PIPE_PP, 0);
    p.len[2] = pipe_len(f, PIPE_RENDER, 0);
    p.gi_pairs = c->gi_pairs > 0 && pipe_latency_variant(f, p.len[2]) ? 1u : 0u;   // whole frames: off unless forced
    const bool side = spec && c->flow_gi_side && c->gi_stream;
    p.len[1] = spec && !side ? pipe_len(f, PIPE_GI, p.gi_pairs ? 2 * count : count) : 0u;
    if (side) {
        // the GI stream starts once the grid this frame renders with is complete (every earlier write of
        // `gi` and gi_tmp on the frame stream: the last copy-back included), then computes the window
        // into gi_tmp beside the flow launch; the next rv_update_gi_data waits for ev_spec
        if (!c->ev_spec) HIP_TRY(c, hipEventCreateWithFlags(&c->ev_spec, hipEventDisableTiming));
        HIP_TRY(c, hipEventRecord(c->ev_spec, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->gi_stream, c->ev_spec, 0));
        launch_gi_update(c->gi_stream, c->gi, c->gi_tmp, current_world(c), sun_dir(), c->gi_frame, first, count,
                         c->counters + ST_GI * NCNT, false);
        LAUNCH_CHECK(c);
    }
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
        HIP_TRY(c, hipEventRecord(c->ev_spec, side ? c->gi_stream : c->stream));
        c->spec_stream = side ? c->gi_stream : c->stream;
        c->spec_rec = true;
        c->spec_gi = true;
        c->spec_fr = c->gi_frame; c->spec_first = first; c->spec_count = count; c->spec_world = c->world_ver;
    }
    if (f.sched == SCHED_COST && ++c->frames_since_order >= (uint32_t)c->order_every) {
        c->frames_since_order = 0;
        launch_chunk_order(c->stream, c->chunk_cost[CG_PREPASS], c->chunk_order[CG_PREPASS], n_chunks(f.hw, f.hh),
                           n_chunks_pad(f.hw, f.hh));
        launch_chunk_order(c->stream, c->chunk_cost[CG_RENDER], c->chunk_order[CG_RENDER], n_chunks(f.W, f.H),
                           n_chunks_pad(f.W, f.H));
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
static rv_status tile_list(rv_ctx* c, const int32_t* tile_ids, int32_t ntiles, int32_t tile_px) {
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

// ===================================================================== render loop
// RCCL, resolved at run time from the library the process already uses
// (torch's bundled librccl when called from Python: pass its path), so no
// second RCCL/HIP runtime is loaded next to it.
namespace {
struct RcclApi {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;   // optional
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;                   // optional
};
RcclApi g_rccl;

bool rccl_load(const char* path, std::string& err) {
    if (g_rccl.h) return true;
    const char* names[] = {path, "librccl.so.1", "librccl.so"};
    for (const char* n : names) {
        if (!n || !*n) continue;
        g_rccl.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
        if (g_rccl.h) break;
    }
    if (!g_rccl.h) { err = std::string("dlopen librccl: ") + dlerror(); return false; }
    auto sym = [&](const char* n) { return dlsym(g_rccl.h, n); };
    g_rccl.get_unique_id = (decltype(g_rccl.get_unique_id))sym("ncclGetUniqueId");
    g_rccl.comm_init_rank = (decltype(g_rccl.comm_init_rank))sym("ncclCommInitRank");
    g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))sym("ncclCommDestroy");
    g_rccl.send = (decltype(g_rccl.send))sym("ncclSend");
    g_rccl.recv = (decltype(g_rccl.recv))sym("ncclRecv");
    g_rccl.all_gather = (decltype(g_rccl.all_gather))sym("ncclAllGather");
    g_rccl.group_start = (decltype(g_rccl.group_start))sym("ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))sym("ncclGroupEnd");
    g_rccl.error_string = (decltype(g_rccl.error_string))sym("ncclGetErrorString");
    g_rccl.async_error = (decltype(g_rccl.async_error))sym("ncclCommGetAsyncError");
    g_rccl.comm_abort = (decltype(g_rccl.comm_abort))sym("ncclCommAbort");
    if (!g_rccl.get_unique_id || !g_rccl.comm_init_rank || !g_rccl.comm_destroy || !g_rccl.send || !g_rccl.recv ||
        !g_rccl.all_gather || !g_rccl.group_start || !g_rccl.group_end || !g_rccl.error_string) {
        err = "librccl lacks a required symbol";
        g_rccl = RcclApi{};
        return false;
    }
    return true;
}
}  // namespace

static double comm_timeout_s() {
    if (const char* e = getenv("RV_COMM_TIMEOUT_S")) {
        char* end = nullptr;
        const double v = strtod(e, &end);
        if (end && *end == '\0' && v > 0) return v;
    }
    return 120.0;
}

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

static void comm_detach(rv_comm* m) { m->ctx = nullptr; }   // its context is being destroyed

#define NCCL_TRY(ctx, expr)                                                                  \
    do {                                                                                     \
        ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess)                                                               \
            return fail((ctx), RV_ERR_HIP, std::string(#expr) + ": " + g_rccl.error_string(r_)); \
    } while (0)

static rv_status loop_round(rv_ctx* c, rv_comm* m, hipStream_t s);

// Waits (host) until every stream of the context has drained, polling the
// communicator's asynchronous error; on an error or after timeout_s the
// communicator is aborted and RV_ERR_HIP returned (per-GPU
// timeouts in the multi-GPU driver) -- a dead peer never hangs the caller.
static rv_status comm_wait_bounded(rv_ctx* c, rv_comm* m, double timeout_s) {
    std::vector<hipStream_t> ss = {c->stream, c->comm_stream, c->gi_stream};
    for (hipStream_t f : c->fstreams) ss.push_back(f);
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        bool busy = false;
        for (hipStream_t s : ss) {
            if (!s && s != c->stream) continue;   // an unused side stream (the caller's may be the NULL stream)
            const hipError_t e = hipStreamQuery(s);
            if (e == hipErrorNotReady) { busy = true; continue; }
            if (e != hipSuccess) return fail(c, RV_ERR_HIP, std::string("hipStreamQuery: ") + hipGetErrorString(e));
        }
        if (!busy) return RV_OK;
        if (m && m->comm && g_rccl.async_error) {
            ncclResult_t ae = ncclSuccess;
            if (g_rccl.async_error(m->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                m->aborted = true;
                if (g_rccl.comm_abort) g_rccl.comm_abort(m->comm);
                return fail(c, RV_ERR_HIP, std::string("RCCL asynchronous error: ") + g_rccl.error_string(ae));
            }
        }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            if (m) {
                m->aborted = true;
                if (m->comm && g_rccl.comm_abort) g_rccl.comm_abort(m->comm);
                if (m->loop) m->loop->abort();
            }
            return fail(c, RV_ERR_HIP, "timed out waiting for the frame loop (a peer rank stalled or died)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

static rv_status comm_all_gather(rv_ctx* c, rv_comm* m, const void* send, void* recv, size_t bytes, hipStream_t s) {
    if (m->aborted) return fail(c, RV_ERR_HIP, "communicator aborted");
    if (m->comm) {
        NCCL_TRY(c, g_rccl.all_gather(send, recv, bytes, ncclUint8, m->comm, s));
        return RV_OK;
    }
    m->pending = LoopGroup::Post{};
    m->pending.kind = 1; m->pending.send = send; m->pending.recv = recv; m->pending.bytes = bytes;
    return loop_round(c, m, s);
}

static rv_status comm_group_start(rv_ctx* c, rv_comm* m) {
    if (m->aborted) return fail(c, RV_ERR_HIP, "communicator aborted");
    if (m->comm) NCCL_TRY(c, g_rccl.group_start());
    m->in_group = true;
    m->pending = LoopGroup::Post{};
    m->pending.kind = 2;
    return RV_OK;
}

static rv_status comm_send(rv_ctx* c, rv_comm* m, const void* buf, size_t bytes, int peer, hipStream_t s) {
    if (m->comm) { NCCL_TRY(c, g_rccl.send(buf, bytes, ncclUint8, peer, m->comm, s)); return RV_OK; }
    m->pending.p2p.emplace_back(1, peer, buf, nullptr, bytes);
    return RV_OK;
}

static rv_status comm_recv(rv_ctx* c, rv_comm* m, void* buf, size_t bytes, int peer, hipStream_t s) {
    if (m->comm) { NCCL_TRY(c, g_rccl.recv(buf, bytes, ncclUint8, peer, m->comm, s)); return RV_OK; }
    m->pending.p2p.emplace_back(0, peer, nullptr, buf, bytes);
    return RV_OK;
}

static rv_status comm_group_end(rv_ctx* c, rv_comm* m, hipStream_t s) {
    m->in_group = false;
    if (m->comm) { NCCL_TRY(c, g_rccl.group_end()); return RV_OK; }
    return loop_round(c, m, s);
}

// One loopback round (see LoopGroup): post, meet, fetch, meet, release.
static rv_status loop_round(rv_ctx* c, rv_comm* m, hipStream_t s) {
    LoopGroup* g = m->loop;
    if (!m->ready) HIP_TRY(c, hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
    if (!m->done) HIP_TRY(c, hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
    HIP_TRY(c, hipEventRecord(m->ready, s));
    m->pending.ready = m->ready; m->pending.done = m->done;
    {
        std::lock_guard<std::mutex> lk(g->m);
        g->post[(size_t)m->rank] = m->pending;
    }
    if (!g->barrier()) { m->aborted = true; return fail(c, RV_ERR_HIP, "loopback: a peer did not arrive (timeout)"); }
    // snapshot of the round: a peer posts its next round only after the second barrier
    std::vector<LoopGroup::Post> post;
    {
        std::lock_guard<std::mutex> lk(g->m);
        post = g->post;
    }
    const LoopGroup::Post& me = post[(size_t)m->rank];
    for (int q = 0; q < g->n; q++) {
        const LoopGroup::Post& o = post[(size_t)q];
        if (o.kind != me.kind) { m->aborted = true; g->abort(); return fail(c, RV_ERR_HIP, "loopback: ranks diverged"); }
    }
    if (me.kind == 1) {   // all-gather: fetch every rank's block
        for (int q = 0; q < g->n; q++) {
            const LoopGroup::Post& o = post[(size_t)q];
            if (o.bytes != me.bytes) { m->aborted = true; g->abort(); return fail(c, RV_ERR_HIP, "loopback: all-gather sizes differ"); }
            if (q != m->rank) HIP_TRY(c, hipStreamWaitEvent(s, o.ready, 0));
            HIP_TRY(c, hipMemcpyAsync(static_cast<char*>(me.recv) + (size_t)q * me.bytes, o.send, me.bytes,
                                      hipMemcpyDeviceToDevice, s));
        }
    } else {              // grouped p2p: every recv fetches the matching send of its peer (k-th with k-th)
        std::vector<int> used((size_t)g->n, 0);
        for (const auto& op : me.p2p) {
            if (std::get<0>(op)) continue;
            const int q = std::get<1>(op);
            if (q < 0 || q >= g->n) { m->aborted = true; g->abort(); return fail(c, RV_ERR_HIP, "loopback: bad peer"); }
            const LoopGroup::Post& o = post[(size_t)q];
            int seen = 0;
            const std::tuple<int, int, const void*, void*, size_t>* match = nullptr;
            for (const auto& so : o.p2p)
                if (std::get<0>(so) && std::get<1>(so) == m->rank && seen++ == used[(size_t)q]) { match = &so; break; }
            if (!match || std::get<4>(*match) != std::get<4>(op)) {
                m->aborted = true; g->abort();
                return fail(c, RV_ERR_HIP, "loopback: send/recv mismatch");
            }
            used[(size_t)q]++;
            if (q != m->rank) HIP_TRY(c, hipStreamWaitEvent(s, o.ready, 0));
            HIP_TRY(c, hipMemcpyAsync(std::get<3>(op), std::get<2>(*match), std::get<4>(op), hipMemcpyDeviceToDevice, s));
        }
    }
    HIP_TRY(c, hipEventRecord(m->done, s));
    if (!g->barrier()) { m->aborted = true; return fail(c, RV_ERR_HIP, "loopback: a peer did not arrive (timeout)"); }
    for (int q = 0; q < g->n; q++)   // my buffers are reusable once every reader's copies ran
        if (q != m->rank) HIP_TRY(c, hipStreamWaitEvent(s, post[(size_t)q].done, 0));
    return RV_OK;
}

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
    // timing probe (env RV_GI_SHARD_PROBE, no communicator): this rank's GI share only, no exchange --
    // the grid is then NOT the reference's; only for sizing the multi-GPU loop on one GPU
    const bool probe = tiles && !comm && N > 1 && getenv("RV_GI_SHARD_PROBE") != nullptr;
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
        HIP_TRY(c, hipMemcpyAsync(c->gi + first, c->gi_tmp + first, count * 4, hipMemcpyDeviceToDevice, S));
    } else if (xchg) {   // ... or kept from the previous call: this rank's share, exchanged now
        if (rv_status as = comm_all_gather(c, comm, c->pipe_gi_stage, c->pipe_gi_all, chunk * 4, c->comm_stream))
            return as;
        HIP_TRY(c, hipEventRecord(c->pipe_ev[1], c->comm_stream));
        HIP_TRY(c, hipStreamWaitEvent(S, c->pipe_ev[1], 0));
        HIP_TRY(c, hipMemcpyAsync(c->gi + first, c->pipe_gi_all, count * 4, hipMemcpyDeviceToDevice, S));
    } else if (!probe) {
        HIP_TRY(c, hipMemcpyAsync(c->gi + first, c->gi_tmp + first, count * 4, hipMemcpyDeviceToDevice, S));
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
        p.prio_blocks = c->prio_blocks;
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
                HIP_TRY(c, hipMemcpyAsync(c->gi + first, c->pipe_gi_all, count * 4, hipMemcpyDeviceToDevice, S));
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
                HIP_TRY(c, hipMemcpyAsync(c->gi + first, c->gi_tmp + first, count * 4, hipMemcpyDeviceToDevice, S));
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
                                   n_chunks_pad(f.hw, f.hh));
                launch_chunk_order(S, c->chunk_cost[CG_RENDER], c->chunk_order[CG_RENDER], n_chunks(f.W, f.H),
                                   n_chunks_pad(f.W, f.H));
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
    const bool probe = tiles && !comm && N > 1 && getenv("RV_GI_SHARD_PROBE") != nullptr;
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
                                   n_chunks_pad(fo.hw, fo.hh));
                launch_chunk_order(S, c->chunk_cost[CG_RENDER], c->chunk_order[CG_RENDER], n_chunks(W, H),
                                   n_chunks_pad(W, H));
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

rv_status rv_comm_unique_id(const char* rccl_path, void* id, size_t bytes) {
    if (!id || bytes < sizeof(ncclUniqueId)) return RV_ERR_INVALID;
    std::string err;
    if (!rccl_load(rccl_path, err)) return RV_ERR_HIP;
    ncclUniqueId u;
    if (g_rccl.get_unique_id(&u) != ncclSuccess) return RV_ERR_HIP;
    memcpy(id, &u, sizeof(u));
    return RV_OK;
}

rv_status rv_comm_create(rv_ctx* c, const char* rccl_path, const void* id, size_t bytes, int32_t nranks, int32_t rank,
                         rv_comm** out) {
    if (!c || !id || !out || bytes < sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
        return RV_ERR_INVALID;
    *out = nullptr;
    std::string err;
    if (!rccl_load(rccl_path, err)) return fail(c, RV_ERR_HIP, err);
    HIP_TRY(c, hipSetDevice(c->device));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    rv_comm* m = new rv_comm();
    m->rank = rank; m->nranks = nranks; m->device = c->device; m->ctx = c;
    ncclResult_t r = g_rccl.comm_init_rank(&m->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete m;
        return fail(c, RV_ERR_HIP, std::string("ncclCommInitRank: ") + g_rccl.error_string(r));
    }
    *out = m;
    return RV_OK;
}

rv_status rv_loopback_group_create(int32_t nranks, int32_t timeout_ms, void** out) {
    if (nranks < 1 || !out) return RV_ERR_INVALID;
    LoopGroup* g = new LoopGroup();
    g->n = nranks;
    g->post.resize((size_t)nranks);
    if (timeout_ms > 0) g->timeout_s = timeout_ms * 1e-3;
    *out = g;
    return RV_OK;
}

void rv_loopback_group_destroy(void* group) { delete static_cast<LoopGroup*>(group); }

rv_status rv_comm_create_loopback(rv_ctx* c, void* group, int32_t nranks, int32_t rank, rv_comm** out) {
    LoopGroup* g = static_cast<LoopGroup*>(group);
    if (!c || !g || !out || nranks != g->n || rank < 0 || rank >= nranks) return RV_ERR_INVALID;
    rv_comm* m = new rv_comm();
    m->loop = g; m->rank = rank; m->nranks = nranks; m->device = c->device; m->ctx = c;
    *out = m;
    return RV_OK;
}

rv_status rv_comm_wait(rv_comm* m, int32_t timeout_ms) {
    if (!m || !m->ctx) return RV_ERR_INVALID;
    return comm_wait_bounded(m->ctx, m, timeout_ms > 0 ? timeout_ms * 1e-3 : comm_timeout_s());
}

void rv_comm_destroy(rv_comm* m) {
    if (!m) return;
    rv_ctx* c = m->ctx;
    const bool ok = !c || comm_wait_bounded(c, m, comm_timeout_s()) == RV_OK;
    if (c && c->comm_attached == m) c->comm_attached = nullptr;
    if (m->comm) {
        hipSetDevice(m->device);
        if (ok && !m->aborted && g_rccl.comm_destroy) g_rccl.comm_destroy(m->comm);
        else if (g_rccl.comm_abort) g_rccl.comm_abort(m->comm);   // a peer is gone: do not wait for it
    }
    if (m->ready) hipEventDestroy(m->ready);
    if (m->done) hipEventDestroy(m->done);
    if (m->vdev) hipFree(m->vdev);
    if (m->vhost) hipHostFree(m->vhost);
    delete m;
}

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
    float w0 = 1.0f;
    if (const char* e = getenv("RV_SHARD_ROOT_WEIGHT")) {   // strict: a value that does not parse is an error
        char* end = nullptr;
        const double v = strtod(e, &end);
        if (!end || end == e || *end != '\0') return fail(c, RV_ERR_INVALID, "RV_SHARD_ROOT_WEIGHT does not parse");
        w0 = (float)v;
    }
    return rv_set_tile_shard_weighted(c, tile_px, rank, nranks, w0);
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
