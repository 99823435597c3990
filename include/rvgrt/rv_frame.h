// rv_frame.h -- frame-kernel helpers shared by the per-pixel kernels
// (rv_kernels.hip) and the wavefront stages (rv_wavefront.hip).
#pragma once
#include "rv_internal.h"

namespace rv {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t nb) {
    uint32_t nb8 = nb & ~7u;
    if (b >= nb8) return b;
    uint32_t per = nb8 >> 3;
    return (b & 7u) * per + (b >> 3);
}

template <int N>
__device__ __forceinline__ void block_count_flush(unsigned long long* counters, uint32_t (&c)[N]) {
    __shared__ uint32_t s_cnt[N];
    if (threadIdx.x < N) s_cnt[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; k++)
        if (c[k]) atomicAdd(&s_cnt[k], c[k]);
    __syncthreads();
    if (threadIdx.x < N && s_cnt[threadIdx.x])
        atomicAdd(&counters[threadIdx.x], (unsigned long long)s_cnt[threadIdx.x]);
}

static constexpr float SHADOW_HIT = 0.199951171875f;   // (float)(half)0.2f

// Workgroup index and frame of a batched launch.  Interleaved (ileave = B > 1,
// chunked grids whose x extent is a multiple of 8): XCD x's k-th workgroup
// runs slot k / B of frame k % B, so the longest chunks of every frame of the
// batch start first and no frame's tail trails the launch.  Otherwise the
// frame is grid y.
__device__ __forceinline__ uint32_t batch_block(const FrameParams& f, uint32_t& frame) {
    uint32_t b = blockIdx.x;
    frame = blockIdx.y;
    if (f.ileave > 1) {
        const uint32_t xcd = b & 7u, k = b >> 3;
        frame = k % f.ileave;
        b = ((k / f.ileave) << 3) | xcd;
    }
    return b;
}

// Frame b of a batched launch: its camera (per-frame table) and its outputs
// (wave-uniform, SGPR math).
// CAMS: the launch has a per-frame camera table (instantiated separately:
// the table's loads cost the kernels without one 3 VGPRs).
template <bool CAMS = false>
__device__ __forceinline__ void batch_frame(FrameParams& f, uint64_t b) {
    f.cam = nullptr;
    if (CAMS) {
        const FrameCam* c = f.cams + b;
        f.cam = c;
        f.pos = c->pos; f.fo = c->fo; f.ri = c->ri; f.up = c->up;
        f.time = c->time; f.jx = c->jx; f.jy = c->jy;
    }
    if (b == 0) return;
    f.color = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(f.color) + b * f.bs_color);
    if (f.mv) f.mv = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(f.mv) + b * f.bs_mv);
    if (f.depth) f.depth = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(f.depth) + b * f.bs_depth);
    f.hdist = reinterpret_cast<float*>(reinterpret_cast<char*>(f.hdist) + b * f.bs_half);
    f.hshadow = reinterpret_cast<float*>(reinterpret_cast<char*>(f.hshadow) + b * f.bs_half);
    if (f.tilebuf) f.tilebuf = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(f.tilebuf) + b * f.bs_tile);
}

__device__ __forceinline__ f3 ray_dir(const FrameParams& f, float x, float y) {
    float nx = x * 2.0f - 1.0f + f.jx;   // StateRender.cu:44
    float ny = y * 2.0f - 1.0f + f.jy;
    return normalize(add(add(f.fo, scale(f.ri, nx)), scale(f.up, ny)));
}

// ---------------------------------------------------------------- scheduling
// Workgroup -> 16x16 pixel block of an nbx x nby grid.
//   SCHED_IDENTITY : row-major
//   SCHED_BAND     : XCD x takes a contiguous 1/8 band (L2 locality, but the
//                    sky/terrain cost gradient makes the bands unequal)
//   SCHED_CHUNK    : 4x4-block chunks (64x64 px) dealt round-robin to XCDs:
//                    locality inside a chunk, balance across XCDs
//   SCHED_COST     : SCHED_CHUNK with the chunks dealt in descending order of
//                    their cost in the previous frame (longest-job-first), so
//                    the waves with the longest rays start first instead of
//                    forming the kernel's tail (chunk_order; identity at first)
static constexpr uint32_t CHUNK_PX = 64;   // chunk = 64 x 64 pixels

__host__ __device__ inline uint32_t chunks_x(uint32_t w) { return (w + CHUNK_PX - 1) / CHUNK_PX; }
__host__ __device__ inline uint32_t n_chunks(uint32_t w, uint32_t h) { return chunks_x(w) * chunks_x(h); }
__host__ __device__ inline uint32_t n_chunks_pad(uint32_t w, uint32_t h) { return (n_chunks(w, h) + 7) & ~7u; }

// Grid of BW x BH-pixel workgroup regions over a w x h image (BW, BH
// divide CHUNK_PX).
template <uint32_t BW, uint32_t BH>
__host__ __device__ inline uint32_t sched_grid(int sched, uint32_t w, uint32_t h) {
    constexpr uint32_t PER = (CHUNK_PX / BW) * (CHUNK_PX / BH);
    if (sched == SCHED_CHUNK || sched == SCHED_COST) return n_chunks_pad(w, h) * PER;
    return ((w + BW - 1) / BW) * ((h + BH - 1) / BH);
}

// Region (bx, by) of this workgroup; false for the padding workgroups of a
// chunked grid and for regions off the image.
template <uint32_t BW, uint32_t BH>
__device__ __forceinline__ bool sched_block(int sched, const int* order, uint32_t w, uint32_t h, uint32_t& bx,
                                            uint32_t& by, uint32_t b) {
    constexpr uint32_t CX = CHUNK_PX / BW, CY = CHUNK_PX / BH, PER = CX * CY;
    const uint32_t nbx = (w + BW - 1) / BW, nby = (h + BH - 1) / BH;
    if (sched == SCHED_CHUNK || sched == SCHED_COST) {
        // workgroup b runs on XCD b % 8: slot k of that XCD takes sorted chunk
        // (k / PER) * 8 + xcd, region k % PER inside it
        uint32_t xcd = b & 7u, k = b >> 3;
        uint32_t pos = (k / PER) * 8 + xcd;
        uint32_t chunk = (sched == SCHED_COST && order) ? (uint32_t)order[pos] : pos;
        uint32_t j = k % PER, ncx = chunks_x(w);
        bx = (chunk % ncx) * CX + j % CX;
        by = (chunk / ncx) * CY + j / CX;
        return bx < nbx && by < nby;
    }
    if (sched == SCHED_BAND) b = xcd_swizzle(b, nbx * nby);
    bx = b % nbx;
    by = b / nbx;
    return by < nby;
}

// SCHED_COST feedback: every wave reports its lifetime to its chunk.
template <uint32_t BW, uint32_t BH>
__device__ __forceinline__ void chunk_cost_report(uint32_t* cost, uint64_t t0, uint32_t w, uint32_t bx, uint32_t by) {
    if (!cost || (threadIdx.x & 63) != 0) return;
    uint64_t dt = wall_clock64() - t0;
    atomicMax(&cost[(by * BH / CHUNK_PX) * chunks_x(w) + bx * BW / CHUNK_PX],
              (uint32_t)(dt > 0xFFFFFFFEull ? 0xFFFFFFFEull : dt) + 1u);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Half-res window of an 8x8-pixel wave: the 8x8 texels of the distance and
// shadow images from (ox, oy) = (X0/2 - 2, Y0/2 - 2), X0/Y0 the tile origin,
// staged in LDS by one coalesced load per image (every minDist / bilinear tap
// of the tile falls inside it when hw = W/2, hh = H/2), so the 8 taps per pixel
// read LDS instead of 8 scattered gathers (rows of the half-res image are
// separate 128-B lines: 8-13 lines per quarter-wave and tap).  Window texel
// (i, j) = image[clamp(oy + j)][clamp(ox + i)], so a tap at unclamped index r
// inside the window reads exactly what image[clamp(r)] holds; a tap outside it
// (other resolutions) reads the image.
struct HalfWin {
    const float* d;   // LDS: 64 distance texels, row-major 8x8 (nullptr: no window)
    const float* s;   // LDS: 64 shadow texels (SHADOW_PENDING: not published yet, flow launches only)
    int ox, oy;
    // flow launches (k_ref_flow): the tagged granules the window came from, for the shadow texels that were
    // still pending when the wave loaded its window (resolve_shadow_taps)
    const uint64_t* gran;
    uint32_t ntx;     // granule tiles per row
    uint32_t want;    // the launch's epoch (30 bits)
};
// A shadow texel whose pre-pass lane has published its distance but not yet its shadow (flow launches:
// the two-phase hand-off); never a value of the image (1 or SHADOW_HIT).
static constexpr float SHADOW_PENDING = -1.0f;
// Flow granule: {distance bits, shadow-hit bit, tag} with tag = epoch << 1 | phase in bits 33..63; phase 0
// carries the distance only (published after the camera ray), phase 1 the distance and the shadow (after
// the shadow ray).
__device__ __forceinline__ uint64_t flow_granule(float d, float s, uint32_t epoch, uint32_t phase) {
    return (uint64_t)__float_as_uint(d) | ((uint64_t)(s != 1.0f) << 32) |
           ((uint64_t)(((epoch & 0x3FFFFFFFu) << 1) | phase) << 33);
}
__device__ __forceinline__ size_t flow_granule_index(uint32_t ntx, int tx, int ty) {
    return (size_t)((uint32_t)(ty >> 3) * ntx + (uint32_t)(tx >> 3)) * 64 + (uint32_t)(ty & 7) * 8 + (uint32_t)(tx & 7);
}
// All 64 lanes of the wave call this (before any per-pixel branch): lane l
// loads texel (l & 7, l >> 3).  lds holds 128 floats for this wave.
__device__ __forceinline__ HalfWin half_window_load(const FrameParams& f, int X0, int Y0, float* lds) {
    HalfWin hw;
    hw.gran = nullptr; hw.ntx = 0; hw.want = 0;
    hw.ox = (X0 >> 1) - 2;
    hw.oy = (Y0 >> 1) - 2;
    const int l = (int)(threadIdx.x & 63u);
    const size_t q = (size_t)clampi(hw.oy + (l >> 3), 0, f.hh - 1) * f.hw + clampi(hw.ox + (l & 7), 0, f.hw - 1);
    lds[l] = f.hdist[q];
    lds[64 + l] = f.hshadow[q];
    hw.d = lds;
    hw.s = lds + 64;
    __syncthreads();
    return hw;
}
__device__ __forceinline__ float half_tap(const float* img, const float* win, const FrameParams& f, int ox, int oy,
                                          int ru, int rv) {
    const int wx = ru - ox, wy = rv - oy;
    if (win && (uint32_t)wx < 8u && (uint32_t)wy < 8u) return win[wy * 8 + wx];
    return img[(size_t)clampi(rv, 0, f.hh - 1) * f.hw + clampi(ru, 0, f.hw - 1)];
}

// minDist (StateRender.cu:182-198) with W/2 x H/2 (Appendix R6).  The
// reference fetches with normalized coordinates: u_low = floor(x*640)/640 and
// u_low + 1/640, each turned back into a texel by the point-sampling unit as
// floor(u*640); RV_F_REF_FETCH restates that float path (the quad can land a
// texel low where k/640*640 rounds below k), otherwise the texels are the
// exact k, k+1.  Indices stay unclamped here; half_tap clamps (point/clamp
// addressing, src/main.cpp:443).
__device__ __forceinline__ float min_dist(const FrameParams& f, float x, float y, const HalfWin* hwin = nullptr) {
    int u, v, u1, v1;
    if (f.flags & RV_F_REF_FETCH) {   // wave-uniform: a scalar branch
        const float fw = (float)f.hw, fh = (float)f.hh;
        const float ul = floorf(x * fw) / fw, vl = floorf(y * fh) / fh;
        const float px = 1.0f / fw, py = 1.0f / fh;
        u = (int)floorf(ul * fw);
        u1 = (int)floorf((ul + px) * fw);
        v = (int)floorf(vl * fh);
        v1 = (int)floorf((vl + py) * fh);
    } else {
        u = (int)floorf(x * (float)f.hw); v = (int)floorf(y * (float)f.hh);
        u1 = u + 1; v1 = v + 1;
    }
    const float* win = hwin ? hwin->d : nullptr;
    const int ox = hwin ? hwin->ox : 0, oy = hwin ? hwin->oy : 0;
    const float* hd = f.hdist;
    RV_GD_KIND(gd::HALF);
    RV_GD(0, hd + (size_t)clampi(v, 0, f.hh - 1) * f.hw + clampi(u, 0, f.hw - 1));
    float d1 = half_tap(hd, win, f, ox, oy, u, v), d2 = half_tap(hd, win, f, ox, oy, u1, v);
    float d3 = half_tap(hd, win, f, ox, oy, u, v1), d4 = half_tap(hd, win, f, ox, oy, u1, v1);
    return fminf(fminf(d1, d2), fminf(d3, d4));
}

// Flow launches: the shadow texels of this lane's 4 bilinear taps (bilinear_tex's indices) that were still
// pending when the window was loaded, read from their granules once their pre-pass lane has published
// the shadow (phase 1) and written back to the window.  The wait needs no bound: a pending texel's
// distance was published by its pre-pass wave, which is therefore running, never waits and publishes the
// shadow next (texels the render wave evaluated itself are never pending).
__device__ __forceinline__ void resolve_shadow_taps(const FrameParams& f, float x, float y, const HalfWin* hwin) {
    if (!hwin || !hwin->gran) return;
    float xb = x * (float)f.hw - 0.5f, yb = y * (float)f.hh - 0.5f;
    const int i0 = (int)floorf(xb), j0 = (int)floorf(yb);
    float* win = const_cast<float*>(hwin->s);
    const uint64_t want = ((uint64_t)hwin->want << 1) | 1u;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ru = i0 + (k & 1), rv = j0 + (k >> 1);
        const int wx = ru - hwin->ox, wy = rv - hwin->oy;
        if ((uint32_t)wx >= 8u || (uint32_t)wy >= 8u || win[wy * 8 + wx] != SHADOW_PENDING) continue;
        const uint64_t* g = hwin->gran + flow_granule_index(hwin->ntx, clampi(ru, 0, f.hw - 1), clampi(rv, 0, f.hh - 1));
        uint64_t v;
        while (((v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 33) != want)
            __builtin_amdgcn_s_sleep(8);
        win[wy * 8 + wx] = ((v >> 32) & 1u) ? SHADOW_HIT : 1.0f;
    }
}

// tex2D<float> linear/clamp/normalized with 1/256 weights (StateRender.cu:230)
__device__ __forceinline__ float bilinear_tex(const FrameParams& f, float x, float y, const HalfWin* hwin = nullptr) {
    float xb = x * (float)f.hw - 0.5f, yb = y * (float)f.hh - 0.5f;
    float fx0 = floorf(xb), fy0 = floorf(yb);
    float a = rintf((xb - fx0) * 256.0f) / 256.0f;
    float b = rintf((yb - fy0) * 256.0f) / 256.0f;
    const int i0 = (int)fx0, j0 = (int)fy0, i1 = i0 + 1, j1 = j0 + 1;
    const float* win = hwin ? hwin->s : nullptr;
    const int ox = hwin ? hwin->ox : 0, oy = hwin ? hwin->oy : 0;
    const float* hs = f.hshadow;
    RV_GD_KIND(gd::HALF);
    RV_GD(1, hs + (size_t)clampi(j0, 0, f.hh - 1) * f.hw + clampi(i0, 0, f.hw - 1));
    float t00 = half_tap(hs, win, f, ox, oy, i0, j0), t10 = half_tap(hs, win, f, ox, oy, i1, j0);
    float t01 = half_tap(hs, win, f, ox, oy, i0, j1), t11 = half_tap(hs, win, f, ox, oy, i1, j1);
    return (1.0f - a) * (1.0f - b) * t00 + a * (1.0f - b) * t10 + (1.0f - a) * b * t01 + a * b * t11;
}

}  // namespace rv
