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
//   SCHED_QUEUE    : persistent workgroups pull blocks (chunk order) from an
//                    atomic counter until the frame is drained
__device__ __forceinline__ bool chunk_block(uint32_t k, uint32_t nbx, uint32_t nby, uint32_t& bx,
                                            uint32_t& by) {
    const uint32_t CB = 4;
    uint32_t ncx = (nbx + CB - 1) / CB;
    uint32_t chunk = k / (CB * CB), j = k % (CB * CB);
    bx = (chunk % ncx) * CB + j % CB;
    by = (chunk / ncx) * CB + j / CB;
    return bx < nbx && by < nby;
}

__host__ __device__ inline uint32_t sched_grid(int sched, uint32_t nbx, uint32_t nby, uint32_t persistent) {
    const uint32_t CB = 4;
    uint32_t nch = ((nbx + CB - 1) / CB) * ((nby + CB - 1) / CB);
    switch (sched) {
    case SCHED_CHUNK: return ((nch + 7) & ~7u) * CB * CB;
    case SCHED_QUEUE: return persistent;
    default: return nbx * nby;
    }
}

// Returns the next block of this workgroup (uniform across it), false when done.
__device__ __forceinline__ bool sched_next(int sched, unsigned* queue, uint32_t nbx, uint32_t nby,
                                           uint32_t& iter, uint32_t& bx, uint32_t& by) {
    if (sched == SCHED_QUEUE) {
        __shared__ uint32_t s_k;
        const uint32_t CB = 4;
        uint32_t total = ((nbx + CB - 1) / CB) * ((nby + CB - 1) / CB) * CB * CB;
        for (;;) {
            __syncthreads();
            if (threadIdx.x == 0) s_k = atomicAdd(queue, 1u);
            __syncthreads();
            uint32_t k = s_k;
            if (k >= total) return false;
            if (chunk_block(k, nbx, nby, bx, by)) return true;
        }
    }
    if (iter++ > 0) return false;
    uint32_t b = blockIdx.x;
    if (sched == SCHED_BAND) {
        b = xcd_swizzle(b, nbx * nby);
    } else if (sched == SCHED_CHUNK) {
        const uint32_t CB = 4;
        uint32_t xcd = b & 7u, k = b >> 3;
        uint32_t chunk = (k / (CB * CB)) * 8 + xcd;
        return chunk_block(chunk * CB * CB + k % (CB * CB), nbx, nby, bx, by);
    }
    bx = b % nbx;
    by = b / nbx;
    return by < nby;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// minDist (StateRender.cu:182-198) with W/2 x H/2 (Appendix R6)
__device__ __forceinline__ float min_dist(const FrameParams& f, float x, float y) {
    int u = (int)floorf(x * (float)f.hw), v = (int)floorf(y * (float)f.hh);
    int u1 = clampi(u + 1, 0, f.hw - 1), v1 = clampi(v + 1, 0, f.hh - 1);
    u = clampi(u, 0, f.hw - 1); v = clampi(v, 0, f.hh - 1);
    const float* hd = f.hdist;
    float d1 = hd[(size_t)v * f.hw + u], d2 = hd[(size_t)v * f.hw + u1];
    float d3 = hd[(size_t)v1 * f.hw + u], d4 = hd[(size_t)v1 * f.hw + u1];
    return fminf(fminf(d1, d2), fminf(d3, d4));
}

// tex2D<float> linear/clamp/normalized with 1/256 weights (StateRender.cu:230)
__device__ __forceinline__ float bilinear_tex(const FrameParams& f, float x, float y) {
    float xb = x * (float)f.hw - 0.5f, yb = y * (float)f.hh - 0.5f;
    float fx0 = floorf(xb), fy0 = floorf(yb);
    float a = rintf((xb - fx0) * 256.0f) / 256.0f;
    float b = rintf((yb - fy0) * 256.0f) / 256.0f;
    int i0 = (int)fx0, j0 = (int)fy0;
    int i1 = clampi(i0 + 1, 0, f.hw - 1), j1 = clampi(j0 + 1, 0, f.hh - 1);
    i0 = clampi(i0, 0, f.hw - 1); j0 = clampi(j0, 0, f.hh - 1);
    const float* hs = f.hshadow;
    float t00 = hs[(size_t)j0 * f.hw + i0], t10 = hs[(size_t)j0 * f.hw + i1];
    float t01 = hs[(size_t)j1 * f.hw + i0], t11 = hs[(size_t)j1 * f.hw + i1];
    return (1.0f - a) * (1.0f - b) * t00 + a * (1.0f - b) * t10 + (1.0f - a) * b * t01 + a * b * t11;
}

// resident workgroups for a persistent launch: occupancy x CUs
template <typename K>
inline uint32_t resident_blocks(K kernel) {
    int dev = 0, ncu = 256, per = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0);
    return (uint32_t)(ncu * (per > 0 ? per : 1));
}


}  // namespace rv
