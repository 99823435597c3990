// rv_wavefront.hip -- the frame as wavefront stages.
//
// The reference evaluates a whole pixel in one thread (renderKernel ->
// computeColor, src/StateRender.cu:33-253): on a 64-wide wave the shadow,
// reflection and cone work of a few lanes stalls the other 63, and the
// kernel's register footprint is the sum of every branch.  Here a frame is
//
//   k_wf_pp_primary  half-res primary rays (distApproximationKernel :255-286)
//   k_wf_pp_shadow   its sun-shadow rays, over the compacted hit queue Q_PP
//   k_wf_primary     full-res primary rays -> hit records (hpos/hinfo) and
//                    ballot-compacted queues: Q_WATER (water hits),
//                    Q_SHADOW (land hits needing a full-res shadow ray),
//                    Q_CONE (land hits needing GI cones)
//   k_wf_shadow      full-res sun-shadow rays            (queue Q_SHADOW)
//   k_wf_water       reflection + reflection-shadow rays (queue Q_WATER)
//   k_wf_cones       6 voxel cones per land hit          (queue Q_CONE)
//   k_wf_shade       texture, lighting, sky, fog, MV/depth, output
//
// Every stage keeps the reference's float operation order, so the result is
// bit-identical to the per-pixel path (rv_kernels.hip) and the CPU oracle.
// Queue order follows the wave ballots of the primary pass (8x8-pixel tiles),
// so secondary rays stay spatially coherent; results are written per pixel,
// so the (scheduling-dependent) queue order never changes the image.
#include "../../include/rvgrt/rv_frame.h"

namespace rv {

// -------------------------------------------------------------- helpers
// XCD of this workgroup under round-robin dispatch of linear workgroup ids
__device__ __forceinline__ uint32_t my_xcd() { return (blockIdx.x + blockIdx.y * gridDim.x) & (NXCD - 1); }

// Wave-aggregated append: one atomic per wave, slots in lane order.
// Must be reached by every lane of the wave (pred false where not wanted).
__device__ __forceinline__ void enqueue(const FrameParams& f, int q, bool pred, int value) {
    const uint64_t m = __ballot(pred);
    if (m == 0) return;
    const uint32_t lane = threadIdx.x & 63u, x = my_xcd();
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned base = 0;
    if ((int)lane == leader) base = atomicAdd(&f.qcount[qc_index(q, x)], (unsigned)__popcll(m));
    base = __shfl(base, leader);
    if (pred) f.queue_wf[q][(size_t)x * f.qcap[q] + base + (unsigned)__popcll(m & ((1ull << lane) - 1ull))] = value;
}

// Workgroup-aggregated append to NQ queues at once: one atomic per (workgroup,
// queue) instead of per (wave, queue) -- same-address device atomics are
// serialised, so a 2M-pixel frame with 32K waves pays for every one of them.
// Every thread of the (256-thread) workgroup must call it.
template <int NQ>
__device__ __forceinline__ void enqueue_block(const FrameParams& f, const int (&qid)[NQ], const bool (&pred)[NQ],
                                              int value) {
    __shared__ uint32_t s_n[NQ][4];
    __shared__ uint32_t s_base[NQ];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u, x = my_xcd();
    const uint64_t below = (1ull << lane) - 1ull;
    uint64_t m[NQ];
#pragma unroll
    for (int i = 0; i < NQ; i++) {
        m[i] = __ballot(pred[i]);
        if (lane == 0) s_n[i][wave] = (uint32_t)__popcll(m[i]);
    }
    __syncthreads();
    if (threadIdx.x < NQ) {
        const int i = (int)threadIdx.x;
        uint32_t tot = s_n[i][0] + s_n[i][1] + s_n[i][2] + s_n[i][3];
        s_base[i] = tot ? atomicAdd(&f.qcount[qc_index(qid[i], x)], tot) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NQ; i++) {
        if (pred[i]) {
            uint32_t off = s_base[i];
            for (uint32_t k = 0; k < wave; k++) off += s_n[i][k];
            f.queue_wf[qid[i]][(size_t)x * f.qcap[qid[i]] + off + (uint32_t)__popcll(m[i] & below)] = value;
        }
    }
}

// Consumer side: workgroup b serves sub-queue b % 8 (the XCD it runs on),
// items (b / 8) * 256 + tid.  False when this thread has no item.
__device__ __forceinline__ bool queue_item(const FrameParams& f, int q, int& p) {
    const uint32_t x = blockIdx.x & (NXCD - 1), k = (blockIdx.x / NXCD) * 256 + threadIdx.x;
    if (k >= f.qcount[qc_index(q, x)]) return false;
    p = f.queue_wf[q][(size_t)x * f.qcap[q] + k];
    return true;
}

// normal (components in {-1, +1, +0}) <-> 3-bit code
__device__ __forceinline__ uint32_t normal_code(f3 n) {
    if (n.x != 0.0f) return n.x > 0.0f ? 1u : 2u;
    if (n.y != 0.0f) return n.y > 0.0f ? 3u : 4u;
    if (n.z != 0.0f) return n.z > 0.0f ? 5u : 6u;
    return 0u;
}
__device__ __forceinline__ f3 normal_of(uint32_t code) {
    f3 n = V(0.0f, 0.0f, 0.0f);
    float s = (code & 1u) ? 1.0f : -1.0f;
    if (code == 1u || code == 2u) n.x = s;
    else if (code == 3u || code == 4u) n.y = s;
    else if (code == 5u || code == 6u) n.z = s;
    return n;
}
__device__ __forceinline__ float uv_bits(float u, float v) {
    return __uint_as_float((uint32_t)hbits(u) | ((uint32_t)hbits(v) << 16));
}
__device__ __forceinline__ float half_of(uint32_t b) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
}

// (ix, iy) of this thread in a one-shot full-frame grid (scheduled like the
// per-pixel kernels) or in a tile-list grid; false when it has no pixel.
template <bool TILES>
__device__ __forceinline__ bool pixel_of(const FrameParams& f, int W, int H, int tile_div, int& ix, int& iy) {
    uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t bx, by;
    if (TILES) {
        int T = f.tile_px / tile_div;                  // tile size at this resolution
        int tile = f.tiles[blockIdx.y];
        int tx = tile % f.tiles_x, ty = tile / f.tiles_x;
        int nb = (T + 15) >> 4;
        int lx = (int)((blockIdx.x % nb) * 16 + (wave & 1) * 8 + (lane & 7));
        int ly = (int)((blockIdx.x / nb) * 16 + (wave >> 1) * 8 + (lane >> 3));
        ix = tx * T + lx; iy = ty * T + ly;
        return lx < T && ly < T && ix < W && iy < H;
    }
    if (!sched_block<16, 16>(f.sched, nullptr, W, H, bx, by, blockIdx.x)) { ix = iy = 0; return false; }
    ix = (int)(bx * 16 + (wave & 1) * 8 + (lane & 7));
    iy = (int)(by * 16 + (wave >> 1) * 8 + (lane >> 3));
    return ix < W && iy < H;
}

// ------------------------------------------------------------ pre-pass
template <bool STATS, bool TILES>
__global__ void __launch_bounds__(256) k_wf_pp_primary(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int ix = 0, iy = 0;
    bool valid;
    if (TILES) {   // half-res footprint of the tile plus a one-texel halo
        int T2 = f.tile_px / 2 + 2, k = (int)(blockIdx.x * 256 + threadIdx.x);
        int tile = f.tiles[blockIdx.y];
        int tx = tile % f.tiles_x, ty = tile / f.tiles_x;
        ix = tx * (f.tile_px / 2) - 1 + k % T2;
        iy = ty * (f.tile_px / 2) - 1 + k / T2;
        valid = k < T2 * T2 && ix >= 0 && iy >= 0 && ix < f.hw && iy < f.hh;
    } else {
        valid = pixel_of<false>(f, f.hw, f.hh, 1, ix, iy);
    }
    bool hit = false;
    const int p = iy * f.hw + ix;
    if (valid) {
        float x = ((float)ix + 0.5f) / (float)f.hw;
        float y = ((float)iy + 0.5f) / (float)f.hh;
        f3 dir = ray_dir(f, x, y);
        StepCount sc{};
        Hit h = trace<STATS>(w, f.pos, dir, 0.0f, sc);
        hit = h.hit;
        f.hdist[p] = (h.hit ? length(sub(h.pos, f.pos)) : 300.0f) - 8.0f;
        if (hit) f.pphit[p] = make_float4(h.pos.x, h.pos.y, h.pos.z, __uint_as_float(normal_code(h.normal)));
        else f.hshadow[p] = 1.0f;
        if (STATS) {
            c[CNT_TRACES]++; c[CNT_PP_PRIMARY]++; c[CNT_UNDEF] += h.undef;
            c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check;
        }
    }
    if (f.enq) enqueue_block<1>(f, {Q_PP}, {hit}, p);
    else enqueue(f, Q_PP, hit, p);
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

template <bool STATS>
__global__ void __launch_bounds__(256) k_wf_pp_shadow(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int p;
    if (queue_item(f, Q_PP, p)) {
        float4 hp = f.pphit[p];
        f3 pos = V(hp.x, hp.y, hp.z), nrm = normal_of(__float_as_uint(hp.w));
        StepCount sc{};
        Hit sh = trace_sun<STATS>(w, add(pos, scale(nrm, 1e-1f)), f.sun, 0.0f, sc);
        f.hshadow[p] = sh.hit ? SHADOW_HIT : 1.0f;
        if (STATS) {
            c[CNT_TRACES]++; c[CNT_PP_SHADOW]++;
            c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check;
        }
    }
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

// ------------------------------------------------------------ primary rays
template <bool STATS, bool TILES>
__global__ void __launch_bounds__(256) k_wf_primary(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int ix = 0, iy = 0;
    const bool valid = pixel_of<TILES>(f, f.W, f.H, 1, ix, iy);
    const int p = iy * f.W + ix;
    bool water = false, land = false;
    if (valid) {
        float x = (float)ix / (float)f.W, y = (float)iy / (float)f.H;
        float dist = (f.flags & RV_F_PREPASS) ? min_dist(f, x, y) : 0.0f;
        f3 dir = ray_dir(f, x, y);
        StepCount sc{};
        Hit h = trace<STATS>(w, f.pos, dir, hround(dist), sc);
        water = h.hit && h.pos.y < 31.001f && (f.flags & RV_F_WATER);
        land = h.hit && !water;
        uint32_t info = (h.hit ? HI_HIT : 0u) | (h.undef ? HI_UNDEF : 0u) | (water ? HI_WATER : 0u) |
                        (normal_code(h.normal) << HI_NSHIFT);
        f.hpos[p] = make_float4(h.pos.x, h.pos.y, h.pos.z, uv_bits(h.u, h.v));
        f.hinfo[p] = info;
        if (STATS) {
            c[CNT_TRACES]++; c[CNT_PRIMARY]++; c[CNT_UNDEF] += h.undef;
            c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check;
        }
    }
    const bool shadow = land && !(f.flags & RV_F_PREPASS) && (f.flags & RV_F_SHADOW);
    const bool cone = land && (f.flags & RV_F_GI);
    if (f.enq) {
        enqueue_block<3>(f, {Q_WATER, Q_SHADOW, Q_CONE}, {water, shadow, cone}, p);
    } else {
        enqueue(f, Q_WATER, water, p);
        enqueue(f, Q_SHADOW, shadow, p);
        enqueue(f, Q_CONE, cone, p);
    }
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

// ------------------------------------------------------------ secondary rays
template <bool STATS>
__global__ void __launch_bounds__(256) k_wf_shadow(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int p;
    if (queue_item(f, Q_SHADOW, p)) {
        float4 hp = f.hpos[p];
        uint32_t info = f.hinfo[p];
        f3 pos = V(hp.x, hp.y, hp.z), nrm = normal_of(info >> HI_NSHIFT);
        StepCount sc{};
        Hit sh = trace_sun<STATS>(w, add(pos, scale(nrm, 1e-1f)), f.sun, 0.0f, sc);
        if (sh.hit) f.hinfo[p] = info | HI_SHADOWED;
        if (STATS) {
            c[CNT_TRACES]++; c[CNT_SHADOW]++;
            c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check;
        }
    }
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

// water branch of computeColor (src/StateRender.cu:53-87) -> pre-fog colour
template <bool STATS>
__global__ void __launch_bounds__(256) k_wf_water(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int p;
    if (queue_item(f, Q_WATER, p)) {
        int ix = p % f.W, iy = p / f.W;
        float x = (float)ix / (float)f.W, y = (float)iy / (float)f.H;
        f3 dir = ray_dir(f, x, y);
        float4 hp = f.hpos[p];
        f3 hpos = V(hp.x, hp.y, hp.z), hn = normal_of(f.hinfo[p] >> HI_NSHIFT);
        float nxw = fbm3D(hpos.x, hpos.z, f.time, 3, 0.06f, 2.0f, 0.6f);
        float nyw = fbm3D(hpos.z, hpos.x, f.time + 112.0f, 3, 0.06f, 2.0f, 0.6f);
        f3 dn = normalize(add(hn, V(nxw * 0.1f, nyw * 0.1f, 0.0f)));
        f3 rdir = reflect(dir, dn);
        StepCount sc{};
        Hit rh = trace<STATS>(w, hpos, rdir, hround(0.001f), sc);
        f3 rc;
        if (rh.hit) {
            rc = sample_texture(w, rh.u, rh.v, rh.pos);
            Hit rs = trace_sun<STATS>(w, add(rh.pos, scale(rh.normal, 1e-3f)), f.sun, hround(0.001f), sc);
            if (rs.hit) rc = scale(rc, 0.1f);
        } else {
            rc = sample_sky(rdir, f.sun);
        }
        float ndv = fmaxf(dot(hn, neg(dir)), 0.0f);
        float fres = 0.08f + (1.0f - 0.08f) * pow5(1.0f - ndv);
        f3 col = lerp(V(0.0f, 0.1f, 0.3f), rc, fres);
        f.hsec[p] = make_float4(col.x, col.y, col.z, 0.0f);
        if (STATS) {
            c[CNT_TRACES] += 1 + rh.hit; c[CNT_REFL]++; c[CNT_REFL_SHADOW] += rh.hit; c[CNT_TEX] += rh.hit;
            c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check;
        }
    }
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

// the six cones of computeColor (src/StateRender.cu:101-115), summed in order
template <bool STATS>
__global__ void __launch_bounds__(256) k_wf_cones(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int p;
    if (queue_item(f, Q_CONE, p)) {
        float4 hp = f.hpos[p];
        f3 pos = V(hp.x, hp.y, hp.z), up = normal_of(f.hinfo[p] >> HI_NSHIFT);
        f3 right = normalize(cross(up, V(0.577f, 0.577f, 0.577f)));
        f3 fwd = normalize(cross(up, right));
        uint32_t steps = 0;
        f3 ind = trace_cone<STATS>(w, pos, up, steps);
        ind = add(ind, trace_cone<STATS>(w, pos, lerp(up, right, 0.5f), steps));
        ind = add(ind, trace_cone<STATS>(w, pos, lerp(up, neg(right), 0.5f), steps));
        ind = add(ind, trace_cone<STATS>(w, pos, lerp(up, fwd, 0.5f), steps));
        ind = add(ind, trace_cone<STATS>(w, pos, lerp(up, neg(fwd), 0.5f), steps));
        ind = add(ind, trace_cone<STATS>(w, pos, lerp(up, lerp(right, fwd, 0.5f), 0.5f), steps));
        f.hsec[p] = make_float4(ind.x, ind.y, ind.z, 0.0f);
        if (STATS) { c[CNT_CONES] += 6; c[CNT_CONE_STEPS] += steps; }
    }
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

// ------------------------------------------------------------ shade + outputs
template <bool STATS, bool TILES>
__global__ void __launch_bounds__(256) k_wf_shade(World w, FrameParams f) {
    uint32_t c[NCNT] = {};
    int ix = 0, iy = 0;
    const bool valid = pixel_of<TILES>(f, f.W, f.H, 1, ix, iy);
    if (valid) {
        const int p = iy * f.W + ix;
        const uint32_t info = f.hinfo[p];
        const float4 hp = f.hpos[p];
        const f3 hpos = V(hp.x, hp.y, hp.z);
        const bool hit = info & HI_HIT;
        float x = (float)ix / (float)f.W, y = (float)iy / (float)f.H;
        f3 color;
        if (info & HI_WATER) {
            float4 s = f.hsec[p];
            color = V(s.x, s.y, s.z);
        } else if (hit) {
            const uint32_t uvb = __float_as_uint(hp.w);
            f3 base = sample_texture(w, half_of(uvb & 0xFFFFu), half_of(uvb >> 16), hpos);
            if (STATS) c[CNT_TEX]++;
            f3 nrm = normal_of(info >> HI_NSHIFT);
            float shadow = 1.0f;
            if (f.flags & RV_F_PREPASS) shadow = bilinear_tex(f, x, y);
            else if (info & HI_SHADOWED) shadow = SHADOW_HIT;
            float diffuse = fmaxf(dot(nrm, f.sun), 0.0f);
            f3 direct = scale(scale(base, diffuse), shadow);
            if (f.flags & RV_F_GI) {
                float4 s = f.hsec[p];
                f3 ind = scale(mul(divs(V(s.x, s.y, s.z), 6.0f), base), 0.6f);
                f3 amb = mul(scale(sample_sky(nrm, f.sun), 0.05f), base);
                color = add(add(direct, ind), amb);
            } else {
                color = direct;
            }
        } else {
            color = sample_sky(ray_dir(f, x, y), f.sun);
        }
        float fog = hit ? fog_pow(length(sub(hpos, f.pos)) * 0.0004f) : 1.0f;
        f3 col = add(scale(color, fog), scale(V(0.95f, 0.95f, 1.0f), 1.0f - fog));
        float mvx = 0.0f, mvy = 0.0f, dep = 1.0f;
        if (hit) {   // mat_mul_vec (cumath.cuh:47-54), glm column-major
            const float* P = f.pvp;
            const float* M = f.vp;
            float pc[4], cc[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                pc[r] = P[r] * hpos.x + P[4 + r] * hpos.y + P[8 + r] * hpos.z + P[12 + r] * 1.0f;
                cc[r] = M[r] * hpos.x + M[4 + r] * hpos.y + M[8 + r] * hpos.z + M[12 + r] * 1.0f;
            }
            if (pc[3] > 0.0f && cc[3] > 0.0f) {
                mvx = cc[0] / cc[3] - pc[0] / pc[3];
                mvy = cc[1] / cc[3] - pc[1] / pc[3];
            }
            if (cc[3] > 0.0f) dep = cc[2] / cc[3];
        }
        col.x = fminf(fmaxf(col.x, 0.0f), 1.0f);
        col.y = fminf(fmaxf(col.y, 0.0f), 1.0f);
        col.z = fminf(fmaxf(col.z, 0.0f), 1.0f);
        uint32_t px = (uint32_t)(uint8_t)(col.x * 255.0f) | ((uint32_t)(uint8_t)(col.y * 255.0f) << 8) |
                      ((uint32_t)(uint8_t)(col.z * 255.0f) << 16) | 0xFF000000u;
        if (TILES) {
            int lx = ix % f.tile_px, ly = iy % f.tile_px;
            f.tilebuf[((size_t)blockIdx.y * f.tile_px + ly) * f.tile_px + lx] = px;
        } else {
            *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(f.color) + (size_t)iy * f.color_pitch +
                                         4 * (size_t)ix) = px;
        }
        if (f.mv) {
            uint32_t m = (uint32_t)hbits(mvx) | ((uint32_t)hbits(-mvy) << 16);
            *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(f.mv) + (size_t)iy * f.mv_pitch + 4 * (size_t)ix) = m;
        }
        if (f.depth)
            *reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(f.depth) + (size_t)iy * f.depth_pitch +
                                         2 * (size_t)ix) = hbits(dep);
    } else if (TILES) {
        // keep the packed tile buffer fully defined past the image edge
        int T = f.tile_px;
        uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        int nb = T >> 4;
        int lx = (int)((blockIdx.x % nb) * 16 + (wave & 1) * 8 + (lane & 7));
        int ly = (int)((blockIdx.x / nb) * 16 + (wave >> 1) * 8 + (lane >> 3));
        if (lx < T && ly < T) f.tilebuf[((size_t)blockIdx.y * T + ly) * T + lx] = 0u;
    }
    if (STATS) block_count_flush<NCNT>(f.counters, c);
}

// ================================================================ launchers
template <typename K>
static void launch_queue_kernel(hipStream_t s, K kernel, const World& w, const FrameParams& f, int q) {
    // NXCD workgroups per 256 sub-queue slots; the queue lengths are only
    // known on the device, so workgroups past them exit at once.
    uint32_t g = NXCD * ((f.qcap[q] + 255) / 256);
    if (g == 0) g = NXCD;
    hipLaunchKernelGGL(kernel, dim3(g), dim3(256), 0, s, w, f);
}

static uint32_t full_grid(const FrameParams& f, int W, int H) {
    return sched_grid<16, 16>(f.sched, W, H);
}

uint32_t wf_producer_blocks(const FrameParams& f, int q, bool tiles) {
    FrameParams g = f;
    if (g.sched == SCHED_COST) g.sched = SCHED_CHUNK;   // no cost feedback for the stage kernels
    if (q == Q_PP) {
        if (!tiles) return full_grid(g, f.hw, f.hh);
        int T2 = f.tile_px / 2 + 2;
        return (uint32_t)((T2 * T2 + 255) / 256) * (uint32_t)f.ntiles;
    }
    if (!tiles) return full_grid(g, f.W, f.H);
    int nb = (f.tile_px + 15) >> 4;
    return (uint32_t)(nb * nb) * (uint32_t)f.ntiles;
}

void launch_wf_pp_primary(hipStream_t s, const World& w, const FrameParams& f, bool tiles) {
    const bool st = (f.flags & RV_F_STATS) != 0;
    FrameParams g = f;
    if (g.sched == SCHED_COST) g.sched = SCHED_CHUNK;   // no cost feedback for the stage kernels
    if (tiles) {
        if (f.ntiles <= 0) return;
        int T2 = f.tile_px / 2 + 2;
        dim3 grid((uint32_t)((T2 * T2 + 255) / 256), (uint32_t)f.ntiles);
        if (st) hipLaunchKernelGGL((k_wf_pp_primary<true, true>), grid, dim3(256), 0, s, w, g);
        else hipLaunchKernelGGL((k_wf_pp_primary<false, true>), grid, dim3(256), 0, s, w, g);
    } else {
        dim3 grid(full_grid(g, f.hw, f.hh));
        if (st) hipLaunchKernelGGL((k_wf_pp_primary<true, false>), grid, dim3(256), 0, s, w, g);
        else hipLaunchKernelGGL((k_wf_pp_primary<false, false>), grid, dim3(256), 0, s, w, g);
    }
}

void launch_wf_pp_shadow(hipStream_t s, const World& w, const FrameParams& f) {
    if (f.flags & RV_F_STATS) launch_queue_kernel(s, k_wf_pp_shadow<true>, w, f, Q_PP);
    else launch_queue_kernel(s, k_wf_pp_shadow<false>, w, f, Q_PP);
}

void launch_wf_primary(hipStream_t s, const World& w, const FrameParams& f, bool tiles) {
    const bool st = (f.flags & RV_F_STATS) != 0;
    FrameParams g = f;
    if (g.sched == SCHED_COST) g.sched = SCHED_CHUNK;   // no cost feedback for the stage kernels
    if (tiles) {
        if (f.ntiles <= 0) return;
        int nb = (f.tile_px + 15) >> 4;
        dim3 grid((uint32_t)(nb * nb), (uint32_t)f.ntiles);
        if (st) hipLaunchKernelGGL((k_wf_primary<true, true>), grid, dim3(256), 0, s, w, g);
        else hipLaunchKernelGGL((k_wf_primary<false, true>), grid, dim3(256), 0, s, w, g);
    } else {
        dim3 grid(full_grid(g, f.W, f.H));
        if (st) hipLaunchKernelGGL((k_wf_primary<true, false>), grid, dim3(256), 0, s, w, g);
        else hipLaunchKernelGGL((k_wf_primary<false, false>), grid, dim3(256), 0, s, w, g);
    }
}

void launch_wf_shadow(hipStream_t s, const World& w, const FrameParams& f) {
    if (f.flags & RV_F_STATS) launch_queue_kernel(s, k_wf_shadow<true>, w, f, Q_SHADOW);
    else launch_queue_kernel(s, k_wf_shadow<false>, w, f, Q_SHADOW);
}

void launch_wf_water(hipStream_t s, const World& w, const FrameParams& f) {
    if (f.flags & RV_F_STATS) launch_queue_kernel(s, k_wf_water<true>, w, f, Q_WATER);
    else launch_queue_kernel(s, k_wf_water<false>, w, f, Q_WATER);
}

void launch_wf_cones(hipStream_t s, const World& w, const FrameParams& f) {
    if (f.flags & RV_F_STATS) launch_queue_kernel(s, k_wf_cones<true>, w, f, Q_CONE);
    else launch_queue_kernel(s, k_wf_cones<false>, w, f, Q_CONE);
}

void launch_wf_shade(hipStream_t s, const World& w, const FrameParams& f, bool tiles) {
    const bool st = (f.flags & RV_F_STATS) != 0;
    FrameParams g = f;
    if (g.sched == SCHED_COST) g.sched = SCHED_CHUNK;   // no cost feedback for the stage kernels
    if (tiles) {
        if (f.ntiles <= 0) return;
        int nb = (f.tile_px + 15) >> 4;
        dim3 grid((uint32_t)(nb * nb), (uint32_t)f.ntiles);
        if (st) hipLaunchKernelGGL((k_wf_shade<true, true>), grid, dim3(256), 0, s, w, g);
        else hipLaunchKernelGGL((k_wf_shade<false, true>), grid, dim3(256), 0, s, w, g);
    } else {
        dim3 grid(full_grid(g, f.W, f.H));
        if (st) hipLaunchKernelGGL((k_wf_shade<true, false>), grid, dim3(256), 0, s, w, g);
        else hipLaunchKernelGGL((k_wf_shade<false, false>), grid, dim3(256), 0, s, w, g);
    }
}

}  // namespace rv
