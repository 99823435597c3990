// rv_shade.h -- the per-pixel device bodies of the frame: distApproximationKernel's
// half-res pixel (prepass_pixel), computeColor (compute_color) and renderKernel's pixel
// (render_pixel), templated on the world view.  Included by the product kernels
// (rv_kernels.hip: World, WorldOv) and by the reference-signature kernels of
// include/rvgrt_kernels.h (LinearWorld: the reference's own buffer layouts), so both run the
// same code.
#pragma once
#include "rv_frame.h"

// Traversal variant (trace<COUNT, G, REUSE>, rv_device.h) of each launch kind:
// G = DDA look-ahead group, REUSE = skip the gather while its address is
// unchanged.  Defaults from the round-1 measurements.
#ifndef RV_G_FRAME        // C1/C2 frames and other feature sets: look-ahead 4 since the round-2
#define RV_G_FRAME 4      // traversal diet (round 1: 1; C2 0.131 -> 0.114 ms, C1 -5 %, profiles/r02/lookahead_ab.txt)
#endif
#ifndef RV_REUSE_FRAME
#define RV_REUSE_FRAME 0
#endif
#ifndef RV_G_REF          // the reference frame (C3-C5)
#define RV_G_REF 4
#endif
#ifndef RV_G_PREPASS      // distApproximationKernel: the longest chains (camera ray + shadow ray)
#define RV_G_PREPASS 8    // 8 (68 VGPRs: the pipelined launch at 7 waves/SIMD) beats 4 at 8 waves:
#endif                    // C4 0.535 -> 0.512 ms, C5 0.782 -> 0.731, C3 -1.5 % (profiles/r02/lookahead_ab.txt)
#ifndef RV_LATE_MATRICES  // pipelined launch: load the MV/depth matrices where they are used (SGPR pressure)
#define RV_LATE_MATRICES 1   // 106 -> 97 SGPRs, 7 -> 8 waves/SIMD: C4 0.631 -> 0.603 ms (profiles/r02/rewalk_ab.txt)
#endif
#ifndef RV_HALF_WINDOW    // minDist / bilinear taps from an LDS window of the wave's half-res texels
#define RV_HALF_WINDOW 0   // measured C4 0.678 (off) vs 0.688 ms (on), C3 equal: the taps are not the limit
#endif
#ifndef RV_G_REFL         // the water reflection ray's look-ahead (0: the frame's G); A/B builds
#define RV_G_REFL 0
#endif
#ifndef RV_COL_REFL       // the water reflection's DDA skips the voxel gathers of groups above the terrain
#define RV_COL_REFL 1     // (rv_device.h trace COL)
#endif
#ifndef RV_COL_PRIMARY    // ... the camera rays (render and pre-pass) too (A/B)
#define RV_COL_PRIMARY 0
#endif
#ifndef RV_COL_GI         // ... the GI update's bounce rays too (A/B)
#define RV_COL_GI 0
#endif
#ifndef RV_G_GI           // GI init / update
#define RV_G_GI 4
#endif

namespace rv {

#ifndef RV_REFL_DIAG   // diagnostics builds: the reflection rays' step counts per wave in STATS frames
#define RV_REFL_DIAG 0
#endif
#if RV_REFL_DIAG
// [0] lanes, [1] waves, [2] sum of lane steps (sphere + DDA), [3] sum over waves of the wave's longest,
// [4 + b] sum over waves of min(longest, B), [8 + b] sum over lanes of max(steps - B, 0), B = 16 << b
static __device__ unsigned long long rv_refl_diag_buf[12];
__device__ inline void refl_diag_add(uint32_t n) {
    uint64_t m = __ballot(1);
    const int first = __builtin_ctzll(m);
    unsigned long long v[12] = {};
    while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)n, l);
        v[0] += 1; v[2] += x; v[3] = v[3] > x ? v[3] : x;
        for (int b = 0; b < 4; b++) v[8 + b] += x > (16u << b) ? x - (16u << b) : 0u;
    }
    v[1] = 1;
    for (int b = 0; b < 4; b++) v[4 + b] = v[3] < (16u << b) ? v[3] : (16u << b);
    if ((int)(threadIdx.x & 63u) == first)
        for (int i = 0; i < 12; i++) atomicAdd(&rv_refl_diag_buf[i], v[i]);
}
#endif

// one half-res pixel of distApproximationKernel (StateRender.cu:255-286): its distance (d - 8, the
// value stored) and shadow texels
// G: the traversal's DDA look-ahead (every G gives the same hit: rv_device.h trace)
struct NoPublish { __device__ void operator()(float) const {} };
// on_dist(d - 8): called once the camera ray is done, before the shadow ray (the flow launch publishes the
// distance there: the two-phase hand-off, rv_kernels.hip flow_pre_part)
template <bool STATS, class WV = World, int G = RV_G_PREPASS, class PUB = NoPublish>
__device__ __forceinline__ void prepass_eval(const WV& w, const FrameParams& f, int ix, int iy,
                                             uint32_t (&c)[NCNT], float& dist_out, float& shadow_out,
                                             const PUB& on_dist = PUB()) {
    float x = ((float)ix + 0.5f) / (float)f.hw;
    float y = ((float)iy + 0.5f) / (float)f.hh;
    f3 dir = ray_dir(f, x, y);
    StepCount sc{};
    RV_GD_KIND(gd::PP_PRIMARY);
    Hit h = trace<STATS, G, false, (RV_DDA_REWALK != 0), false, WV, RV_COL_PRIMARY && (G > 1) && RV_DDA_REWALK>(
        w, f.pos, dir, 0.0f, sc);
    float d = h.hit ? length(sub(h.pos, f.pos)) : 300.0f;
    float s = 1.0f;
    on_dist(d - 8.0f);
    if (STATS) { c[CNT_TRACES]++; c[CNT_PP_PRIMARY]++; c[CNT_UNDEF] += h.undef; }
    if (h.hit) {
        RV_GD_KIND(gd::PP_SHADOW);
        Hit sh = trace_sun<STATS, G, false, WV, (RV_COL_SUN != 0) && (G > 1) && (RV_DDA_REWALK != 0)>(
            w, add(h.pos, scale(h.normal, 1e-1f)), f.sun, 0.0f, sc);
        s = sh.hit ? SHADOW_HIT : 1.0f;
        if (STATS) { c[CNT_TRACES]++; c[CNT_PP_SHADOW]++; }
    }
    if (STATS) { c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check; }
    dist_out = d - 8.0f;
    shadow_out = s;
}
template <bool STATS, class WV = World>
__device__ __forceinline__ void prepass_pixel(const WV& w, const FrameParams& f, int ix, int iy,
                                              uint32_t (&c)[NCNT]) {
    float d, s;
    prepass_eval<STATS, WV>(w, f, ix, iy, c, d, s);
    f.hdist[(size_t)iy * f.hw + ix] = d;
    f.hshadow[(size_t)iy * f.hw + ix] = s;
}

// Frame outputs: an 8x8-pixel wave writes 32-B (colour, motion) and 16-B (depth) row pieces.
// Plain stores (default) let L2 merge the pieces of neighbouring waves into whole lines: HBM
// writes = the image bytes (C2 21.0 MiB per 1080p frame of 19.8 MiB images, C4 107 MiB per 4K
// frame incl. half-res and GI).  RV_NT_STORES=1 (non-temporal) keeps the images from displacing
// the world's bricks in L2 (C2 reads 15.8 -> 2.5 MiB/frame) but each piece then reaches memory
// alone: 2.72x the image bytes on C2, 2.1x on C4, for C2 -1.5 %, C3/C4 within 1 %
// (profiles/r02/nt_stores_ab.txt).
#ifndef RV_NT_STORES
#define RV_NT_STORES 0
#endif
template <typename T>
__device__ __forceinline__ void out_store(T* p, T v) {
    if (RV_NT_STORES) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// Frame kernels are instantiated per feature set: FEAT = the RV_F_* bits the
// frame uses, known at compile time, so a C2 frame (shadow only) carries
// neither the water nor the cone-tracing code and their registers; FEAT_DYN
// reads the bits from FrameParams (any other combination).
static constexpr uint32_t FEAT_DYN = 0xFFFFFFFFu;
static constexpr uint32_t FEAT_MASK = RV_F_PREPASS | RV_F_WATER | RV_F_GI | RV_F_SHADOW;
template <uint32_t FEAT>
__device__ __forceinline__ bool has(const FrameParams& f, uint32_t bit) {
    return FEAT == FEAT_DYN ? (f.flags & bit) != 0 : (FEAT & bit) != 0;
}

// Traversal variant per frame kind (rv_device.h trace<>): latency-bound
// launches (the pre-pass, the reference frame's secondary rays, the GI
// update: few or incoherent waves) take the DDA look-ahead; the C1/C2 frame
// is throughput bound and does not.  Measured in DESIGN.md s5.
template <uint32_t FEAT> struct TraceCfg {
    static constexpr bool REF = FEAT == (uint32_t)(RV_F_PREPASS | RV_F_WATER | RV_F_GI);
    static constexpr int G = REF ? RV_G_REF : RV_G_FRAME;
    static constexpr bool REUSE = !REF && RV_REUSE_FRAME;
};

// The land branch's indirect light (StateRender.cu:100-127): the 6 cones of a hit (up, lerp(up, +-right,
// .5), lerp(up, +-fwd, .5), lerp(up, lerp(right, fwd, .5), .5) -- not normalised, R12) from the GI grid,
// their first-step gathers issued together (trace_cones6), and the sky ambient.
template <bool STATS, int CB, class WV>
__device__ __forceinline__ void cone_lighting(const WV& w, const FrameParams& f, const Hit& hit, f3 base,
                                              uint32_t (&c)[NCNT], f3& ind, f3& amb) {
    f3 up = hit.normal;
    f3 right, fwd;
    if ((up.x != 0.0f) | (up.y != 0.0f) | (up.z != 0.0f)) {   // axis normal: constant scales
        right = scale(cross(up, V(0.577f, 0.577f, 0.577f)), f.cone_k1);
        fwd = scale(cross(up, right), f.cone_k2);
    } else {
        right = normalize(cross(up, V(0.577f, 0.577f, 0.577f)));
        fwd = normalize(cross(up, right));
    }
    uint32_t steps = 0;
    ind = trace_cones6<STATS, CB>(w, hit.pos, up, right, fwd, steps);
    if (STATS) { c[CNT_CONES] += 6; c[CNT_CONE_STEPS] += steps; }
    ind = scale(mul(divs(ind, 6.0f), base), 0.6f);
    amb = mul(scale(sample_sky(hit.normal, f.sun), 0.05f), base);
}

// computeColor (StateRender.cu:33-146)
// COLOK: the launch may take the water reflection's column skip (k_ref_flow: no -- its render waits inside
// the launch and the skip's registers cost it 3.5 %, profiles/r04/col_skip_atlas_ab.txt)
// DS (k_ref_flow): the pre-pass shadow is fetched only where the land branch uses it, after the cones
// (bilinear_tex over hwin once resolve_shadow_taps has its texels): the render's primary and secondary
// rays run while the pre-pass lanes still trace their shadow rays.  Same arithmetic either way.
template <bool STATS, uint32_t FEAT, int CB = RV_CONE_GROUP, int GR = 0, class WV = World, bool COLOK = true,
          bool DS = false>
__device__ __forceinline__ f3 compute_color(const WV& w, const FrameParams& f, float x, float y,
                                            float dist, float shadow_in, Hit& hit, uint32_t (&c)[NCNT],
                                            const HalfWin* hwin = nullptr) {
    const bool prepass = has<FEAT>(f, RV_F_PREPASS);
    f3 dir = ray_dir(f, x, y);
    StepCount sc{};
    constexpr int G = GR ? GR : TraceCfg<FEAT>::G;
    constexpr bool RE = TraceCfg<FEAT>::REUSE;
    RV_GD_KIND(gd::PRIMARY);
    hit = trace<STATS, G, RE, (RV_DDA_REWALK != 0), false, WV, RV_COL_PRIMARY && GR == 0 && (G > 1) && RV_DDA_REWALK>(
        w, f.pos, dir, hround(dist), sc);
    if (STATS) { c[CNT_TRACES]++; c[CNT_PRIMARY]++; c[CNT_UNDEF] += hit.undef; }
    f3 color;
    if (hit.hit && hit.pos.y < 31.001f && has<FEAT>(f, RV_F_WATER)) {
        float nxw = fbm3D(hit.pos.x, hit.pos.z, f.time, 3, 0.06f, 2.0f, 0.6f);
        float nyw = fbm3D(hit.pos.z, hit.pos.x, f.time + 112.0f, 3, 0.06f, 2.0f, 0.6f);
        f3 dn = normalize(add(hit.normal, V(nxw * 0.1f, nyw * 0.1f, 0.0f)));
        f3 rdir = reflect(dir, dn);
        RV_GD_KIND(gd::REFL);
        constexpr int GG = RV_G_REFL ? RV_G_REFL : G;
        constexpr bool COLR = RV_COL_REFL && (GG > 1) && RV_DDA_REWALK && GR == 0 && COLOK;   // throughput launches
#if RV_REFL_DIAG
        const uint32_t s0 = sc.sphere + sc.dda;
#endif
        Hit rh = trace<STATS, GG, RE, (RV_DDA_REWALK != 0), false, WV, COLR>(w, hit.pos, rdir, hround(0.001f), sc);
#if RV_REFL_DIAG
        if (STATS) refl_diag_add(sc.sphere + sc.dda - s0);
#endif
        if (STATS) { c[CNT_TRACES]++; c[CNT_REFL]++; }
        f3 rc;
        if (rh.hit) {
            rc = sample_texture(w, rh.u, rh.v, rh.pos);
            RV_GD_KIND(gd::REFL_SHADOW);
            Hit rs = trace_sun<STATS, G, RE>(w, add(rh.pos, scale(rh.normal, 1e-3f)), f.sun, hround(0.001f), sc);
            if (STATS) { c[CNT_TRACES]++; c[CNT_REFL_SHADOW]++; c[CNT_TEX]++; }
            if (rs.hit) rc = scale(rc, 0.1f);
        } else {
            rc = sample_sky(rdir, f.sun);
        }
        float ndv = fmaxf(dot(hit.normal, neg(dir)), 0.0f);
        float fres = 0.08f + (1.0f - 0.08f) * pow5(1.0f - ndv);
        color = lerp(V(0.0f, 0.1f, 0.3f), rc, fres);
    } else if (hit.hit) {
        f3 base = sample_texture(w, hit.u, hit.v, hit.pos);
        if (STATS) c[CNT_TEX]++;
        float shadow = shadow_in;
        if (!prepass) {
            shadow = 1.0f;
            if (has<FEAT>(f, RV_F_SHADOW)) {
                RV_GD_KIND(gd::SHADOW);
                Hit sh = trace_sun<STATS, G, RE>(w, add(hit.pos, scale(hit.normal, 1e-1f)), f.sun, 0.0f, sc);
                if (STATS) { c[CNT_TRACES]++; c[CNT_SHADOW]++; }
                shadow = sh.hit ? SHADOW_HIT : 1.0f;
            }
        }
        float diffuse = fmaxf(dot(hit.normal, f.sun), 0.0f);
        f3 ind, amb;
        const bool gi = has<FEAT>(f, RV_F_GI);
        if (gi) cone_lighting<STATS, CB>(w, f, hit, base, c, ind, amb);   // DS: the cones before the shadow taps
        if (DS && prepass) {
            resolve_shadow_taps(f, x, y, hwin);
            shadow = bilinear_tex(f, x, y, hwin);
        }
        f3 direct = scale(scale(base, diffuse), shadow);
        color = gi ? add(add(direct, ind), amb) : direct;
    } else {
        color = sample_sky(dir, f.sun);
    }
    if (STATS) { c[CNT_SPHERE] += sc.sphere; c[CNT_DDA] += sc.dda; c[CNT_CHECK] += sc.check; }
    float fog = hit.hit ? fog_pow(length(sub(hit.pos, f.pos)) * 0.0004f) : 1.0f;
    return add(scale(color, fog), scale(V(0.95f, 0.95f, 1.0f), 1.0f - fog));
}

// previous / current clip positions of a hit (mat_mul_vec, cumath.cuh:47-54)
// LATE (the pipelined launch): an opaque zero defined here offsets the matrix pointers, so the
// 32 matrix floats (kernel arguments) load after the traversal instead of at kernel entry and
// do not hold 32 SGPRs through the whole launch (106 -> 96 SGPRs: 8 waves/SIMD instead of 7).
// Not for kernels that modify their FrameParams copy (k_render): the dynamic offset into it
// would put the copy in scratch.
template <bool LATE = false>
__device__ __forceinline__ void clip_pos(const float* P, const float* M, f3 p, float (&pc)[4], float (&cc)[4]) {
    if (LATE) {
        uint32_t z;
        asm volatile("s_mov_b32 %0, 0" : "=s"(z));
        P += z;
        M += z;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        pc[r] = P[r] * p.x + P[4 + r] * p.y + P[8 + r] * p.z + P[12 + r] * 1.0f;
        cc[r] = M[r] * p.x + M[4 + r] * p.y + M[8 + r] * p.z + M[12 + r] * 1.0f;
    }
}

// renderKernel body for one pixel (StateRender.cu:200-253); returns RGBA8
template <bool STATS, uint32_t FEAT, bool CAMS = false, bool LATE = false, int CB = RV_CONE_GROUP, int GR = 0,
          class WV = World, bool COLOK = true, bool DS = false>
__device__ __forceinline__ uint32_t render_pixel(const WV& w, const FrameParams& f, int ix, int iy,
                                                 uint32_t (&c)[NCNT], const HalfWin* hwin = nullptr) {
    float x = (float)ix / (float)f.W, y = (float)iy / (float)f.H;
    float dist = 0.0f, shadow = 1.0f;
    if (has<FEAT>(f, RV_F_PREPASS)) {
        dist = min_dist(f, x, y, hwin);
        if (!DS) shadow = bilinear_tex(f, x, y, hwin);   // DS: where the land branch uses it (compute_color)
    }
    Hit h;
    f3 col = compute_color<STATS, FEAT, CB, GR, WV, COLOK, DS>(w, f, x, y, dist, shadow, h, c, hwin);
    float mvx = 0.0f, mvy = 0.0f, dep = 1.0f;
    if (h.hit) {   // mat_mul_vec (cumath.cuh:47-54), glm column-major
        float pc[4], cc[4];
        if (CAMS && f.cam) clip_pos(f.cam->pvp, f.cam->vp, h.pos, pc, cc);   // per-frame table of a batched launch
        else clip_pos<LATE>(f.pvp, f.vp, h.pos, pc, cc);
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
    RV_GD_KIND(gd::OUTPUT);
    RV_GD(0, reinterpret_cast<char*>(f.mv) + (size_t)iy * f.mv_pitch + 4 * (size_t)ix);
    RV_GD(1, reinterpret_cast<char*>(f.depth) + (size_t)iy * f.depth_pitch + 2 * (size_t)ix);
    RV_GD(2, reinterpret_cast<char*>(f.color) + (size_t)iy * f.color_pitch + 4 * (size_t)ix);
    // images are < 4 GiB: 32-bit byte offsets on the SGPR base
    if (f.mv) {
        uint32_t m = (uint32_t)hbits(mvx) | ((uint32_t)hbits(-mvy) << 16);
        out_store(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(f.mv) + ((uint32_t)iy * (uint32_t)f.mv_pitch + 4u * (uint32_t)ix)), m);
    }
    if (f.depth) {
        out_store(reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(f.depth) + ((uint32_t)iy * (uint32_t)f.depth_pitch + 2u * (uint32_t)ix)),
                  hbits(dep));
    }
    return px;
}

}  // namespace rv
