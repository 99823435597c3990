/*
 * rvgrt_device.h -- the reference's __device__ traversal/shading API for HIP
 * kernels on gfx950, with the reference's names, signatures and hitInfo
 * layout, over reference-layout buffers.
 *
 * Reference interface replaced (include/raytracing_functions.cuh):
 *   struct hitInfo                                   :14-21
 *   IsSolid(int3, bits)                              :23-26
 *   getDistance(float3, csdf) / getDistance(int3, csdf)   :35-67
 *   approximateCSDF(float3, float3, csdf)            :69  (src/raytracing_functions.cu:65-83)
 *   trace(float3, float3, half, bits, csdf)          :71-72 (src/raytracing_functions.cu:85-202)
 *   traceCone(float3, float3, const float4*, csdf)   :74-75 (declared, never defined upstream)
 *   traceCone(float3, float3, const uchar4*, csdf)   :77-80 (src/raytracing_functions.cu:212-273)
 *   sampleSky(float3, float3)                        :83  (src/raytracing_functions.cu:10-26)
 *   sampleTexture(half2, float3, <atlas>)            :84  (src/raytracing_functions.cu:28-62)
 *   toIndex(int3) / toIndex(x, y, z)                 include/cumath.cuh:33-45
 *
 * Buffers are the reference's own layouts, so reference-style kernels can
 * keep their arguments: bits = uint32 words with bit index
 * x | y<<SHIX | z<<(SHIX+SHIY); csdf = uint8 (X/2)(Y/2)(Z/2) x fastest;
 * GI = uchar4 (X/4)(Y/4)(Z/4) x fastest.  The world dimensions are
 * compile-time, as in the reference (include/cumath.cuh:19-21): define
 * RVGRT_SHIX / RVGRT_SHIY / RVGRT_SHIZ before including (default 12, 9, 12 =
 * the reference's 4096 x 512 x 4096; SHIX >= 5).
 *
 * The texture atlas is not a texture object here: sampleTexture takes an
 * rvgrtAtlas (RGBA8 device array, 256 x 256 in the reference) and performs
 * the point / wrap / normalized-coordinate fetch of the reference's texture
 * descriptor (src/Texturepack.cu:105-111) exactly in arithmetic.
 *
 * The implementation is the library's traversal (include/rvgrt/rv_device.h)
 * instantiated on the reference layout; results are bit-identical with the
 * CPU oracle (tests/test_gpu_devapi.py).  Compile with -ffp-contract=off, as
 * the library is, for bit-exact results.
 */
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "rvgrt/rv_device.h"

#ifndef RVGRT_SHIX
#define RVGRT_SHIX 12
#endif
#ifndef RVGRT_SHIY
#define RVGRT_SHIY 9
#endif
#ifndef RVGRT_SHIZ
#define RVGRT_SHIZ 12
#endif
static_assert(RVGRT_SHIX >= 5, "the x-fastest bit words need SHIX >= 5");
static_assert(RVGRT_SHIX + RVGRT_SHIY + RVGRT_SHIZ <= 34, "32-bit word offsets: at most 2^34 voxels");

/* include/raytracing_functions.cuh:14-21 -- layout preserved: 36 bytes */
struct hitInfo {
    float3 pos;
    float3 normal;
    __half2 uv;
    bool hit;
    int its;
};
static_assert(sizeof(hitInfo) == 36, "hitInfo is 36 B in the reference");
static_assert(offsetof(hitInfo, pos) == 0 && offsetof(hitInfo, normal) == 12 && offsetof(hitInfo, uv) == 24 &&
                  offsetof(hitInfo, hit) == 28 && offsetof(hitInfo, its) == 32,
              "hitInfo field offsets");

/* Texture atlas in device memory (the reference's cudaTextureObject_t). */
struct rvgrtAtlas {
    const uint32_t* rgba8;  /* row-major RGBA8 */
    int width, height;      /* 256 x 256 in the reference */
};

namespace rvgrt_dev {
constexpr uint64_t SHIX = RVGRT_SHIX, SHIY = RVGRT_SHIY, SHIZ = RVGRT_SHIZ;
constexpr uint64_t MODX = (1ull << SHIX) - 1, MODY = (1ull << SHIY) - 1, MODZ = (1ull << SHIZ) - 1;

__device__ __forceinline__ rv::LinearWorld world(const uint32_t* bits, const unsigned char* csdf,
                                                 const uint32_t* gi = nullptr, rvgrtAtlas atlas = {nullptr, 256, 256}) {
    return rv::linear_world(RVGRT_SHIX, RVGRT_SHIY, RVGRT_SHIZ, bits, csdf, gi, atlas.rgba8, atlas.width,
                            atlas.height);
}
__device__ __forceinline__ rv::f3 F3(float3 v) { return rv::V(v.x, v.y, v.z); }
__device__ __forceinline__ float3 T3(rv::f3 v) { return make_float3(v.x, v.y, v.z); }

/* GI view over a float4 radiance grid (traceCone's first overload) */
struct RadianceWorld : rv::LinearWorld {
    const float4* rad;
};
__device__ __forceinline__ float4 gi_radiance(const RadianceWorld& w, uint64_t idx) { return w.rad[idx]; }
}  // namespace rvgrt_dev

/* include/cumath.cuh:33-45 */
__device__ __forceinline__ uint64_t toIndex(int3 p) {
    using namespace rvgrt_dev;
    return (((uint64_t)p.x) & MODX) | ((((uint64_t)p.y) & MODY) << SHIX) | ((((uint64_t)p.z) & MODZ) << (SHIX + SHIY));
}
__device__ __forceinline__ uint64_t toIndex(uint64_t x, uint64_t y, uint64_t z) {
    using namespace rvgrt_dev;
    return (x & MODX) | ((y & MODY) << SHIX) | ((z & MODZ) << (SHIX + SHIY));
}

/* include/raytracing_functions.cuh:23-26 (coordinates wrap, as toIndex does) */
__device__ __forceinline__ bool IsSolid(int3 p, const uint32_t* __restrict__ bits) {
    const uint64_t index = toIndex(p);
    return (bits[index >> 5] >> (index & 31)) & 1;
}

/* include/raytracing_functions.cuh:35-51 */
__device__ __forceinline__ float getDistance(float3 pos, const unsigned char* __restrict__ csdf) {
    return rv::get_distance_f(rvgrt_dev::world(nullptr, csdf), rvgrt_dev::F3(pos));
}
/* include/raytracing_functions.cuh:52-67 */
__device__ __forceinline__ unsigned char getDistance(int3 pos, const unsigned char* __restrict__ csdf) {
    return (unsigned char)rv::get_distance_i(rvgrt_dev::world(nullptr, csdf), pos.x, pos.y, pos.z);
}

/* src/raytracing_functions.cu:65-83 */
__device__ __forceinline__ float3 approximateCSDF(float3 pos, float3 dir, const unsigned char* __restrict__ csdf) {
    const rv::LinearWorld w = rvgrt_dev::world(nullptr, csdf);
    rv::f3 p = rvgrt_dev::F3(pos);
    const rv::f3 d = rvgrt_dev::F3(dir);
    for (int it = 0; it < 100; it++) {
        if (p.x < 0 || p.y < 0 || p.z < 0 || p.x >= (float)w.X || p.y >= (float)w.Y || p.z >= (float)w.Z)
            return make_float3(-100.0f, -100.0f, -100.0f);
        const float dist = rv::get_distance_f(w, p);
        if (dist <= 1.0f) return rvgrt_dev::T3(p);
        p = rv::add(p, rv::scale(d, dist));
    }
    return rvgrt_dev::T3(p);
}

/* src/raytracing_functions.cu:85-202.  An undefined reference hit
 * (mask == -128) has pos (-500)^3 and normal / uv 0. */
__device__ __forceinline__ hitInfo trace(float3 camPos, float3 camDir, __half distance,
                                         const uint32_t* __restrict__ bits, const unsigned char* __restrict__ csdf) {
    rv::StepCount sc{};
    const rv::Hit h = rv::trace<true, 1, false>(rvgrt_dev::world(bits, csdf), rvgrt_dev::F3(camPos),
                                                rvgrt_dev::F3(camDir), __half2float(distance), sc);
    hitInfo r;
    r.pos = rvgrt_dev::T3(h.pos);
    r.normal = rvgrt_dev::T3(h.normal);
    r.uv = __floats2half2_rn(h.u, h.v);   /* exact: u, v are already half values */
    r.hit = h.hit;
    r.its = (int)sc.its;
    return r;
}

/* src/raytracing_functions.cu:212-273 */
__device__ __forceinline__ float3 traceCone(float3 pos, float3 dir, const uchar4* __restrict__ GIdata,
                                            const unsigned char* __restrict__ csdf) {
    uint32_t steps = 0;
    return rvgrt_dev::T3(rv::trace_cone<false>(
        rvgrt_dev::world(nullptr, csdf, reinterpret_cast<const uint32_t*>(GIdata)), rvgrt_dev::F3(pos),
        rvgrt_dev::F3(dir), steps));
}

/* include/raytracing_functions.cuh:74-75: the float4 radiance-grid overload
 * (declared upstream, never defined); the same march with the texel taken as
 * colour xyz, alpha w instead of RGBA8 / 255. */
__device__ __forceinline__ float3 traceCone(float3 pos, float3 dir, const float4* __restrict__ radianceVoxels,
                                            const unsigned char* __restrict__ csdf) {
    rvgrt_dev::RadianceWorld w;
    static_cast<rv::LinearWorld&>(w) = rvgrt_dev::world(nullptr, csdf);
    w.rad = radianceVoxels;
    rv::f3 acc = rv::V(0.0f, 0.0f, 0.0f);
    float alpha = 0.0f, cd = 1.5f * 2.0f;
    const rv::f3 p0 = rvgrt_dev::F3(pos), d = rvgrt_dev::F3(dir);
    for (int i = 0; i < 20; ++i) {
        if (alpha > 0.99f || cd > 64.0f) break;
        const rv::f3 p = rv::add(p0, rv::scale(d, cd));
        const float scene = rv::get_distance_f(w, p) * 2.0f;
        const float width = cd * RV_TAN_CONE;
        if (scene < width) { alpha = 1.0f; continue; }
        const int gx = (int)(floorf(p.x) / 4.0f), gy = (int)(floorf(p.y) / 4.0f), gz = (int)(floorf(p.z) / 4.0f);
        if (gx >= 0 && gx < w.GX && gy >= 0 && gy < w.GY && gz >= 0 && gz < w.GZ) {
            const float4 s = rvgrt_dev::gi_radiance(w, (uint64_t)gz * (uint64_t)(w.GX * w.GY) + (uint64_t)gy * w.GX + gx);
            const float blend = (1.0f - alpha) * s.w;
            acc = rv::add(acc, rv::scale(rv::V(s.x, s.y, s.z), blend));
            alpha += blend;
        }
        cd += fmaxf(1.5f, width * 0.5f);
    }
    return rvgrt_dev::T3(acc);
}

/* src/raytracing_functions.cu:10-26 */
__device__ __forceinline__ float3 sampleSky(float3 dir, float3 sunDir) {
    return rvgrt_dev::T3(rv::sample_sky(rvgrt_dev::F3(dir), rvgrt_dev::F3(sunDir)));
}

/* src/raytracing_functions.cu:28-62 (fp16 UV math, swapped atlas coordinates) */
__device__ __forceinline__ float3 sampleTexture(__half2 uv, float3 pos, rvgrtAtlas atlas) {
    return rvgrt_dev::T3(rv::sample_texture(rvgrt_dev::world(nullptr, nullptr, nullptr, atlas), __low2float(uv),
                                            __high2float(uv), rvgrt_dev::F3(pos)));
}
