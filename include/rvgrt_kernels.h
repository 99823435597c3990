/*
 * rvgrt_kernels.h -- the reference's two frame kernels with their argument lists, for HIP
 * code that launches them itself the way drawCUDA does, on reference-layout buffers.
 *
 * Reference interface replaced (src/StateRender.cu):
 *   __constant__ float c_cam[19]; c_currentViewProjection_unjittered;
 *   c_previousViewProjection_unjittered                          :15-29
 *   renderKernel(uchar4* framebuffer, half2* motionVectorBuffer, half* depthBuffer,
 *                cudaTextureObject_t halfDepthTex, cudaTextureObject_t shadowTex,
 *                size_t fbPitchInBytes, size_t mvPitchInBytes, size_t depthPitchInBytes,
 *                int width, int height, bits, csdf, uchar4* GIdata, cudaTextureObject_t texObj)
 *                                                                 :200-253
 *   distApproximationKernel(cudaSurfaceObject_t distSurf, cudaSurfaceObject_t shadowSurf,
 *                           int width, int height, bits, csdf)     :255-286
 *   the uploads of drawCUDA                                        :295-307
 *
 * Argument lists are the reference's, with its texture / surface objects replaced by what they
 * point at on gfx950 (no CUDA texture objects here):
 *   - the half-res distance and shadow images (float cudaArrays of W/2 x H/2 in the reference,
 *     SURVEY Appendix R6) are dense float arrays: rvgrtFloatSurf for the writes of
 *     distApproximationKernel, rvgrtFloatTex for renderKernel's reads.  renderKernel performs
 *     the reference's fetches in arithmetic: minDist's normalized-coordinate point fetch
 *     (including the texel-low quirk, RV_F_REF_FETCH) and tex2D's linear filter with 1/256
 *     weights (Appendix R9);
 *   - the atlas is an rvgrtAtlas (include/rvgrt_device.h).
 * Frame constants live in __constant__ memory as in the reference, under prefixed names:
 * rvgrt_c_cam[20] (the reference's c_cam layout: pos, fo, ri, up, sun, then the 3 floats
 * drawCUDA writes at [15..17] and reads back as c_time = [17], c_jitterX = [18],
 * c_jitterY = [19]: Appendix R1, reproduced when 18 floats are uploaded, as drawCUDA does)
 * and the two unjittered view-projection matrices (glm column-major).
 * rvgrtUploadFrameConstants() is drawCUDA's three cudaMemcpyToSymbol calls.
 *
 * Launch as drawCUDA does: 8 x 8 blocks over W/2 x H/2 for distApproximationKernel, then over
 * W x H for renderKernel, on one stream.  The bodies are the library's own per-pixel code
 * (include/rvgrt/rv_shade.h) on the reference layout: frames are bit-identical with the CPU
 * oracle (tests/test_gpu_devapi.py).  Include in one translation unit (the __constant__
 * symbols are defined here); compile with -ffp-contract=off for bit-exact results.
 */
#pragma once

#include "rvgrt_device.h"
#include "rvgrt/rv_shade.h"

/* half-res float images (the reference's cudaArrays behind its surface / texture objects) */
struct rvgrtFloatSurf {
    float* data;          /* width * height floats, row-major */
    int width, height;
};
struct rvgrtFloatTex {
    const float* data;
    int width, height;
};

/* src/StateRender.cu:15-17 */
__constant__ float rvgrt_c_cam[20];
__constant__ float rvgrt_c_currentViewProjection_unjittered[16];
__constant__ float rvgrt_c_previousViewProjection_unjittered[16];

/* drawCUDA's uploads (src/StateRender.cu:295-307): cam = the 18 floats it packs
 * {pos, fo, ri, up, sunDir, time, jitterX, jitterY}; vp / prevVp = glm::mat4 (16 floats). */
static inline hipError_t rvgrtUploadFrameConstants(const float cam[18], const float vp[16], const float prevVp[16],
                                                   hipStream_t stream = 0) {
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(rvgrt_c_previousViewProjection_unjittered), prevVp,
                                          16 * sizeof(float), 0, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess)
        e = hipMemcpyToSymbolAsync(HIP_SYMBOL(rvgrt_c_currentViewProjection_unjittered), vp, 16 * sizeof(float), 0,
                                   hipMemcpyHostToDevice, stream);
    if (e == hipSuccess)
        e = hipMemcpyToSymbolAsync(HIP_SYMBOL(rvgrt_c_cam), cam, 18 * sizeof(float), 0, hipMemcpyHostToDevice, stream);
    return e;
}

namespace rvgrt_dev {
/* The frame's constants as the library's per-pixel code reads them. */
__device__ __forceinline__ rv::FrameParams frame_params(int W, int H, int hw, int hh) {
    rv::FrameParams f{};
    const float* c = rvgrt_c_cam;
    f.pos = rv::V(c[0], c[1], c[2]);
    f.fo = rv::V(c[3], c[4], c[5]);
    f.ri = rv::V(c[6], c[7], c[8]);
    f.up = rv::V(c[9], c[10], c[11]);
    f.sun = rv::V(c[12], c[13], c[14]);
    f.time = c[17];            /* c_time (Appendix R1) */
    f.jx = c[18];              /* c_jitterX */
    f.jy = c[19];              /* c_jitterY */
    rv::cone_basis_scales(f.cone_k1, f.cone_k2);
#pragma unroll
    for (int i = 0; i < 16; i++) {
        f.vp[i] = rvgrt_c_currentViewProjection_unjittered[i];
        f.pvp[i] = rvgrt_c_previousViewProjection_unjittered[i];
    }
    f.W = W; f.H = H; f.hw = hw; f.hh = hh;
    f.flags = RV_F_PREPASS | RV_F_WATER | RV_F_GI | RV_F_REF_FETCH;
    return f;
}
constexpr uint32_t FEAT_REF = RV_F_PREPASS | RV_F_WATER | RV_F_GI;
}  // namespace rvgrt_dev

/* src/StateRender.cu:255-286 */
__global__ void distApproximationKernel(rvgrtFloatSurf distSurf, rvgrtFloatSurf shadowSurf, int width, int height,
                                        const uint32_t* __restrict__ bits, const unsigned char* __restrict__ csdf) {
    const int ix = blockIdx.x * blockDim.x + threadIdx.x, iy = blockIdx.y * blockDim.y + threadIdx.y;
    if (ix >= width || iy >= height) return;
    rv::FrameParams f = rvgrt_dev::frame_params(2 * width, 2 * height, width, height);
    f.hdist = distSurf.data;
    f.hshadow = shadowSurf.data;
    uint32_t cnt[rv::NCNT];
    rv::prepass_pixel<false>(rvgrt_dev::world(bits, csdf), f, ix, iy, cnt);
}

/* src/StateRender.cu:200-253 */
__global__ void renderKernel(uchar4* framebuffer, __half2* motionVectorBuffer, __half* depthBuffer,
                             rvgrtFloatTex halfDepthTex, rvgrtFloatTex shadowTex, size_t fbPitchInBytes,
                             size_t mvPitchInBytes, size_t depthPitchInBytes, int width, int height,
                             const uint32_t* __restrict__ bits, const unsigned char* __restrict__ csdf,
                             uchar4* __restrict__ GIdata, rvgrtAtlas texObj) {
    const int ix = blockIdx.x * blockDim.x + threadIdx.x, iy = blockIdx.y * blockDim.y + threadIdx.y;
    if (ix >= width || iy >= height) return;
    rv::FrameParams f = rvgrt_dev::frame_params(width, height, halfDepthTex.width, halfDepthTex.height);
    f.hdist = const_cast<float*>(halfDepthTex.data);
    f.hshadow = const_cast<float*>(shadowTex.data);
    f.mv = reinterpret_cast<uint32_t*>(motionVectorBuffer); f.mv_pitch = mvPitchInBytes;
    f.depth = reinterpret_cast<uint16_t*>(depthBuffer); f.depth_pitch = depthPitchInBytes;
    uint32_t cnt[rv::NCNT];
    const uint32_t px = rv::render_pixel<false, rvgrt_dev::FEAT_REF>(
        rvgrt_dev::world(bits, csdf, reinterpret_cast<const uint32_t*>(GIdata), texObj), f, ix, iy, cnt);
    *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(framebuffer) + (size_t)iy * fbPitchInBytes + 4 * (size_t)ix) = px;
}
