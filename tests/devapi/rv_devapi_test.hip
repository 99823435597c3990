// rv_devapi_test.hip -- test harness for include/rvgrt_device.h: small HIP
// kernels written the way the reference's kernels call its __device__ API
// (src/StateRender.cu:48,275-281, src/CoarseArray.cu:324-340), over
// reference-layout buffers, exported to the pytest suite through a C ABI.
// Built for a 128 x 64 x 128 world (RVGRT_SHIX/Y/Z from the Makefile).
// Test infrastructure: nothing in the product links it.
#include "../../include/rvgrt_device.h"
#include "../../include/rvgrt_kernels.h"

#include <vector>

namespace {

__global__ void k_trace(const uint32_t* bits, const unsigned char* csdf, const float* org, const float* dir,
                        const float* dist, int n, hitInfo* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = trace(make_float3(org[3 * i], org[3 * i + 1], org[3 * i + 2]),
                   make_float3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), (__half)dist[i], bits, csdf);
}

__global__ void k_approx(const unsigned char* csdf, const float* org, const float* dir, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float3 p = approximateCSDF(make_float3(org[3 * i], org[3 * i + 1], org[3 * i + 2]),
                                     make_float3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), csdf);
    out[3 * i] = p.x; out[3 * i + 1] = p.y; out[3 * i + 2] = p.z;
}

__global__ void k_cone(const unsigned char* csdf, const uchar4* gi, const float4* rad, const float* pos,
                       const float* dir, int n, float* out8, float* outf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float3 p = make_float3(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]);
    const float3 d = make_float3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    const float3 a = traceCone(p, d, gi, csdf);
    const float3 b = traceCone(p, d, rad, csdf);
    out8[3 * i] = a.x; out8[3 * i + 1] = a.y; out8[3 * i + 2] = a.z;
    outf[3 * i] = b.x; outf[3 * i + 1] = b.y; outf[3 * i + 2] = b.z;
}

__global__ void k_texture(rvgrtAtlas atlas, const float* uv, const float* pos, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float3 c = sampleTexture(__floats2half2_rn(uv[2 * i], uv[2 * i + 1]),
                                   make_float3(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]), atlas);
    out[3 * i] = c.x; out[3 * i + 1] = c.y; out[3 * i + 2] = c.z;
}

__global__ void k_sky(const float* dir, float3 sun, int n, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float3 c = sampleSky(make_float3(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), sun);
    out[3 * i] = c.x; out[3 * i + 1] = c.y; out[3 * i + 2] = c.z;
}

// IsSolid, getDistance(int3) and getDistance(float3) at integer / float points
__global__ void k_lookup(const uint32_t* bits, const unsigned char* csdf, const int* ip, const float* fp, int n,
                         int* solid, int* di, float* df) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int3 q = make_int3(ip[3 * i], ip[3 * i + 1], ip[3 * i + 2]);
    solid[i] = IsSolid(q, bits);
    di[i] = getDistance(q, csdf);
    df[i] = getDistance(make_float3(fp[3 * i], fp[3 * i + 1], fp[3 * i + 2]), csdf);
}

// Device buffers freed at scope exit; every HIP status is checked.
struct Dev {
    std::vector<void*> ptrs;
    hipError_t err = hipSuccess;
    template <class T>
    T* up(const void* host, size_t bytes) {
        void* p = nullptr;
        if (err == hipSuccess) err = hipMalloc(&p, bytes ? bytes : 4);
        if (err == hipSuccess && host && bytes) err = hipMemcpy(p, host, bytes, hipMemcpyHostToDevice);
        if (p) ptrs.push_back(p);
        return static_cast<T*>(p);
    }
    void down(void* host, const void* dev, size_t bytes) {
        if (err == hipSuccess && bytes) err = hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost);
    }
    void launched() {
        if (err == hipSuccess) err = hipGetLastError();
        if (err == hipSuccess) err = hipDeviceSynchronize();
    }
    ~Dev() { for (void* p : ptrs) (void)hipFree(p); }
};

inline unsigned blocks(int n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" {

int rvt_dims(int* out3) {
    out3[0] = RVGRT_SHIX; out3[1] = RVGRT_SHIY; out3[2] = RVGRT_SHIZ;
    return (int)sizeof(hitInfo);
}

int rvt_trace(const uint32_t* bits, size_t nbits, const uint8_t* csdf, size_t ncsdf, const float* org,
              const float* dir, const float* dist, int n, void* out) {
    if (n <= 0) return 0;
    Dev d;
    auto* b = d.up<uint32_t>(bits, nbits);
    auto* c = d.up<unsigned char>(csdf, ncsdf);
    auto* o = d.up<float>(org, 12ull * n);
    auto* r = d.up<float>(dir, 12ull * n);
    auto* t = d.up<float>(dist, 4ull * n);
    auto* h = d.up<hitInfo>(nullptr, sizeof(hitInfo) * n);
    if (d.err == hipSuccess) hipLaunchKernelGGL(k_trace, dim3(blocks(n)), dim3(256), 0, 0, b, c, o, r, t, n, h);
    d.launched();
    d.down(out, h, sizeof(hitInfo) * n);
    return (int)d.err;
}

int rvt_approx(const uint8_t* csdf, size_t ncsdf, const float* org, const float* dir, int n, float* out) {
    if (n <= 0) return 0;
    Dev d;
    auto* c = d.up<unsigned char>(csdf, ncsdf);
    auto* o = d.up<float>(org, 12ull * n);
    auto* r = d.up<float>(dir, 12ull * n);
    auto* p = d.up<float>(nullptr, 12ull * n);
    if (d.err == hipSuccess) hipLaunchKernelGGL(k_approx, dim3(blocks(n)), dim3(256), 0, 0, c, o, r, n, p);
    d.launched();
    d.down(out, p, 12ull * n);
    return (int)d.err;
}

int rvt_cone(const uint8_t* csdf, size_t ncsdf, const uint8_t* gi, size_t ngi, const float* pos, const float* dir,
             int n, float* out8, float* outf) {
    if (n <= 0) return 0;
    std::vector<float4> rad(ngi / 4);   // the float4 overload's grid: RGBA8 / 255
    for (size_t k = 0; k < rad.size(); k++)
        rad[k] = make_float4(gi[4 * k] / 255.0f, gi[4 * k + 1] / 255.0f, gi[4 * k + 2] / 255.0f, gi[4 * k + 3] / 255.0f);
    Dev d;
    auto* c = d.up<unsigned char>(csdf, ncsdf);
    auto* g = d.up<uchar4>(gi, ngi);
    auto* f = d.up<float4>(rad.data(), rad.size() * sizeof(float4));
    auto* p = d.up<float>(pos, 12ull * n);
    auto* r = d.up<float>(dir, 12ull * n);
    auto* a = d.up<float>(nullptr, 12ull * n);
    auto* b = d.up<float>(nullptr, 12ull * n);
    if (d.err == hipSuccess) hipLaunchKernelGGL(k_cone, dim3(blocks(n)), dim3(256), 0, 0, c, g, f, p, r, n, a, b);
    d.launched();
    d.down(out8, a, 12ull * n);
    d.down(outf, b, 12ull * n);
    return (int)d.err;
}

int rvt_texture(const uint32_t* atlas, int aw, int ah, const float* uv, const float* pos, int n, float* out) {
    if (n <= 0) return 0;
    Dev d;
    rvgrtAtlas at{d.up<uint32_t>(atlas, 4ull * aw * ah), aw, ah};
    auto* u = d.up<float>(uv, 8ull * n);
    auto* p = d.up<float>(pos, 12ull * n);
    auto* o = d.up<float>(nullptr, 12ull * n);
    if (d.err == hipSuccess) hipLaunchKernelGGL(k_texture, dim3(blocks(n)), dim3(256), 0, 0, at, u, p, n, o);
    d.launched();
    d.down(out, o, 12ull * n);
    return (int)d.err;
}

int rvt_sky(const float* dir, const float* sun, int n, float* out) {
    if (n <= 0) return 0;
    Dev d;
    auto* r = d.up<float>(dir, 12ull * n);
    auto* o = d.up<float>(nullptr, 12ull * n);
    if (d.err == hipSuccess)
        hipLaunchKernelGGL(k_sky, dim3(blocks(n)), dim3(256), 0, 0, r, make_float3(sun[0], sun[1], sun[2]), n, o);
    d.launched();
    d.down(out, o, 12ull * n);
    return (int)d.err;
}

int rvt_lookup(const uint32_t* bits, size_t nbits, const uint8_t* csdf, size_t ncsdf, const int* ip, const float* fp,
               int n, int* solid, int* di, float* df) {
    if (n <= 0) return 0;
    Dev d;
    auto* b = d.up<uint32_t>(bits, nbits);
    auto* c = d.up<unsigned char>(csdf, ncsdf);
    auto* i = d.up<int>(ip, 12ull * n);
    auto* f = d.up<float>(fp, 12ull * n);
    auto* s = d.up<int>(nullptr, 4ull * n);
    auto* x = d.up<int>(nullptr, 4ull * n);
    auto* y = d.up<float>(nullptr, 4ull * n);
    if (d.err == hipSuccess) hipLaunchKernelGGL(k_lookup, dim3(blocks(n)), dim3(256), 0, 0, b, c, i, f, n, s, x, y);
    d.launched();
    d.down(solid, s, 4ull * n);
    d.down(di, x, 4ull * n);
    d.down(df, y, 4ull * n);
    return (int)d.err;
}

// drawCUDA's sequence (src/StateRender.cu:289-346) through the reference-signature kernels of
// include/rvgrt_kernels.h: the three constant uploads, distApproximationKernel over W/2 x H/2 and
// renderKernel over W x H in 8 x 8 blocks, into pitched outputs (pitch = row + 192 B).  Returns
// the images row-packed: colour W*H*4, motion W*H*4, depth W*H*2, half distance / shadow.
int rvt_frame(const uint32_t* bits, size_t nbits, const uint8_t* csdf, size_t ncsdf, const uint8_t* gi, size_t ngi,
              const uint32_t* atlas, int aw, int ah, const float* cam18, const float* vp, const float* pvp, int W,
              int H, uint8_t* color, uint8_t* mv, uint8_t* depth, float* hdist, float* hshadow) {
    if (W <= 0 || H <= 0 || (W & 1) || (H & 1)) return -1;
    const int hw = W / 2, hh = H / 2;
    const size_t pc = 4ull * W + 192, pm = 4ull * W + 192, pd = 2ull * W + 192;
    Dev d;
    auto* b = d.up<uint32_t>(bits, nbits);
    auto* c = d.up<unsigned char>(csdf, ncsdf);
    auto* g = d.up<uchar4>(gi, ngi);
    rvgrtAtlas at{d.up<uint32_t>(atlas, 4ull * aw * ah), aw, ah};
    auto* fb = d.up<uchar4>(nullptr, pc * H);
    auto* m = d.up<__half2>(nullptr, pm * H);
    auto* z = d.up<__half>(nullptr, pd * H);
    auto* hd = d.up<float>(nullptr, 4ull * hw * hh);
    auto* hs = d.up<float>(nullptr, 4ull * hw * hh);
    if (d.err == hipSuccess) d.err = rvgrtUploadFrameConstants(cam18, vp, pvp, 0);
    const dim3 block(8, 8);
    if (d.err == hipSuccess)
        hipLaunchKernelGGL(distApproximationKernel, dim3((hw + 7) / 8, (hh + 7) / 8), block, 0, 0,
                           rvgrtFloatSurf{hd, hw, hh}, rvgrtFloatSurf{hs, hw, hh}, hw, hh, b, c);
    if (d.err == hipSuccess)
        hipLaunchKernelGGL(renderKernel, dim3((W + 7) / 8, (H + 7) / 8), block, 0, 0, fb, m, z,
                           rvgrtFloatTex{hd, hw, hh}, rvgrtFloatTex{hs, hw, hh}, pc, pm, pd, W, H, b, c, g, at);
    d.launched();
    if (d.err == hipSuccess) d.err = hipMemcpy2D(color, 4ull * W, fb, pc, 4ull * W, H, hipMemcpyDeviceToHost);
    if (d.err == hipSuccess) d.err = hipMemcpy2D(mv, 4ull * W, m, pm, 4ull * W, H, hipMemcpyDeviceToHost);
    if (d.err == hipSuccess) d.err = hipMemcpy2D(depth, 2ull * W, z, pd, 2ull * W, H, hipMemcpyDeviceToHost);
    d.down(hdist, hd, 4ull * hw * hh);
    d.down(hshadow, hs, 4ull * hw * hh);
    return (int)d.err;
}

}  // extern "C"
