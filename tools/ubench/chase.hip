// Micro-benchmark: latency of one dependent gather on gfx950 by where the line lives -- the floor of a
// lone ray's chain (a sphere step's next address is its gather's result).  One lane chases a random
// cyclic permutation of 128-B lines over a buffer of S bytes (S from L2-resident to far beyond the
// 256 MB Infinity Cache), optionally while every other CU streams through a separate buffer (the load
// the tail of a frame launch runs under).  Mode 2: the same load kept off the chasing lane's CU (CU-masked
// streams), to split the load's cost into the CU's own memory pipeline and the shared L2 / fabric.
// Argument 2: lanes of the chasing wave (each its own stretch of the cycle: a wave-wide divergent gather
// per hop, as a sphere step of a full wave).  Prints ns per hop.  Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

__global__ void k_chase(const unsigned* __restrict__ buf, const unsigned* __restrict__ starts, int hops, unsigned* out,
                        unsigned long long* ticks, int lanes) {
    if ((int)threadIdx.x >= lanes) return;
    unsigned p = starts[threadIdx.x];   // lane l: lines / lanes further along the cycle (disjoint stretches)
    const unsigned long long t0 = __builtin_readcyclecounter();
    const unsigned long long r0 = wall_clock64();
    for (int i = 0; i < hops; i++) p = buf[p];
    const unsigned long long r1 = wall_clock64();
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) {
        out[0] = p;
        ticks[0] = r1 - r0;
        ticks[1] = t1 - t0;
    } else if (p == 0xFFFFFFFFu) out[1] = p;
}

// background load: each wave streams a private slice (coalesced dword loads), until *stop is set
__global__ void k_load(const unsigned* __restrict__ buf, size_t n, volatile unsigned* stop, unsigned* out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (int rep = 0; rep < 8000 && !*stop; rep++)
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride * 64) acc += buf[i];
    if (acc == 0x9e3779b9u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int lanes = argc > 2 ? atoi(argv[2]) : 1;   // lanes of the chasing wave, each on its own stretch
    const bool loaded = mode != 0;
    const size_t sizes[] = {1u << 20, 4u << 20, 16u << 20, 64u << 20, 128u << 20, 256u << 20, 1024u << 20};
    unsigned *out, *stop, *lbuf = nullptr;
    unsigned long long* ticks;
    hipMalloc(&out, 16);
    hipMalloc(&ticks, 16);
    hipHostMalloc(&stop, 4, hipHostMallocCoherent);
    const size_t ln = (size_t)512 << 20;   // 2 GiB background buffer
    if (loaded) { hipMalloc(&lbuf, ln * 4); hipMemset(lbuf, 1, ln * 4); }
    hipStream_t sl, sc;
    if (mode == 2) {
        hipDeviceProp_t prop;
        hipGetDeviceProperties(&prop, 0);
        const int ncu = prop.multiProcessorCount, words = (ncu + 31) / 32;
        std::vector<uint32_t> mc(words, 0u), ml(words, 0u);
        mc[0] = 1u;   // the chaser: CU 0
        for (int i = 1; i < ncu; i++) ml[i / 32] |= 1u << (i % 32);   // the load: every other CU
        hipExtStreamCreateWithCUMask(&sc, (uint32_t)words, mc.data());
        hipExtStreamCreateWithCUMask(&sl, (uint32_t)words, ml.data());
        printf("mode 2: %d CUs, chaser on CU 0, load on the other %d\n", ncu, ncu - 1);
    } else {
        hipStreamCreateWithFlags(&sl, hipStreamNonBlocking);
        hipStreamCreateWithFlags(&sc, hipStreamNonBlocking);
    }
    for (size_t S : sizes) {
        const size_t lines = S / 128;
        std::vector<unsigned> perm(lines);
        for (size_t i = 0; i < lines; i++) perm[i] = (unsigned)i;
        std::mt19937 rng(7);
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<unsigned> h(S / 4, 0);
        for (size_t i = 0; i < lines; i++) h[(size_t)perm[i] * 32] = perm[(i + 1) % lines] * 32;   // a cycle over all lines
        unsigned* buf;
        hipMalloc(&buf, S);
        hipMemcpy(buf, h.data(), S, hipMemcpyHostToDevice);
        const int hops = 20000;
        unsigned hst[64], *dst;
        for (int l = 0; l < 64; l++) hst[l] = perm[(12345 + (size_t)l * (lines / 64)) % lines] * 32u;
        hipMalloc(&dst, sizeof hst);
        hipMemcpy(dst, hst, sizeof hst, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, sc, buf, dst, 2000, out, ticks, 1);   // warm
        hipStreamSynchronize(sc);
        if (loaded) {
            *stop = 0;
            hipLaunchKernelGGL(k_load, dim3(2048), dim3(256), 0, sl, lbuf, ln, stop, out + 1);
        }
        hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, sc, buf, dst, hops, out, ticks, lanes);
        hipStreamSynchronize(sc);
        if (loaded) { *stop = 1; hipStreamSynchronize(sl); }
        unsigned long long t[2];
        hipMemcpy(t, ticks, 16, hipMemcpyDeviceToHost);
        printf("%s %2d lanes, buffer %7zu KiB: %7.1f ns per dependent gather (%6.0f cycles)\n",
               mode == 2 ? "isolat" : loaded ? "loaded" : "idle  ", lanes, S >> 10, t[0] * 10.0 / hops, (double)t[1] / hops);
        hipFree(buf);
        hipFree(dst);
    }
    return 0;
}
