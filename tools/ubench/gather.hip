// Micro-benchmark: cost of an L1-resident gather on gfx950 per wave
// instruction, as a function of the distinct 128-B lines it touches, the
// active lanes, the lane->line mapping and the load width.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int W>   // dwords per lane
__global__ void __launch_bounds__(256) k_gather(const unsigned* __restrict__ buf, unsigned* out, int iters,
                                                int lines, int active, int blocked, unsigned zero) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * 4 + (threadIdx.x >> 6));
    unsigned acc = 0;
    const int per = 64 / lines;
    unsigned line = blocked ? (unsigned)(lane / per) : (unsigned)(lane % lines);
    unsigned word = blocked ? (unsigned)((lane % per) * W & 31) : (unsigned)(((lane / lines) * W) & 31);
    unsigned base = (line * 32u + word + (unsigned)(wave & 7) * 1024u) & 4095u;
    if (lane < active) {
        for (int i = 0; i < iters; i++) {
            unsigned o = base + (acc & zero);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                unsigned a = (o + (unsigned)k * 256u) & (4095u & ~(unsigned)(W - 1));
                if (W == 1) acc += buf[a];
                if (W == 2) { uint2 v = *reinterpret_cast<const uint2*>(buf + a); acc += v.x ^ v.y; }
                if (W == 4) { uint4 v = *reinterpret_cast<const uint4*>(buf + a); acc += v.x ^ v.y ^ v.z ^ v.w; }
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    unsigned *buf, *out;
    (void)hipMalloc(&buf, 16384 * 4);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(buf, 1, 16384 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    int iters = 2000, blocks = 256 * 6;
    printf("width lines active blocked  cycles/wave-instr/CU (2.4 GHz)\n");
    int cfg[][4] = {{1, 1, 64, 0}, {1, 2, 64, 0}, {1, 4, 64, 0}, {1, 8, 64, 0}, {1, 16, 64, 0}, {1, 64, 64, 0},
                    {1, 2, 64, 1}, {1, 4, 64, 1}, {1, 8, 64, 1}, {1, 16, 64, 1}, {1, 32, 64, 1},
                    {1, 16, 40, 0}, {1, 16, 8, 0}, {1, 4, 8, 0},
                    {2, 1, 64, 1}, {2, 4, 64, 1}, {2, 16, 64, 1}, {2, 64, 64, 0},
                    {4, 1, 64, 1}, {4, 4, 64, 1}, {4, 16, 64, 1}, {4, 64, 64, 0}};
    for (auto& c : cfg) {
        auto launch = [&](int it) {
            if (c[0] == 1) hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(256), 0, 0, buf, out, it, c[1], c[2], c[3], 0u);
            if (c[0] == 2) hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(256), 0, 0, buf, out, it, c[1], c[2], c[3], 0u);
            if (c[0] == 4) hipLaunchKernelGGL(k_gather<4>, dim3(blocks), dim3(256), 0, 0, buf, out, it, c[1], c[2], c[3], 0u);
        };
        launch(10);
        (void)hipEventRecord(a);
        launch(iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        double instr_per_cu = (double)blocks * 4 * iters * 8 / 256.0;
        printf("%5d %5d %6d %7d  %8.1f\n", c[0] * 4, c[1], c[2], c[3], ms * 1e6 / instr_per_cu * 2.4);
    }
    return 0;
}
