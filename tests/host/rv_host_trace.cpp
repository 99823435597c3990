// rv_host_trace.cpp -- TEST INFRASTRUCTURE: the product's traversal source
// (include/rvgrt/rv_device.h, host+device functions) compiled for the CPU,
// so tests/test_host_trace.py can check that exact code -- including its
// compile-time variants (DDA look-ahead group, word reuse) -- against the oracle on
// hosts without a GPU.  Not linked into librvgrt_hip.so and not used by it.
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/rvgrt/rv_device.h"

using namespace rv;

namespace {
struct HostWorld {
    std::vector<uint32_t> brick;
    World w{};
};

// Canonical (reference) bits (toIndex order, include/cumath.cuh:33-45) and
// CSDF (x fastest) -> the product's split brick layout (rv_device.h).
void build(HostWorld& h, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf) {
    World& w = h.w;
    w.X = 1 << lx; w.Y = 1 << ly; w.Z = 1 << lz;
    w.lbx = lx - 3; w.lbxy = (lx - 3) + (ly - 3);
    w.lbz = lz - 3; w.lbzy = (lz - 3) + (ly - 3);
    w.SX = w.X / 2; w.SY = w.Y / 2; w.SZ = w.Z / 2;
    w.GX = w.X / 4; w.GY = w.Y / 4; w.GZ = w.Z / 4;
    w.fX = (float)w.X; w.fY = (float)w.Y; w.fZ = (float)w.Z;
    const uint64_t nbricks = ((uint64_t)w.X * w.Y * w.Z) / 512;
    world_set_regions(w, nbricks);
    // 128 B per brick, then the sun horizon (UINT32_MAX: no sun exit until world_horizon builds it), then
    // the DDA's column-neighbourhood tops (0x7F7F7F7F: no column skip until world_dtop builds them)
    h.brick.assign((size_t)(((uint64_t)w.X * w.Y * w.Z) / 16) + horizon_bytes(w.X, w.Z) / 4 + dtop_bytes(w.X, w.Z) / 4,
                   0u);
    std::fill(h.brick.begin() + (long)(horizon_byte(w.coff) / 4),
              h.brick.begin() + (long)(dtop_byte(w.coff, w.X, w.Z) / 4), 0xFFFFFFFFu);
    std::fill(h.brick.begin() + (long)(dtop_byte(w.coff, w.X, w.Z) / 4), h.brick.end(), 0x7F7F7F7Fu);
    for (uint64_t z = 0; z < (uint64_t)w.Z; z++)
        for (uint64_t y = 0; y < (uint64_t)w.Y; y++)
            for (uint64_t x = 0; x < (uint64_t)w.X; x++) {
                uint64_t ci = x | (y << lx) | (z << (lx + ly));
                if (!((bits[ci >> 5] >> (ci & 31)) & 1u)) continue;
                uint64_t b = brick_of(w, x >> 3, y >> 3, z >> 3);
                uint32_t bit = (uint32_t)((x & 7) | ((y & 7) << 3) | ((z & 7) << 6));
                h.brick[bits_word_index(b, bit >> 5)] |= 1u << (bit & 31);
            }
    uint8_t* bytes = reinterpret_cast<uint8_t*>(h.brick.data());
    for (uint64_t cz = 0; cz < (uint64_t)w.SZ; cz++)
        for (uint64_t cy = 0; cy < (uint64_t)w.SY; cy++)
            for (uint64_t cx = 0; cx < (uint64_t)w.SX; cx++) {
                uint64_t b = brick_of(w, cx >> 2, cy >> 2, cz >> 2);
                uint32_t local = (uint32_t)((cx & 3) | ((cy & 3) << 2) | ((cz & 3) << 4));
                bytes[csdf_byte_index(w.coff, b, local)] = csdf[(cz * w.SY + cy) * w.SX + cx];
            }
    world_set_brick(w, h.brick.data());
}
// World::ytop as rv_abi.cpp's world_top sets it: highest solid row + 2, at most Y
uint32_t world_ytop(const HostWorld& h) {
    const World& w = h.w;
    const uint64_t nb = ((uint64_t)w.X * w.Y * w.Z) / 512;
    uint32_t top = 0;
    for (uint64_t b = 0; b < nb; b++) {
        uint32_t bx, by, bz;
        brick_coords(w, b, bx, by, bz);
        const uint32_t t = brick_top_y(&h.brick[bits_word_index(b, 0)], by);
        top = t > top ? t : top;
    }
    return top + 1u < (uint32_t)w.Y ? top + 1u : (uint32_t)w.Y;
}

// World::horizon as rv_abi.cpp's world_top builds it for the sun direction `sun` (k_column_top +
// k_horizon: the same brick_subcolumn_tops and horizon_column, topmax = World::ytop)
void world_horizon(HostWorld& h, const float* sun, std::vector<uint32_t>& coltop, std::vector<uint32_t>& hz) {
    World& w = h.w;
    const int ncx = w.X >> 1, ncz = w.Z >> 1, lcx = w.lbx + 2;
    coltop.assign((size_t)ncx * ncz, 0u);
    hz.assign((size_t)ncx * ncz, 0u);
    const uint64_t nb = ((uint64_t)w.X * w.Y * w.Z) / 512;
    for (uint64_t b = 0; b < nb; b++) {
        uint32_t bx, by, bz;
        brick_coords(w, b, bx, by, bz);
        uint32_t t[16];
        brick_subcolumn_tops(&h.brick[bits_word_index(b, 0)], by, t);
        for (uint32_t q = 0; q < 16; q++) {
            uint32_t& c = coltop[(bx * 4u + (q & 3u)) | ((bz * 4u + (q >> 2)) << (uint32_t)lcx)];
            c = t[q] > c ? t[q] : c;
        }
    }
    const double hxz = std::sqrt((double)sun[0] * sun[0] + (double)sun[2] * sun[2]);
    const float k = (float)((double)sun[1] / hxz * (1.0 - 1e-3));
    for (int j = 0; j < ncz; j++)
        for (int i = 0; i < ncx; i++)
            hz[(uint32_t)i | ((uint32_t)j << lcx)] = horizon_column(coltop.data(), ncx, ncz, lcx, i, j, (float)(sun[0] / hxz),
                                                                    (float)(sun[2] / hxz), k, (float)w.ytop);
    std::copy(hz.begin(), hz.end(), h.brick.begin() + (long)(horizon_byte(w.coff) / 4));   // where horizon_at reads
}

// The DDA's empty-column skip table (dtop_at) as rv_abi.cpp's world_top builds it: the 2x2-column tops
// (k_column_top: brick_subcolumn_tops), then per brick column the highest of them over the 3x3 brick
// columns around it (k_dtop).
void world_dtop(HostWorld& h) {
    World& w = h.w;
    const int ncx = w.X >> 1, ncz = w.Z >> 1, lcx = w.lbx + 2, nbx = w.X >> 3, nbz = w.Z >> 3;
    std::vector<uint32_t> coltop((size_t)ncx * ncz, 0u);
    const uint64_t nb = ((uint64_t)w.X * w.Y * w.Z) / 512;
    for (uint64_t b = 0; b < nb; b++) {
        uint32_t bx, by, bz;
        brick_coords(w, b, bx, by, bz);
        uint32_t t[16];
        brick_subcolumn_tops(&h.brick[bits_word_index(b, 0)], by, t);
        for (uint32_t q = 0; q < 16; q++) {
            uint32_t& c = coltop[(bx * 4u + (q & 3u)) | ((bz * 4u + (q >> 2)) << (uint32_t)lcx)];
            c = t[q] > c ? t[q] : c;
        }
    }
    int* dt = reinterpret_cast<int*>(reinterpret_cast<char*>(h.brick.data()) + dtop_byte(w.coff, w.X, w.Z));
    for (int bz = 0; bz < nbz; bz++)
        for (int bx = 0; bx < nbx; bx++) {
            uint32_t t = 0;
            for (int z = std::max(bz - 1, 0) * 4; z < std::min(bz + 2, nbz) * 4; z++)
                for (int x = std::max(bx - 1, 0) * 4; x < std::min(bx + 2, nbx) * 4; x++)
                    t = std::max(t, coltop[(uint32_t)x | ((uint32_t)z << lcx)]);
            dt[bx | (bz << w.lbx)] = (int)t;
        }
}

template <int G, bool REUSE, bool RW = true>
Hit trace_v(const World& w, f3 o, f3 d, float t, StepCount& sc) {
    return trace<true, G, REUSE, RW, false, World, false>(w, o, d, t, sc);
}
}  // namespace

extern "C" {

// Out record per ray (48 B): pos[3], normal[3], u, v, hit, undef, sphere, dda, check (ints)
struct HostHit { float pos[3], normal[3], u, v; int32_t hit, undef, sphere, dda, check, pad; };

// variant: 0..3 = DDA look-ahead group 1/2/4/8 (stop search + re-walk), 4 = group 1 with word
// reuse, 5..6 = group 4 / 8 with the step-by-step replay (trace RW = false)
int rvh_variants(void) { return 7; }

// rv::u8f, the device's byte -> float conversion
float rvh_u8f(uint32_t b) { return rv::u8f(b); }

// rv::simplex3D (texture and water noise, world build) over n points
void rvh_simplex3D(const float* xyz, float* out, int64_t n) {
    for (int64_t i = 0; i < n; i++) out[i] = rv::simplex3D(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
}

// sampleTexture's tile (0xYX) for n positions in a 2^lx x 2^ly x 2^lz world, through the World::tex
// table (built on the host with k_tex_table's element function) and through the noise (tex = null)
// ny: the rows the table covers (0: all; else a multiple of 8, the band below the sky exit)
void rvh_texture_tiles(int lx, int ly, int lz, int ny, const float* pos, int64_t n, int32_t* via_table,
                       int32_t* via_noise) {
    World w{};
    w.X = 1 << lx; w.Y = 1 << ly; w.Z = 1 << lz;
    w.lbx = lx - 3; w.lbz = lz - 3; w.lbzy = (lz - 3) + (ly - 3);
    w.tex_ny = ny ? (uint32_t)ny : (uint32_t)w.Y;
    std::vector<uint32_t> tex((size_t)w.X * w.tex_ny * w.Z, 0xFFFFFFFFu);
    for (uint32_t z = 0; z < (uint32_t)w.Z; z++)
        for (uint32_t y = 0; y < w.tex_ny; y++)
            for (uint32_t x = 0; x < (uint32_t)w.X; x++) tex[tex_index(w, x, y, z)] = tex_table_entry(x, y, z);
    for (size_t i = 0; i < tex.size(); i++) {   // every entry written once, by k_tex_table's order too
        uint32_t bx, by, bz;
        tex_brick_coords(w, i >> 9, bx, by, bz);
        const uint32_t l = (uint32_t)i & 511u;
        if (tex[i] != tex_table_entry(bx * 8u + ((l >> 3) & 7u), by * 8u + (l >> 6), bz * 8u + (l & 7u))) return;
    }
    World wn = w;
    w.tex = tex.data();
    for (int64_t i = 0; i < n; i++) {
        const f3 p = V(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]);
        via_table[i] = texture_tile(w, p);
        via_noise[i] = texture_tile(wn, p);
    }
}

// sky_exit: 1 = World::ytop from the bricks (world_top_y over every brick, as k_world_top), the
// frame kernels' traversal; 0 = ytop = Y, the reference's step counts.
static int trace_rays(int variant, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf, const float* org,
                      const float* dir, const float* dist, int64_t n, HostHit* out, int sky_exit);

int rvh_trace_rays(int variant, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf, const float* org,
                   const float* dir, const float* dist, int64_t n, HostHit* out) {
    return trace_rays(variant, lx, ly, lz, bits, csdf, org, dir, dist, n, out, 0);
}

int rvh_trace_rays_sky_exit(int variant, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf,
                            const float* org, const float* dir, const float* dist, int64_t n, HostHit* out,
                            uint32_t* ytop) {
    const int r = trace_rays(variant, lx, ly, lz, bits, csdf, org, dir, dist, n, out, 1);
    HostWorld h;
    build(h, lx, ly, lz, bits, csdf);
    *ytop = world_ytop(h);
    return r;
}

// Rays toward the sun through trace_sun with the sky exit and the sun horizon built for `sun`
// (every direction must be exactly `sun`, as for the kernels' shadow rays); hz_out: the horizon map.
// g8: 1 = look-ahead 8 (else 4)
int rvh_trace_sun(int g8, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf, const float* sun,
                  const float* org, const float* dist, int64_t n, HostHit* out, uint32_t* hz_out) {
    g8 &= 1;
    HostWorld h;
    build(h, lx, ly, lz, bits, csdf);
    h.w.ytop = world_ytop(h);
    std::vector<uint32_t> coltop, hz;
    world_horizon(h, sun, coltop, hz);
    memcpy(hz_out, hz.data(), hz.size() * 4);
    const f3 d = V(sun[0], sun[1], sun[2]);
    for (int64_t i = 0; i < n; i++) {
        StepCount sc{};
        const f3 o = V(org[3 * i], org[3 * i + 1], org[3 * i + 2]);
        Hit r = g8 ? trace_sun<true, 8, false>(h.w, o, d, hround(dist[i]), sc)
                   : trace_sun<true, 4, false>(h.w, o, d, hround(dist[i]), sc);
        HostHit& q = out[i];
        q.pos[0] = r.pos.x; q.pos[1] = r.pos.y; q.pos[2] = r.pos.z;
        q.normal[0] = r.normal.x; q.normal[1] = r.normal.y; q.normal[2] = r.normal.z;
        q.u = r.u; q.v = r.v; q.hit = r.hit; q.undef = r.undef;
        q.sphere = (int)sc.sphere; q.dda = (int)sc.dda; q.check = (int)sc.check; q.pad = 0;
    }
    return 0;
}

// The empty-column skip (trace COL = true, look-ahead 4 or 8 with re-walk, the sky exit and the dtop table
// built as the library builds it): the variant the water reflections of the pipelined and grouped launches
// take.  col = 0 traces the same rays without the skip (same sky exit), for comparison.
int rvh_trace_col(int g8, int col, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf, const float* org,
                  const float* dir, const float* dist, int64_t n, HostHit* out) {
    HostWorld h;
    build(h, lx, ly, lz, bits, csdf);
    h.w.ytop = world_ytop(h);
    world_dtop(h);
    for (int64_t i = 0; i < n; i++) {
        StepCount sc{};
        const f3 o = V(org[3 * i], org[3 * i + 1], org[3 * i + 2]);
        const f3 d = V(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
        const float t = hround(dist[i]);
        Hit r;
        if (g8) r = col ? trace<true, 8, false, true, false, World, true>(h.w, o, d, t, sc)
                        : trace<true, 8, false, true, false, World, false>(h.w, o, d, t, sc);
        else r = col ? trace<true, 4, false, true, false, World, true>(h.w, o, d, t, sc)
                     : trace<true, 4, false, true, false, World, false>(h.w, o, d, t, sc);
        HostHit& q = out[i];
        q.pos[0] = r.pos.x; q.pos[1] = r.pos.y; q.pos[2] = r.pos.z;
        q.normal[0] = r.normal.x; q.normal[1] = r.normal.y; q.normal[2] = r.normal.z;
        q.u = r.u; q.v = r.v; q.hit = r.hit; q.undef = r.undef;
        q.sphere = (int)sc.sphere; q.dda = (int)sc.dda; q.check = (int)sc.check; q.pad = (int)sc.col_skip;
    }
    return 0;
}

static int trace_rays(int variant, int lx, int ly, int lz, const uint32_t* bits, const uint8_t* csdf, const float* org,
                      const float* dir, const float* dist, int64_t n, HostHit* out, int sky_exit) {
    Hit (*fn)(const World&, f3, f3, float, StepCount&) = nullptr;
    switch (variant) {
    case 0: fn = trace_v<1, false>; break;
    case 1: fn = trace_v<2, false>; break;
    case 2: fn = trace_v<4, false>; break;
    case 3: fn = trace_v<8, false>; break;
    case 4: fn = trace_v<1, true>; break;
    case 5: fn = trace_v<4, false, false>; break;
    case 6: fn = trace_v<8, false, false>; break;
    default: return -1;
    }
    HostWorld h;
    build(h, lx, ly, lz, bits, csdf);
    if (sky_exit) h.w.ytop = world_ytop(h);
    for (int64_t i = 0; i < n; i++) {
        StepCount sc{};
        Hit r = fn(h.w, V(org[3 * i], org[3 * i + 1], org[3 * i + 2]),
                   V(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), hround(dist[i]), sc);
        HostHit& o = out[i];
        o.pos[0] = r.pos.x; o.pos[1] = r.pos.y; o.pos[2] = r.pos.z;
        o.normal[0] = r.normal.x; o.normal[1] = r.normal.y; o.normal[2] = r.normal.z;
        o.u = r.u; o.v = r.v; o.hit = r.hit; o.undef = r.undef;
        o.sphere = (int)sc.sphere; o.dda = (int)sc.dda; o.check = (int)sc.check; o.pad = 0;
    }
    return 0;
}

}  // extern "C"
