// rv_render -- C++ host driver of the render path: the reference's
// renderLoop (src/main.cpp:104-234) minus Win32/D3D12/DLSS, which the north
// star replaces with an offscreen framebuffer dump.  Uses only the C++
// facade include/StateRender.hpp over the C ABI (no HIP headers).
//
//   rv_render [--config c1..c5] [--frames N] [--warmup N] [--out frame.ppm]
//             [--atlas texturepack.png] [--lg L] [--res WxH] [--flags F]
//             [--sweeps S] [--gi-per-frame 0|1] [--pose x,y,z,yaw,pitch]
// --config picks a BASELINE configuration; the other options override its
// world size, resolution, RV_F_* flags, GI sweeps, per-frame GI update and
// camera pose (default: the reference's defaults scaled to the world,
// src/Character.cpp:30,45-46).  Frames go through drawCUDA with the
// reference's ref_compat settings (Settings defaults).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include <zlib.h>

#include "StateRender.hpp"

namespace {

struct Cfg { const char* name; int lg, w, h, flags, sweeps; bool gi_per_frame; };
const Cfg kConfigs[] = {
    {"c1", 8, 640, 360, 0, -1, false},
    {"c2", 9, 1920, 1080, RV_F_SHADOW, -1, false},
    {"c3", 10, 1920, 1080, RV_FLAGS_REFERENCE, 1, true},
    {"c4", 10, 3840, 2160, RV_FLAGS_REFERENCE, 2, true},
    {"c5", 11, 3840, 2160, RV_FLAGS_REFERENCE, 2, true},
};

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// Minimal PNG decoder: 8-bit RGB/RGBA, non-interlaced (the reference atlas
// is 256x256 RGBA; src/Texturepack.cu:20-33 decodes it with stb_image).
bool decode_png(const std::vector<uint8_t>& f, std::vector<uint8_t>& rgba, int& w, int& h) {
    if (f.size() < 8 || std::memcmp(f.data(), "\x89PNG\r\n\x1a\n", 8) != 0) return false;
    std::vector<uint8_t> idat;
    int bpp = 0;
    for (size_t p = 8; p + 8 <= f.size();) {
        uint32_t len = be32(&f[p]);
        const char* t = (const char*)&f[p + 4];
        const uint8_t* d = &f[p + 8];
        if (!std::strncmp(t, "IHDR", 4)) {
            w = (int)be32(d); h = (int)be32(d + 4);
            if (d[8] != 8 || (d[9] != 6 && d[9] != 2) || d[12] != 0) return false;
            bpp = d[9] == 6 ? 4 : 3;
        } else if (!std::strncmp(t, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::strncmp(t, "IEND", 4)) {
            break;
        }
        p += 12 + len;
    }
    if (!bpp) return false;
    size_t stride = (size_t)w * bpp;
    std::vector<uint8_t> raw((stride + 1) * h);
    uLongf n = raw.size();
    if (uncompress(raw.data(), &n, idat.data(), idat.size()) != Z_OK) return false;
    std::vector<uint8_t> img(stride * h), prev(stride, 0);
    for (int y = 0; y < h; y++) {
        uint8_t ft = raw[y * (stride + 1)];
        const uint8_t* in = &raw[y * (stride + 1) + 1];
        uint8_t* cur = &img[y * stride];
        for (size_t i = 0; i < stride; i++) {
            int a = i >= (size_t)bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= (size_t)bpp ? prev[i - bpp] : 0;
            int pr = 0;
            if (ft == 1) pr = a;
            else if (ft == 2) pr = b;
            else if (ft == 3) pr = (a + b) >> 1;
            else if (ft == 4) {
                int q = a + b - c, pa = std::abs(q - a), pb = std::abs(q - b), pc = std::abs(q - c);
                pr = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
            }
            cur[i] = (uint8_t)(in[i] + pr);
        }
        std::memcpy(prev.data(), cur, stride);
    }
    rgba.resize((size_t)w * h * 4);
    for (size_t i = 0; i < (size_t)w * h; i++)
        for (int k = 0; k < 4; k++) rgba[i * 4 + k] = k < bpp ? img[i * bpp + k] : 255;
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    std::string config = "c2", out = "frame.ppm", atlas_path = "rvgrt_amd/assets/texturepack.png";
    int frames = 60, warmup = 5;
    int lg = -1, w = -1, h = -1, flags = -1, sweeps = -2, gpf = -1;
    float pose[5] = {0, 0, 0, 0, 0};
    bool have_pose = false;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i];
        const char* v = argv[i + 1];
        if (k == "--config") config = v;
        else if (k == "--frames") frames = std::atoi(v);
        else if (k == "--warmup") warmup = std::atoi(v);
        else if (k == "--out") out = v;
        else if (k == "--atlas") atlas_path = v;
        else if (k == "--lg") lg = std::atoi(v);
        else if (k == "--res") { if (std::sscanf(v, "%dx%d", &w, &h) != 2) { std::fprintf(stderr, "bad --res\n"); return 2; } }
        else if (k == "--flags") flags = std::atoi(v);
        else if (k == "--sweeps") sweeps = std::atoi(v);
        else if (k == "--gi-per-frame") gpf = std::atoi(v);
        else if (k == "--pose") {
            if (std::sscanf(v, "%f,%f,%f,%f,%f", &pose[0], &pose[1], &pose[2], &pose[3], &pose[4]) != 5) {
                std::fprintf(stderr, "bad --pose\n");
                return 2;
            }
            have_pose = true;
        } else { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    }
    const Cfg* base = nullptr;
    for (const Cfg& c : kConfigs) if (config == c.name) base = &c;
    if (!base) { std::fprintf(stderr, "unknown config %s\n", config.c_str()); return 2; }
    Cfg cfg_v = *base;
    if (lg > 0) cfg_v.lg = lg;
    if (w > 0) { cfg_v.w = w; cfg_v.h = h; }
    if (flags >= 0) cfg_v.flags = flags;
    if (sweeps >= -1) cfg_v.sweeps = sweeps;
    if (gpf >= 0) cfg_v.gi_per_frame = gpf != 0;
    const Cfg* cfg = &cfg_v;

    std::vector<uint8_t> atlas;
    int aw = 0, ah = 0;
    {
        std::ifstream f(atlas_path, std::ios::binary);
        std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        if (!decode_png(bytes, atlas, aw, ah)) { std::fprintf(stderr, "cannot decode %s\n", atlas_path.c_str()); return 2; }
    }
    try {
        rvgrt::Settings s;
        s.log2_x = s.log2_y = s.log2_z = cfg->lg;
        s.width = cfg->w; s.height = cfg->h; s.flags = cfg->flags;
        rvgrt::StateRender render(s, atlas.data(), aw, ah);
        auto t0 = std::chrono::steady_clock::now();
        render.create();
        for (int k = 0; k < cfg->sweeps; k++) rvgrt::check(rv_gi_update(render.handle(), k, 0, ~0ull >> 1), render.handle(), "rv_gi_update");
        render.sync();
        double build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        int n = 1 << cfg->lg;
        rvgrt::mat4 vp;
        if (!have_pose) {
            pose[0] = 0.1f * n; pose[1] = std::fmin(0.6f * n, 350.0f); pose[2] = 0.1f * n;
            pose[3] = -0.7f; pose[4] = (float)(-M_PI - 0.3);
        }
        rvgrt::Camera cam = rvgrt::StateRender::cameraFromPose(pose[0], pose[1], pose[2], pose[3], pose[4], cfg->w,
                                                               cfg->h, &vp);
        rvgrt::mat4 prev = vp;
        auto frame = [&]() {
            if (cfg->gi_per_frame) render.updateGIData();      // renderLoop order (main.cpp:119-132)
            render.drawCUDA(cam.pos, cam.forward, cam.up, cam.right, &vp, &prev, 0.0f, 0.0f);
        };
        for (int k = 0; k < warmup; k++) frame();
        render.sync();
        t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < frames; k++) frame();
        render.sync();
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() /
                    std::max(frames, 1);
        std::vector<uint8_t> px = render.readbackColor();
        std::FILE* f = std::fopen(out.c_str(), "wb");
        std::fprintf(f, "P6\n%d %d\n255\n", cfg->w, cfg->h);
        for (size_t i = 0; i < (size_t)cfg->w * cfg->h; i++) std::fwrite(&px[i * 4], 1, 3, f);
        std::fclose(f);
        std::printf("{\"config\": \"%s\", \"world_build_ms\": %.3f, \"ms_per_frame\": %.4f, \"fps\": %.2f, \"dump\": \"%s\"}\n",
                    cfg->name, build_ms, ms, 1000.0 / ms, out.c_str());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "rv_render: %s\n", e.what());
        return 1;
    }
    return 0;
}
