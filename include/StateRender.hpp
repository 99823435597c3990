// StateRender.hpp -- header-only C++ facade over the C ABI (rvgrt.h) with
// the reference's host interface, so the reference's host code keeps its
// call sites:
//   class StateRender           <- include/StateRender.cuh:11-47
//   StateRender::drawCUDA(...)  <- src/StateRender.cu:289-346 (same signature)
//   CoarseArray::UpdateGIData   <- src/CoarseArray.cu:376-395 (updateGIData)
//   State::Create init sequence <- src/State.cpp:24-56 (create)
//   Camera                      <- include/Camera.hpp:5-17
// The vector/matrix types are layout-compatible with glm::vec3 / glm::mat4
// (3 floats; 16 floats, column-major).  With glm on the include path define
// RVGRT_USE_GLM to take glm's own types.  Errors throw std::runtime_error
// (as the reference's CUDA_CHECK does, include/cumath.cuh:10-14).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "rvgrt.h"

#ifdef RVGRT_USE_GLM
#include <glm/glm.hpp>
#endif

namespace rvgrt {

#ifdef RVGRT_USE_GLM
using vec3 = glm::vec3;
using mat4 = glm::mat4;
inline const float* data(const vec3& v) { return &v.x; }
inline const float* data(const mat4* m) { return m ? &(*m)[0][0] : nullptr; }
#else
struct vec3 { float x = 0, y = 0, z = 0; };
struct mat4 { float m[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}; };
inline const float* data(const vec3& v) { return &v.x; }
inline const float* data(const mat4* m) { return m ? m->m : nullptr; }
#endif

// include/Camera.hpp:5-17
struct Camera {
    vec3 pos, forward, right, up;
    float cameraMultiplyFactor[2] = {0, 0};
    float cameraAddFactor[2] = {0, 0};
};

inline void check(rv_status s, rv_ctx* c, const char* what) {
    if (s != RV_OK)
        throw std::runtime_error(std::string(what) + " failed (" + std::to_string((int)s) +
                                 "): " + (c ? rv_last_error(c) : ""));
}

struct Settings {
    int log2_x = 12, log2_y = 9, log2_z = 12;   // reference world 4096 x 512 x 4096
    int width = 1280, height = 800;             // reference dispWIDTH x dispHEIGHT
    int flags = RV_FLAGS_REFERENCE;             // INCLUDEGI build
    bool ref_compat = true;                     // c_cam off-by-one
    int device = 0;
};

class StateRender {
public:
    explicit StateRender(const Settings& s = Settings(), const uint8_t* atlas_rgba8 = nullptr, int atlas_w = 256,
                         int atlas_h = 256) : settings_(s) {
        rv_config cfg{};
        cfg.log2_x = s.log2_x; cfg.log2_y = s.log2_y; cfg.log2_z = s.log2_z;
        cfg.width = s.width; cfg.height = s.height; cfg.flags = s.flags;
        cfg.ref_compat = s.ref_compat ? 1 : 0;
        cfg.atlas_rgba8 = atlas_rgba8; cfg.atlas_w = atlas_w; cfg.atlas_h = atlas_h;
        check(rv_create(&cfg, s.device, &ctx_), nullptr, "rv_create");
    }
    ~StateRender() { rv_destroy(ctx_); }
    StateRender(const StateRender&) = delete;
    StateRender& operator=(const StateRender&) = delete;

    // State::Create: CArray::fill -> CoarseArray::GenerateSDF -> InitializeGIData
    void create() { check(rv_world_build(ctx_), ctx_, "rv_world_build"); }

    // CoarseArray::UpdateGIData: RAYPS cells per call, rolling offset
    void updateGIData() { check(rv_update_gi_data(ctx_), ctx_, "rv_update_gi_data"); }

    // StateRender::drawCUDA, identical parameter list and order
    void drawCUDA(const vec3& pos, const vec3& fo, const vec3& up, const vec3& ri,
                  mat4* unjitteredViewProjectionMatrix, mat4* prevUnjitteredViewProjectionMatrix,
                  float jitterX, float jitterY) {
        check(rv_draw_cuda(ctx_, data(pos), data(fo), data(up), data(ri), data(unjitteredViewProjectionMatrix),
                           data(prevUnjitteredViewProjectionMatrix), jitterX, jitterY),
              ctx_, "rv_draw_cuda");
    }

    // Offscreen replacement of the D3D12 present: RGBA8, tightly packed rows
    std::vector<uint8_t> readbackColor() {
        std::vector<uint8_t> px((size_t)settings_.width * settings_.height * 4);
        check(rv_readback(ctx_, RV_IMAGE_COLOR, px.data(), 0), ctx_, "rv_readback");
        return px;
    }

    // Bind caller-owned device buffers like the reference's interop heaps
    void bindOutput(rv_image_kind kind, void* devPtr, size_t pitch) {
        check(rv_bind_output(ctx_, kind, devPtr, pitch), ctx_, "rv_bind_output");
    }

    static Camera cameraFromPose(float px, float py, float pz, float yaw, float pitch, int w, int h, mat4* vp) {
        rv_camera c{};
        check(rv_camera_from_pose(px, py, pz, yaw, pitch, w, h, &c, vp ? const_cast<float*>(data(vp)) : nullptr),
              nullptr, "rv_camera_from_pose");
        Camera out;
        out.pos = {c.pos[0], c.pos[1], c.pos[2]};
        out.forward = {c.forward[0], c.forward[1], c.forward[2]};
        out.right = {c.right[0], c.right[1], c.right[2]};
        out.up = {c.up[0], c.up[1], c.up[2]};
        for (int i = 0; i < 2; i++) { out.cameraMultiplyFactor[i] = c.mul[i]; out.cameraAddFactor[i] = c.add[i]; }
        return out;
    }

    void sync() { check(rv_sync(ctx_), ctx_, "rv_sync"); }
    rv_ctx* handle() { return ctx_; }
    const Settings& settings() const { return settings_; }

private:
    Settings settings_;
    rv_ctx* ctx_ = nullptr;
};

}  // namespace rvgrt
