// mcpt_qe_viewer.hpp -- header-only progressive viewer adapter over mcpt.h.
//
// Stands in for the QuinEngine RTX renderer behind Quin::Core::Graphics
// (MCRT/QuinEngine/Core/Graphics.hpp:17-20: Initialize / Shutdown / OnUpdate),
// whose per-frame work is GraphicsRTX::DoOnUpdate (QE/RTX/GraphicsRTX.cpp:163-232):
//   * scene01 loaded once (tinyobjloader), KD tree built once        (:165-167)
//   * camera LookAtRH (0,5,17)->(0,5,16), PerspectiveFovRH(pi/4, W/H) (:173-184)
//   * frame seed = uniform_int_distribution<unsigned>(mt19937(1234)),
//     prevCount = frame counter                                        (:168-193)
//   * one sample per pixel, gamma-2.2 running mean into the screen     (rtx.hlsl:373-404)
//   * every 100th frame the render target is saved as "temp.png"     (:216-219)
// The D3D11 swap chain / Win32 message pump are not reproduced: Screen()
// returns the host copy of the render target that a window would present.
#pragma once

#include <cstdint>
#include <random>
#include <string>
#include <vector>

#include "mcpt.h"
#include "mcpt_image_io.hpp"

namespace mcpt {
namespace qe {

class Viewer {
public:
    Viewer() = default;
    ~Viewer() { Shutdown(); }
    Viewer(const Viewer&) = delete;
    Viewer& operator=(const Viewer&) = delete;

    // GraphicsRTX::Initialize + the static scene setup of DoOnUpdate
    // QuinEngine reads its scene through tinyobjloader (QE/Utils/Structure.hpp:9-12),
    // hence the default flavor; its window is 640x480 (QE/Main.cpp:11)
    int Initialize(const std::string& obj_path, uint32_t width = 640, uint32_t height = 480, int32_t device = 0,
                   int32_t flavor = MCPT_OBJ_TINYOBJ) {
        Shutdown();
        int rc = mcpt_init(&device, 1);
        if (rc != MCPT_OK) return rc;
        mcpt_model* m = nullptr;
        rc = mcpt_model_read_obj_ex(obj_path.c_str(), flavor, &m);
        if (rc != MCPT_OK) return rc;
        rc = mcpt_scene_create(m, &scene_);
        mcpt_model_free(m);
        if (rc != MCPT_OK) return rc;
        mcpt_render_params_quinengine(&p_);
        p_.width = static_cast<int32_t>(width);
        p_.height = static_cast<int32_t>(height);
        screen_.assign(static_cast<size_t>(width) * height * 3, 0.0f);
        rng_.seed(1234);
        frames_ = 0;
        return MCPT_OK;
    }

    void Shutdown() {
        if (scene_) mcpt_scene_destroy(scene_);
        scene_ = nullptr;
    }

    // One progressive frame (GraphicsRTX::DoOnUpdate); 0 on success
    int OnUpdate() {
        if (!scene_) return MCPT_E_INVALID;
        last_seed_ = dist_(rng_);
        p_.seed = last_seed_;
        p_.prev_count = frames_++;
        const int rc = mcpt_render(scene_, &p_, screen_.data(), nullptr);
        if (rc != MCPT_OK) return rc;
        if (save_every_ > 0 && frames_ % static_cast<uint32_t>(save_every_) == 0)
            image::write_png(save_path_, screen_.data(), p_.width, p_.height);
        return MCPT_OK;
    }

    // save the screen every n frames (the reference: 100, "temp.png"); 0 = never
    void SetSaveEvery(int n, const std::string& path = "temp.png") { save_every_ = n; save_path_ = path; }

    const float* Screen() const { return screen_.data(); }     // gamma-encoded RGB, row-major
    uint32_t Frames() const { return frames_; }
    uint32_t LastSeed() const { return last_seed_; }
    mcpt_render_params& Params() { return p_; }                 // camera / depth overrides

private:
    mcpt_scene* scene_ = nullptr;
    mcpt_render_params p_{};
    std::vector<float> screen_;
    std::mt19937 rng_{1234};
    std::uniform_int_distribution<unsigned int> dist_;
    uint32_t frames_ = 0, last_seed_ = 0;
    int save_every_ = 0;
    std::string save_path_ = "temp.png";
};

}  // namespace qe
}  // namespace mcpt
