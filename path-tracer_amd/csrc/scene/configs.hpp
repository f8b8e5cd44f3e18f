// configs.hpp — benchmark scene builders (BASELINE.json configs C1..C5).
#pragma once

#include "scene.hpp"

#define PT_RENDER_FLAG_ACCUMULATE_ 1u
#define PT_RENDER_FLAG_JITTER_ 2u

namespace pth {

struct config_info {
    uint32_t width, height;
    uint32_t spp;
    uint32_t camera_count;
    uint32_t render_flags;
    float termination_probability;
    uint32_t mesh_face_count;
    uint32_t shape_count;
};

// Builds and packs config 1..5; returns nullptr for an unknown id.
scene* CreateConfigScene(int config, config_info* info);

}  // namespace pth
