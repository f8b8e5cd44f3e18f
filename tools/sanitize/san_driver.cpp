// san_driver.cpp -- host sanitizer harness ("host ASan/UBSan on
// the oracle", TSan on the threaded BVH builder).  Built from the scene
// library's sources and the oracle with -fsanitize=... by tools/sanitize/
// Makefile, so the instrumented code runs in an instrumented executable (no
// preloading into Python).  Test infrastructure; not part of the product.
//
//   san_driver decode FILE...   every image decoder LoadTexture reaches
//                               (LoadImageFloat, LoadImageRGBA8): "ok W H" or
//                               "error: ..." per file; a crash or sanitizer
//                               report is the failure
//   san_driver model FILE...    LoadModelAsPrefab (OBJ/MTL + textures) + PackSceneData
//   san_driver scene FILE...    LoadScene + PackSceneData
//   san_driver render           configs C1-C5 packed; oracle Reset/Run(2)/Run(1)
//                               on small frames, resolve, preview
//   san_driver bvh FACES        random triangle soup through CreateMesh (the
//                               threaded builder, PT_BVH_THREADS) + PackSceneData
#include "../../path-tracer_amd/csrc/scene/scene.hpp"
#include "../../path-tracer_amd/csrc/scene/configs.hpp"
#include "../../path-tracer_amd/csrc/scene/image.hpp"
#include "../../oracle/pt_oracle.h"

#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

using namespace pth;

static int Decode(int argc, char** argv)
{
    for (int i = 0; i < argc; i++) {
        int w = 0, h = 0;
        std::vector<uint8_t> rgba;
        std::string e1;
        FILE* fp = std::fopen(argv[i], "rb");
        char magic[2] = {0, 0};
        if (fp) { (void)!std::fread(magic, 1, 2, fp); std::fclose(fp); }
        if (magic[0] == '#' && magic[1] == '?') {   // Radiance HDR: the float path only
            std::vector<vec4> px;
            if (LoadImageFloat(argv[i], w, h, px, e1)) std::printf("%s: ok %d %d\n", argv[i], w, h);
            else std::printf("%s: error: %s\n", argv[i], e1.c_str());
            continue;
        }
        if (!LoadImageRGBA8(argv[i], w, h, rgba, e1)) {
            std::printf("%s: error: %s\n", argv[i], e1.c_str());
            continue;
        }
        std::printf("%s: ok %d %d\n", argv[i], w, h);
        // LoadTexture's float path (16 B/px) only for images of sane size:
        // the crafted huge-but-legal headers of the corpus would otherwise
        // allocate gigabytes under ASan.
        if ((uint64_t)w * (uint64_t)h <= (16u << 20)) {
            std::vector<vec4> px;
            std::string e2;
            int w2 = 0, h2 = 0;
            if (!LoadImageFloat(argv[i], w2, h2, px, e2) || w2 != w || h2 != h)
                std::printf("%s: float path disagrees: %s\n", argv[i], e2.c_str());
        }
    }
    return 0;
}

static int Model(int argc, char** argv)
{
    for (int i = 0; i < argc; i++) {
        scene* s = CreateScene();
        load_model_options opt;
        std::string err;
        prefab* p = LoadModelAsPrefab(s, argv[i], &opt, &err);
        if (p) {
            CreateEntity(s, p, nullptr);
            PackSceneData(s);
            std::printf("%s: ok\n", argv[i]);
        } else {
            std::printf("%s: error: %s\n", argv[i], err.c_str());
        }
        DestroyScene(s);
    }
    return 0;
}

static int Scene(int argc, char** argv)
{
    for (int i = 0; i < argc; i++) {
        std::string err;
        scene* s = LoadScene(argv[i], &err);
        if (s) {
            PackSceneData(s);
            std::printf("%s: ok\n", argv[i]);
            DestroyScene(s);
        } else {
            std::printf("%s: error: %s\n", argv[i], err.c_str());
        }
    }
    return 0;
}

static int Render()
{
    for (int c = 1; c <= 5; c++) {
        config_info info{};
        scene* s = CreateConfigScene(c, &info);
        if (!s) { std::printf("C%d: no scene\n", c); return 1; }
        pt_scene_packs packs{};
        GetScenePacks(s, &packs);
        const uint32_t W = 48, H = 40;
        for (uint32_t nranks : {1u, 2u}) {
            oracle_renderer* o = oracle_create(&packs, W, H, 0, nranks, 4);
            pt_basic_renderer_params* P = oracle_params(o);
            P->RenderFlags = 3;
            P->CameraIndex = c == 5 ? 1 : 0;
            oracle_reset(o);
            oracle_run(o, 2);
            oracle_run(o, 1);
            std::vector<float> acc(4 * W * H);
            oracle_read_accum(o, acc.data());
            std::vector<pt_pixel_state> st(W * H);
            oracle_read_state(o, st.data());
            std::vector<float> out(4 * W * H);
            std::vector<uint8_t> out8(4 * W * H);
            pt_resolve_parameters rp{1.0f, 3, 1.0f};
            oracle_resolve(acc.data(), W * H, &rp, out.data(), out8.data());
            uint64_t rays = 0, samples = 0;
            oracle_counters(o, &rays, &samples);
            std::printf("C%d nranks %u: rays %llu samples %llu\n", c, nranks, (unsigned long long)rays,
                        (unsigned long long)samples);
            oracle_destroy(o);
        }
        pt_preview_parameters pp{};
        std::memcpy(&pp.CameraTransform, &packs.cameras[0].Transform, sizeof(pp.CameraTransform));
        pp.RenderMode = 1; pp.Brightness = 1; pp.SelectedShapeIndex = 0xFFFFFFFFu;
        pp.RenderSizeX = 32; pp.RenderSizeY = 24; pp.MouseX = 3; pp.MouseY = 4;
        std::vector<float> img(4 * 32 * 24);
        std::vector<pt_preview_aov> aov(32 * 24);
        uint32_t q = 0;
        oracle_preview(&packs, &pp, img.data(), aov.data(), &q);
        DestroyScene(s);
    }
    return 0;
}

static int Bvh(uint32_t faces)
{
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> u(-10.0f, 10.0f), d(-0.3f, 0.3f);
    std::vector<float> pos(9 * (size_t)faces);
    std::vector<uint32_t> idx(3 * (size_t)faces);
    for (uint32_t f = 0; f < faces; f++) {
        float cx = u(rng), cy = u(rng), cz = u(rng);
        for (int k = 0; k < 3; k++) {
            pos[9 * (size_t)f + 3 * k + 0] = cx + d(rng);
            pos[9 * (size_t)f + 3 * k + 1] = cy + d(rng);
            pos[9 * (size_t)f + 3 * k + 2] = cz + d(rng);
            idx[3 * (size_t)f + k] = 3 * f + k;
        }
    }
    scene* s = CreateScene();
    mesh* m = CreateMesh(s, "soup", 3 * faces, pos.data(), nullptr, nullptr, faces, idx.data());
    entity* e = CreateEntity(s, ENTITY_TYPE_MESH_INSTANCE, nullptr);
    e->Mesh = m;
    PackSceneData(s);
    std::printf("bvh: %u faces, %zu nodes, depth %u\n", faces, m->Nodes.size(), m->Depth);
    DestroyScene(s);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) { std::fprintf(stderr, "usage: san_driver decode|model|scene|render|bvh ...\n"); return 2; }
    std::string cmd = argv[1];
    if (cmd == "decode") return Decode(argc - 2, argv + 2);
    if (cmd == "model") return Model(argc - 2, argv + 2);
    if (cmd == "scene") return Scene(argc - 2, argv + 2);
    if (cmd == "render") return Render();
    if (cmd == "bvh") return Bvh(argc > 2 ? (uint32_t)std::strtoul(argv[2], nullptr, 10) : 200000u);
    std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
    return 2;
}
