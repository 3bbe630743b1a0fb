// tpt_render -- the reference's CLI (main.cpp:14-46, 147-148) on the GPU path.
// Flags and defaults as the reference: -o output.jpg, -spp 1, -j 8 (accepted,
// unused by the GPU path), -bdpt 1.  Additions: -scene <preset> (default
// "silver" = main.cpp HEAD), -models <dir>, -dump <file.f32>, -device <n>, -gpus <n>,
// -pti 1 (PathTrace with the indirect bounce, TPT_MODE_PT_INDIRECT; with -bdpt 0).
#include <iostream>
#include <sstream>
#include <string>

#include "../../include/tpt_scene_api.hpp"

template <typename T>
T tryParseArg(int argc, char** argv, const char* name, const T& def) {  // main.cpp:14-26
    for (int i = 0; i < argc; i++) {
        if (std::string(argv[i]) == name && i + 1 != argc) {
            T v;
            std::stringstream ss(argv[i + 1]);
            ss >> v;
            return v;
        }
    }
    return def;
}

#ifndef TPT_DEFAULT_MODELS
#define TPT_DEFAULT_MODELS "models"
#endif

int main(int argc, char** argv) {
    std::string out = tryParseArg(argc, argv, "-o", std::string("output.jpg"));
    int spp = tryParseArg(argc, argv, "-spp", 1);
    int threads = tryParseArg(argc, argv, "-j", 8);
    bool bdpt = tryParseArg(argc, argv, "-bdpt", 1);
    std::string preset = tryParseArg(argc, argv, "-scene", std::string("silver"));
    std::string models = tryParseArg(argc, argv, "-models", std::string(TPT_DEFAULT_MODELS));
    RenderOptions opt;
    opt.float_dump = tryParseArg(argc, argv, "-dump", std::string());
    opt.device = tryParseArg(argc, argv, "-device", 0);
    opt.gpus = tryParseArg(argc, argv, "-gpus", 1);  // >1: tpt_render_multi over devices device..device+gpus-1
    opt.pt_indirect = tryParseArg(argc, argv, "-pti", 0) != 0;  // off by default
    Scene scene(784, 784);
    if (!BuildPresetScene(models, preset, scene)) {
        std::cerr << "unknown scene preset or missing models: " << preset << " (" << models << ")\n";
        return 2;
    }
    Renderer r;
    r.Render(out, scene, spp, threads, bdpt, opt);
    return r.last_error ? 1 : 0;
}
