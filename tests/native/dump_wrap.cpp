// tests/native/dump_wrap.cpp -- TEST INFRASTRUCTURE for build_inref.sh: linked with
// -Wl,--wrap=<SaveFloatImageToJpg>, it writes the float framebuffer Renderer::Render
// hands to SaveFloatImageToJpg (SceneRenderingHelper.cpp:57-70) to $TPT_DUMP as raw
// fp32 (W*H*3), then calls the reference's own function.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "Vector.hpp"

void real_save(std::vector<Vector3f> fb, int w, int h, std::string path) __asm__(
    "__real__Z19SaveFloatImageToJpgSt6vectorI8Vector3fSaIS0_EEiiNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEE");
void wrapped_save(std::vector<Vector3f> fb, int w, int h, std::string path) __asm__(
    "__wrap__Z19SaveFloatImageToJpgSt6vectorI8Vector3fSaIS0_EEiiNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEE");
void wrapped_save(std::vector<Vector3f> fb, int w, int h, std::string path) {
    if (const char* dump = std::getenv("TPT_DUMP")) {
        if (FILE* f = std::fopen(dump, "wb")) {
            for (int i = 0; i < w * h; ++i) {
                const float v[3] = {fb[i].x, fb[i].y, fb[i].z};
                std::fwrite(v, sizeof(float), 3, f);
            }
            std::fclose(f);
        }
    }
    real_save(fb, w, h, path);
}
