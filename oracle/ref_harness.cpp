// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped, never measured
// as the product).  Linked against the reference's own object files (compiled
// in place from /root/reference by oracle/build_ref.sh) to produce
// oracle/_ref/libref.so: the *real* reference renderer behind a small C ABI, used
// to pin the CPU restatement (oracle/tpt_oracle.cpp) and to generate the golden
// fixtures under tests/golden/.
//
// Scene presets mirror the reference's hard-coded scene in main.cpp:49-103
// (materials :52-81, meshes :83-93, Add order :95-102, BuildBVH :103); the
// variants (standard / refractive_ball / occlusion / smooth_dielectric / bunny)
// follow SURVEY.md §8(d).
//
// Per-pixel replay mirrors FillBufferThread (Renderer.cpp:32-63): ResetRandom(i+1)
// once per pixel, then a serial spp loop accumulating (1.0f/spp) * L.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "global.hpp"
#include "Renderer.hpp"
#include "Scene.hpp"
#include "Triangle.hpp"
#include "Sphere.hpp"
#include "Material.hpp"
#include "GGX.hpp"
#include "SceneRenderingHelper.hpp"
#include "SampleHelperFunctions.hpp"
#include "PathTracer.hpp"
#include "BDPT.hpp"

// ---------------------------------------------------------------------------
// Framebuffer capture: Renderer::Render ends with SaveFloatImageToJpg(fb, ...)
// (Renderer.cpp:126).  The link uses -Wl,--wrap=<mangled name>, so that call
// lands here; we copy the float framebuffer out instead of writing a JPEG.
static float* g_capture = nullptr;
void wrapped_save(std::vector<Vector3f> fb, int w, int h, std::string path) __asm__(
    "__wrap__Z19SaveFloatImageToJpgSt6vectorI8Vector3fSaIS0_EEiiNSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEE");
void wrapped_save(std::vector<Vector3f> fb, int w, int h, std::string) {
    if (!g_capture) return;
    for (int i = 0; i < w * h; ++i) {
        g_capture[3 * i + 0] = fb[i].x;
        g_capture[3 * i + 1] = fb[i].y;
        g_capture[3 * i + 2] = fb[i].z;
    }
}

// Renderer.cpp:29 -- FillBufferThread reads the scene through this global.
extern const Scene* curScene;

// PathTracer.cpp compiled a second time without the HEAD `break` (:109), see
// oracle/build_ref.sh: the reference for TPT_MODE_PT_INDIRECT.
Vector3f PathTraceIndirect(const Scene* scene, const Ray& ray, int& outBounces);

namespace {
struct Preset {
    Scene* scene = nullptr;
    std::vector<Material*> mats;
    std::vector<Object*> objs;
};
Preset g;

Material* keep(Material* m) { g.mats.push_back(m); return m; }
}

extern "C" {

// Build one of the named presets.  Returns 0 on success, -1 on an unknown preset.
// Edge-case presets (builder-declared, VERDICT r1 "Missing" #4), all on the standard
// box: "multi_light" adds the reference's light2.obj / light3.obj as two more
// emitters (PathTracer.cpp:82 loops over all of them); "emissive_sphere" adds a
// glowing Sphere ahead of the light, so it is m_emissionObjects[0] (BDPT.cpp:287
// starts every light path on it: Sphere::Sample, Sphere.cpp:48-55); "background"
// keeps Scene.hpp:23's default backgroundColor instead of main.cpp:51's 0 (read by
// BDPT.cpp:182 and BDPT.hpp:124).
int ref_setup(const char* models_dir, const char* preset, int width, int height) {
    std::string dir(models_dir);
    std::string p(preset);
    g = Preset();
    Scene* scene = new Scene(width, height);
    scene->eyePos = Vector3f(278, 278, -800);
    if (p != "background") scene->backgroundColor = 0.0f;
    Material* red = keep(new Material(Dieletric, Vector3f(0.0f)));
    red->Kd = Vector3f(0.63f, 0.065f, 0.05f);
    Material* green = keep(new Material(Dieletric, Vector3f(0.0f)));
    green->Kd = Vector3f(0.14f, 0.45f, 0.091f);
    Material* white = keep(new Material(Dieletric, Vector3f(0.0f)));
    white->Kd = Vector3f(0.725f, 0.71f, 0.68f);
    // main.cpp:58 uses .1f; the smooth_dielectric preset's value is not in HEAD and
    // is declared here -- both sides of every parity test use it.
    white->SetSmoothness(p == "smooth_dielectric" ? 0.7f : .1f);
    Material* light = keep(new Material(Dieletric, (8.0f * Vector3f(0.747f + 0.058f, 0.747f + 0.258f, 0.747f) +
                                                  15.6f * Vector3f(0.740f + 0.287f, 0.740f + 0.160f, 0.740f) +
                                                  18.4f * Vector3f(0.737f + 0.642f, 0.737f + 0.159f, 0.737f))));
    light->Kd = Vector3f(0.65f);
    Material* silver = keep(new Material(Metal));
    silver->ior_m = Vector3f(0.041000f, 0.53285f, 0.049317f);
    silver->ior_m_k = Vector3f(4.8025f, 3.4101f, 2.8545f);
    silver->SetSmoothness(1.f);
    Material* glass = keep(new Material(Transparent));
    glass->ior_d = 1.5f;
    glass->SetSmoothness(.9f);

    Material* lightball = keep(new Material(Dieletric, Vector3f(3.0f, 2.4f, 1.5f)));
    lightball->Kd = Vector3f(0.65f);

    Material* boxes = nullptr;
    if (p == "silver") boxes = silver;
    else if (p == "standard" || p == "refractive_ball" || p == "occlusion" || p == "smooth_dielectric" || p == "bunny" ||
             p == "multi_light" || p == "emissive_sphere" || p == "background")
        boxes = white;
    else return -1;

    auto mesh = [&](const char* f, Material* m) {
        MeshTriangle* t = new MeshTriangle(dir + "/" + f, m);
        g.objs.push_back(t);
        return t;
    };
    if (p == "bunny") {
        scene->Add(mesh("floor.obj", white));
        scene->Add(mesh("left.obj", red));
        scene->Add(mesh("right.obj", green));
        scene->Add(mesh("light.obj", light));
        scene->Add(mesh("bunny_cornell.obj", white));
    } else {
        scene->Add(mesh("floor.obj", boxes));
        scene->Add(mesh("shortbox.obj", boxes));
        scene->Add(mesh("tallbox.obj", boxes));
        scene->Add(mesh("left.obj", red));
        scene->Add(mesh("right.obj", green));
        if (p == "emissive_sphere") {
            Sphere* s = new Sphere(Vector3f(420.0f, 60.0f, 150.0f), 60.0f, lightball);
            g.objs.push_back(s);
            scene->Add(s);
        }
        scene->Add(mesh("light.obj", light));
        if (p == "multi_light") {
            scene->Add(mesh("light2.obj", light));
            scene->Add(mesh("light3.obj", light));
        }
        if (p == "refractive_ball") {
            Sphere* s = new Sphere(Vector3f(278.0f, 278.0f, 200.0f), 50.0f, glass);
            g.objs.push_back(s);
            scene->Add(s);
        }
        if (p == "occlusion") scene->Add(mesh("lightocculuder.obj", white));
    }
    scene->BuildBVH();
    g.scene = scene;
    curScene = scene;
    return 0;
}

// Full image through the real Renderer::Render (Renderer.cpp:68-127).
void ref_render(int spp, int threads, int bdpt, float* out_rgb) {
    g_capture = out_rgb;
    Renderer r;
    r.Render("/dev/null", *g.scene, spp, threads, bdpt != 0);
    g_capture = nullptr;
}

// Per-pixel replay (Renderer.cpp:38-60) for an arbitrary pixel subset; mode
// `bdpt`: 0 PathTrace, 1 BDPT, 2 PathTraceIndirect.  `splat`
// (W*H*3, may be null) receives the t=1 light-tracing splats of those pixels,
// already scaled by 1/spp as in Renderer.cpp:58-60.  `bounces` (may be null)
// receives the per-pixel outBounces sum.
void ref_trace_pixels(int bdpt, int spp, const int64_t* pix, int n, float* out_rgb, float* splat, int64_t* bounces) {
    const Scene* s = g.scene;
    float scale = CalculateScale(s->fov);
    std::vector<Vector3f> emission(s->width * s->height);
    for (int k = 0; k < n; ++k) {
        int64_t i = pix[k];
        int xPixel = i % s->width, yPixel = i / s->width;
        ResetRandom((int)i + 1);
        Vector3f acc;
        int64_t nb = 0;
        for (int ispp = 0; ispp < spp; ++ispp) {
            Vector3f dir = PixelPosToRay(xPixel, yPixel, s->width, s->height, scale);
            int b = 0;
            if (bdpt == 1) acc += (1.0f / spp) * BDPT(s, Ray(s->eyePos, dir), b, &emission[0]);
            else if (bdpt == 2) acc += (1.0f / spp) * PathTraceIndirect(s, Ray(s->eyePos, dir), b);
            else acc += (1.0f / spp) * PathTrace(s, Ray(s->eyePos, dir), b);
            nb += b;
        }
        out_rgb[3 * k + 0] = acc.x; out_rgb[3 * k + 1] = acc.y; out_rgb[3 * k + 2] = acc.z;
        if (bounces) bounces[k] = nb;
    }
    if (splat) {
        for (int i = 0; i < s->width * s->height; ++i) {
            Vector3f e = emission[i] * 1.0f / spp;
            splat[3 * i + 0] = e.x; splat[3 * i + 1] = e.y; splat[3 * i + 2] = e.z;
        }
    }
}

// XorShift32 / GetRandomFloat stream (global.cpp:5-22).
void ref_rng(uint32_t seed, int n, uint32_t* out_u32, float* out_f) {
    ResetRandom((int)seed);
    for (int i = 0; i < n; ++i) out_u32[i] = XorShift32();
    ResetRandom((int)seed);
    for (int i = 0; i < n; ++i) out_f[i] = GetRandomFloat();
}

// Closest-hit queries through Scene::Intersect (Scene.cpp:21-35).
// out: per ray {hit, x.xyz, N.xyz, object-ordinal} ; ordinal = index of the hit
// Triangle/Sphere in the scene's depth-first enumeration (meshes in Add order,
// triangles in file order), -1 on miss.
void ref_intersect(const float* rays, int n, int cull, float* out) {
    const Scene* s = g.scene;
    // ordinal map
    std::vector<std::pair<Object*, int>> ords;
    int ord = 0;
    for (Object* o : s->objects) {
        if (auto* m = dynamic_cast<MeshTriangle*>(o)) {
            for (auto& t : m->triangles) ords.push_back({&t, ord++});
        } else ords.push_back({o, ord++});
    }
    for (int k = 0; k < n; ++k) {
        const float* r = rays + 6 * k;
        Ray ray(Vector3f(r[0], r[1], r[2]), Vector3f(r[3], r[4], r[5]));
        PTVertex v = s->Intersect(ray, (FaceCulling)cull);
        float* o = out + 8 * k;
        o[0] = v.type == PTVertex::Type::Background ? 0.f : 1.f;
        o[1] = v.x.x; o[2] = v.x.y; o[3] = v.x.z;
        o[4] = v.N.x; o[5] = v.N.y; o[6] = v.N.z;
        o[7] = -1.f;
        for (auto& pr : ords) if (pr.first == v.obj) { o[7] = (float)pr.second; break; }
    }
}

// Material KATs (Material.cpp:11-72, 105-147, 150-214, 221-252).
// mat: {type, ior_d, ior_m.xyz, ior_m_k.xyz, Kd.xyz, rough}  (12 floats)
// in : per case {w_o.xyz, n.xyz, w_i.xyz, seed}               (10 floats)
// out: per case {sample.xyz, sample_pdf, pdf(w_o,n,w_i), eval.xyz (cos), eval.xyz (no cos), fresnel(w_i,n).xyz}
static Material make_mat(const float* m) {
    Material mat((MaterialType)(int)m[0]);
    mat.ior_d = m[1];
    mat.ior_m = Vector3f(m[2], m[3], m[4]);
    mat.ior_m_k = Vector3f(m[5], m[6], m[7]);
    mat.Kd = Vector3f(m[8], m[9], m[10]);
    mat.rough = m[11];
    return mat;
}
void ref_material_kat(const float* m, const float* in, int n, float* out) {
    Material mat = make_mat(m);
    for (int k = 0; k < n; ++k) {
        const float* c = in + 10 * k;
        Vector3f wo(c[0], c[1], c[2]), nn(c[3], c[4], c[5]), wi(c[6], c[7], c[8]);
        uint32_t seed; std::memcpy(&seed, &c[9], 4);
        float* o = out + 17 * k;
        ResetRandom((int)seed);
        float spdf = 0.f;
        Vector3f s = mat.sample(wo, nn, &spdf);
        o[0] = s.x; o[1] = s.y; o[2] = s.z; o[3] = spdf;
        o[4] = mat.pdf(wo, nn, wi);
        Vector3f e1 = mat.evalGivenSample(wo, wi, nn, true);
        Vector3f e2 = mat.evalGivenSample(wo, wi, nn, false);
        o[5] = e1.x; o[6] = e1.y; o[7] = e1.z;
        o[8] = e2.x; o[9] = e2.y; o[10] = e2.z;
        Vector3f f = mat.fresnel(wi, nn);
        o[11] = f.x; o[12] = f.y; o[13] = f.z;
        // cosine-weighted sample continuing the same stream
        float cpdf = 0.f;
        Vector3f cw = GetCosineWeightedSample(nn, cpdf);
        o[14] = cw.x; o[15] = cw.y; o[16] = cpdf;
    }
}

// Scalar helper KATs (SampleHelperFunctions.{hpp,cpp}, GGX.hpp).
// in : per case {a.xyz, b.xyz, f0, f1}  out: per case 16 floats, see below.
void ref_helper_kat(const float* in, int n, float* out) {
    for (int k = 0; k < n; ++k) {
        const float* c = in + 8 * k;
        Vector3f a(c[0], c[1], c[2]), b(c[3], c[4], c[5]);
        float* o = out + 16 * k;
        Vector3f r = Reflect(a, b);
        Vector3f rf = Refract(a, b, c[6]);
        Vector3f ap = AnyPerpendicular(a);
        o[0] = r.x; o[1] = r.y; o[2] = r.z;
        o[3] = rf.x; o[4] = rf.y; o[5] = rf.z;
        o[6] = ap.x; o[7] = ap.y; o[8] = ap.z;
        o[9] = Visibility(c[6], c[7], 0.3f);
        o[10] = GGXTerm(c[6], 0.3f);
        float x0 = 0, x1 = 0;
        bool ok = SolveQuadratic(c[6], c[7], c[0], x0, x1);
        o[11] = ok ? 1.f : 0.f; o[12] = ok ? x0 : 0.f; o[13] = ok ? x1 : 0.f;
        o[14] = SmoothnessToRoughenss(c[6]);
        o[15] = (float)DotProduct(a, b);
    }
}

float ref_scale(float fov) { return CalculateScale(fov); }
}
