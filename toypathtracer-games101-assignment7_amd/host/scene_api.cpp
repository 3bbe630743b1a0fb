// scene_api.cpp -- the reference's C++ caller surface on top of the C ABI
// (include/tpt_scene_api.hpp).  Host code only: scene ingest (triangle-only OBJ
// reader), the hard-coded scenes of main.cpp, and Renderer::Render driving
// libtpt's kernels.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/tpt_host.h"
#include "../../include/tpt_scene_api.hpp"

// GGX.hpp:38-40 SmoothnessToRoughenss
void Material::SetSmoothness(float smooth) {
    float r = (1.0f - smooth) * (1.0f - smooth);
    rough = 0.002f < r ? r : 0.002f;  // std::max(0.002f, r)
}

// Triangle-only OBJ ingest.  The reference reads `v` with std::stof (strtof) and
// emits one soup vertex per face corner (OBJ_Loader.hpp:533-590), then consumes
// them in groups of three (Triangle.cpp:46-65).  1-based and negative indices.
MeshTriangle::MeshTriangle(const std::string& filename, Material* m_) : Object(m_) {
    std::ifstream f(filename);
    if (!f) {
        std::fprintf(stderr, "MeshTriangle: cannot open %s\n", filename.c_str());
        return;
    }
    std::vector<float> pos;
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tok;
        if (!(ss >> tok)) continue;
        if (tok == "v") {
            std::string a, b, c;
            ss >> a >> b >> c;
            pos.push_back(std::strtof(a.c_str(), nullptr));
            pos.push_back(std::strtof(b.c_str(), nullptr));
            pos.push_back(std::strtof(c.c_str(), nullptr));
        } else if (tok == "f") {
            std::string w;
            while (ss >> w) {
                long idx = std::strtol(w.c_str(), nullptr, 10);
                long nv = (long)pos.size() / 3;
                long k = idx < 0 ? nv + idx : idx - 1;
                if (k < 0 || k >= nv) continue;
                vertices.push_back(pos[3 * k]);
                vertices.push_back(pos[3 * k + 1]);
                vertices.push_back(pos[3 * k + 2]);
            }
        }
    }
    vertices.resize(vertices.size() / 9 * 9);
    numTriangles = (uint32_t)(vertices.size() / 9);
    loaded = true;
}

void Scene::BuildBVH() {  // Scene.cpp:11-19 (emitter list; the BVH is built on upload)
    m_emissionObjects.clear();
    for (Object* o : objects)
        if (o->hasEmit()) m_emissionObjects.push_back(o);
}

void Scene::Flatten(Flat& s) const {
    s.materials.clear();
    s.objects.clear();
    s.vertices.clear();
    std::vector<const Material*> seen;
    auto mat_index = [&](const Material* m) {
        for (size_t i = 0; i < seen.size(); ++i)
            if (seen[i] == m) return (int)i;
        seen.push_back(m);
        tpt_material t;
        std::memset(&t, 0, sizeof(t));
        t.type = (int32_t)m->m_type;
        t.emission[0] = m->m_emission.x; t.emission[1] = m->m_emission.y; t.emission[2] = m->m_emission.z;
        t.ior_d = m->ior_d;
        t.ior_m[0] = m->ior_m.x; t.ior_m[1] = m->ior_m.y; t.ior_m[2] = m->ior_m.z;
        t.ior_m_k[0] = m->ior_m_k.x; t.ior_m_k[1] = m->ior_m_k.y; t.ior_m_k[2] = m->ior_m_k.z;
        t.kd[0] = m->Kd.x; t.kd[1] = m->Kd.y; t.kd[2] = m->Kd.z;
        t.rough = m->rough;
        s.materials.push_back(t);
        return (int)seen.size() - 1;
    };
    for (const Object* o : objects) {
        tpt_object t;
        std::memset(&t, 0, sizeof(t));
        t.material = mat_index(o->m);
        if (const MeshTriangle* mt = dynamic_cast<const MeshTriangle*>(o)) {
            t.kind = TPT_OBJ_MESH;
            t.first_triangle = (int32_t)(s.vertices.size() / 9);
            t.num_triangles = (int32_t)mt->numTriangles;
            s.vertices.insert(s.vertices.end(), mt->vertices.begin(), mt->vertices.end());
        } else if (const Sphere* sp = dynamic_cast<const Sphere*>(o)) {
            t.kind = TPT_OBJ_SPHERE;
            t.center[0] = sp->center.x; t.center[1] = sp->center.y; t.center[2] = sp->center.z;
            t.radius = sp->radius;
        } else {
            continue;
        }
        s.objects.push_back(t);
    }
    std::memset(&s.desc, 0, sizeof(s.desc));
    s.desc.width = width;
    s.desc.height = height;
    s.desc.eye[0] = eyePos.x; s.desc.eye[1] = eyePos.y; s.desc.eye[2] = eyePos.z;
    s.desc.background[0] = backgroundColor.x; s.desc.background[1] = backgroundColor.y; s.desc.background[2] = backgroundColor.z;
    s.desc.fov = fov;
    s.desc.num_materials = (int32_t)s.materials.size();
    s.desc.materials = s.materials.data();
    s.desc.num_objects = (int32_t)s.objects.size();
    s.desc.objects = s.objects.data();
    s.desc.num_vertices = (int64_t)s.vertices.size() / 3;
    s.desc.vertices = s.vertices.data();
}

void Renderer::Render(std::string out, const Scene& scene, int spp, int thread_count, bool bdpt) {
    Render(out, scene, spp, thread_count, bdpt, RenderOptions());
}

// Renderer::Render (Renderer.cpp:68-127): same stdout lines; the pixel/spp loop runs
// on the GPU; splats are merged into the framebuffer after the radiance
// (Renderer.cpp:98-114); "Rays" is the 64-bit sum of outBounces.
void Renderer::Render(std::string out, const Scene& scene, int spp, int thread_count, bool bdpt,
                      const RenderOptions& opt) {
    (void)thread_count;
    last_error = 0;
    if (!opt.quiet) {
        std::cout << (bdpt ? "Tracing mode: Bidirectional Ptah Tracing" : "Tracing mode: Path tracing") << std::endl;
    }
    auto start = std::chrono::system_clock::now();
    if (!opt.quiet) std::cout << "SPP: " << spp << "\n";
    Scene::Flat flat;
    scene.Flatten(flat);
    const int64_t n = (int64_t)scene.width * scene.height * 3;
    framebuffer.assign(n, 0.0f);
    std::vector<float> splat(bdpt ? n : 0, 0.0f);
    tpt_render_params p;
    std::memset(&p, 0, sizeof(p));
    p.spp = spp;
    p.mode = bdpt ? TPT_MODE_BDPT : opt.pt_indirect ? TPT_MODE_PT_INDIRECT : TPT_MODE_PT;
    p.pixel_begin = 0;
    p.pixel_stride = 1;
    int rc = TPT_OK;
    std::string err;
    if (opt.gpus > 1) {
        // the reference's j std::async workers (Renderer.cpp:86-91) become opt.gpus
        // devices; its thread-order splat merge (:98-114) one RCCL reduce
        std::vector<int> devs;
        for (int g = 0; g < opt.gpus; ++g) devs.push_back(opt.device + g);
        tpt_multi* m = nullptr;
        rc = tpt_multi_create(opt.gpus, devs.data(), &m);
        if (rc) err = "tpt_multi_create failed (" + std::to_string(rc) + ")";
        if (!rc) rc = tpt_multi_upload_scene(m, &flat.desc);
        if (!rc) rc = tpt_render_multi(m, &p, framebuffer.data(), bdpt ? splat.data() : nullptr, &stats);
        if (rc && m) err = tpt_multi_last_error(m);
        tpt_multi_destroy(m);
    } else {
        tpt_ctx* ctx = nullptr;
        rc = tpt_create(opt.device, &ctx);
        if (rc) err = "tpt_create failed (" + std::to_string(rc) + ")";
        if (!rc) rc = tpt_upload_scene(ctx, &flat.desc);
        if (!rc) rc = tpt_render(ctx, &p, framebuffer.data(), bdpt ? splat.data() : nullptr, &stats);
        if (rc && ctx) err = tpt_last_error(ctx);
        tpt_destroy(ctx);
    }
    if (rc) {
        std::cerr << "render failed: " << err << "\n";
        last_error = rc;
        return;
    }
    if (bdpt) {
        if (!opt.quiet) std::cout << "Tracing finished, merge emission buffer\n";
        for (int64_t j = 0; j < n; ++j) framebuffer[j] += splat[j];
    }
    auto stop = std::chrono::system_clock::now();
    if (!opt.quiet) {
        std::cout << std::endl << "Render complete: \n";
        auto d = stop - start;
        std::cout << "Time taken: " << std::chrono::duration_cast<std::chrono::hours>(d).count() << " hours\n";
        std::cout << "          : " << std::chrono::duration_cast<std::chrono::minutes>(d).count() << " minutes\n";
        std::cout << "          : " << std::chrono::duration_cast<std::chrono::seconds>(d).count() << " seconds\n";
        std::cout << "Rays: " << stats.bounces << std::endl;
        double ms = (double)std::chrono::duration_cast<std::chrono::milliseconds>(d).count();
        std::cout << "Rays Per Second: " << (ms > 0 ? (double)stats.bounces / 1e3 / ms : 0.0) << "MRays" << std::endl;
        std::cout << "Samples Per Second: " << (double)stats.samples / 1e3 / std::max(stats.kernel_ms, 1e-9)
                  << " MSamples (kernel)" << std::endl;
    }
    if (!out.empty() && out != "/dev/null") tpt_save_image(framebuffer.data(), scene.width, scene.height, out.c_str());
    if (!opt.float_dump.empty()) {
        FILE* f = std::fopen(opt.float_dump.c_str(), "wb");
        if (f) {
            std::fwrite(framebuffer.data(), sizeof(float), framebuffer.size(), f);
            std::fclose(f);
        }
    }
}

// main.cpp:49-103 (+ SURVEY §8(d) variants).  Materials and Add order as in the
// reference; the smooth_dielectric preset declares white's smoothness = 0.7.  Edge
// cases: "multi_light" (+ light2.obj, light3.obj as emitters), "emissive_sphere" (a
// glowing Sphere as m_emissionObjects[0]), "background" (Scene.hpp:23's default
// backgroundColor kept).
bool BuildPresetScene(const std::string& dir, const std::string& p, Scene& scene) {
    static std::vector<Material*> keep_m;
    static std::vector<Object*> keep_o;
    scene.eyePos = Vector3f(278, 278, -800);
    // main.cpp:51 sets the background to 0; "background" keeps Scene.hpp:23's default
    scene.backgroundColor = p == "background" ? Vector3f(0.235294f, 0.67451f, 0.843137f) : Vector3f(0.0f);
    auto M = [&](Material* m) { keep_m.push_back(m); return m; };
    Material* red = M(new Material(Dieletric, Vector3f(0.0f)));
    red->Kd = Vector3f(0.63f, 0.065f, 0.05f);
    Material* green = M(new Material(Dieletric, Vector3f(0.0f)));
    green->Kd = Vector3f(0.14f, 0.45f, 0.091f);
    Material* white = M(new Material(Dieletric, Vector3f(0.0f)));
    white->Kd = Vector3f(0.725f, 0.71f, 0.68f);
    white->SetSmoothness(p == "smooth_dielectric" ? 0.7f : .1f);
    Material* light = M(new Material(Dieletric, (8.0f * Vector3f(0.747f + 0.058f, 0.747f + 0.258f, 0.747f) +
                                               15.6f * Vector3f(0.740f + 0.287f, 0.740f + 0.160f, 0.740f) +
                                               18.4f * Vector3f(0.737f + 0.642f, 0.737f + 0.159f, 0.737f))));
    light->Kd = Vector3f(0.65f);
    Material* silver = M(new Material(Metal));
    silver->ior_m = Vector3f(0.041000f, 0.53285f, 0.049317f);
    silver->ior_m_k = Vector3f(4.8025f, 3.4101f, 2.8545f);
    silver->SetSmoothness(1.f);
    Material* glass = M(new Material(Transparent));
    glass->ior_d = 1.5f;
    glass->SetSmoothness(.9f);
    Material* lightball = M(new Material(Dieletric, Vector3f(3.0f, 2.4f, 1.5f)));
    lightball->Kd = Vector3f(0.65f);
    Material* boxes = nullptr;
    if (p == "silver") boxes = silver;
    else if (p == "standard" || p == "refractive_ball" || p == "occlusion" || p == "smooth_dielectric" || p == "bunny" ||
             p == "multi_light" || p == "emissive_sphere" || p == "background")
        boxes = white;
    else return false;
    bool ok = true;
    auto mesh = [&](const char* f, Material* m) {
        MeshTriangle* t = new MeshTriangle(dir + "/" + f, m);
        keep_o.push_back(t);
        ok = ok && t->loaded;
        scene.Add(t);
    };
    if (p == "bunny") {
        mesh("floor.obj", white);
        mesh("left.obj", red);
        mesh("right.obj", green);
        mesh("light.obj", light);
        mesh("bunny_cornell.obj", white);
    } else {
        mesh("floor.obj", boxes);
        mesh("shortbox.obj", boxes);
        mesh("tallbox.obj", boxes);
        mesh("left.obj", red);
        mesh("right.obj", green);
        if (p == "emissive_sphere") {  // the glowing ball is m_emissionObjects[0] (BDPT.cpp:287)
            Sphere* s = new Sphere(Vector3f(420.0f, 60.0f, 150.0f), 60.0f, lightball);
            keep_o.push_back(s);
            scene.Add(s);
        }
        mesh("light.obj", light);
        if (p == "multi_light") {
            mesh("light2.obj", light);
            mesh("light3.obj", light);
        }
        if (p == "refractive_ball") {
            Sphere* s = new Sphere(Vector3f(278.0f, 278.0f, 200.0f), 50.0f, glass);
            keep_o.push_back(s);
            scene.Add(s);
        }
        if (p == "occlusion") mesh("lightocculuder.obj", white);
    }
    scene.BuildBVH();
    return ok;
}

struct tpt_preset {
    Scene scene{784, 784};
    Scene::Flat flat;
};

extern "C" {
int tpt_preset_load(const char* models_dir, const char* name, int32_t w, int32_t h, tpt_preset** out) {
    if (!models_dir || !name || !out || w <= 0 || h <= 0) return TPT_E_INVALID;
    tpt_preset* p = new tpt_preset();
    p->scene.width = w;
    p->scene.height = h;
    if (!BuildPresetScene(models_dir, name, p->scene)) {
        delete p;
        *out = nullptr;
        return TPT_E_INVALID;
    }
    p->scene.Flatten(p->flat);
    *out = p;
    return TPT_OK;
}
const tpt_scene_desc* tpt_preset_desc(const tpt_preset* p) { return p ? &p->flat.desc : nullptr; }
void tpt_preset_free(tpt_preset* p) { delete p; }
}
