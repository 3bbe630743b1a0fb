// tpt_scene_api.hpp -- the reference's C++ caller surface, re-declared on top of the
// C ABI (tpt.h) so a program written against the reference (main.cpp:36-152)
// compiles unchanged and renders on the GPU.
//
//   reference                                       here
//   Vector3f            Vector.hpp:13-83            Vector3f (data + the operators main.cpp uses)
//   MaterialType/Material Material.hpp:11-44        same names, fields, SetSmoothness
//   Object / MeshTriangle / Sphere                  Object.hpp, Triangle.hpp:53, Sphere.hpp
//   Scene               Scene.hpp:15-39             width/height/fov/eyePos/backgroundColor,
//                                                    Add, BuildBVH, objects, m_emissionObjects
//   Renderer::Render    Renderer.hpp:11             same signature; runs libtpt on the GPU
//
// Geometry stays on the host until Renderer::Render flattens the Scene into a
// tpt_scene_desc; the BVH itself is built inside tpt_upload_scene.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "tpt.h"

class Vector3f {
public:
    float x, y, z;
    Vector3f() : x(0), y(0), z(0) {}
    Vector3f(float xx) : x(xx), y(xx), z(xx) {}
    Vector3f(float xx, float yy, float zz) : x(xx), y(yy), z(zz) {}
    Vector3f operator*(const float& r) const { return Vector3f(x * r, y * r, z * r); }
    Vector3f operator/(const float& r) const { return Vector3f(x / r, y / r, z / r); }
    Vector3f operator+(const Vector3f& v) const { return Vector3f(x + v.x, y + v.y, z + v.z); }
    Vector3f operator-(const Vector3f& v) const { return Vector3f(x - v.x, y - v.y, z - v.z); }
    Vector3f operator*(const Vector3f& v) const { return Vector3f(x * v.x, y * v.y, z * v.z); }
    Vector3f operator-() const { return Vector3f(-x, -y, -z); }
    Vector3f& operator+=(const Vector3f& v) { x += v.x; y += v.y; z += v.z; return *this; }
    friend Vector3f operator*(const float& r, const Vector3f& v) { return Vector3f(v.x * r, v.y * r, v.z * r); }
};

enum MaterialType { Dieletric, Metal, Transparent };

class Material {
public:
    MaterialType m_type;
    Vector3f m_emission;
    float ior_d = 1.5f;
    Vector3f ior_m = Vector3f(0.13100f, 0.55758f, 1.4561f), ior_m_k = Vector3f(4.0624f, 2.2039f, 1.9541f);
    Vector3f Kd;
    float rough = 0.2f;
    Material(MaterialType t = Dieletric, Vector3f e = Vector3f(0, 0, 0)) : m_type(t), m_emission(e), Kd(0.5f, 0.5f, 0.5f) {}
    void SetSmoothness(float smooth);  // GGX.hpp:38-40 SmoothnessToRoughenss
    MaterialType getType() const { return m_type; }
    Vector3f GetEmission() const { return m_emission; }
    bool hasEmission() const { return m_emission.x > 0.0f || m_emission.y > 0.0f || m_emission.z > 0.0f; }
};

class Object {
public:
    explicit Object(Material* m_) : m(m_) {}
    virtual ~Object() {}
    bool hasEmit() const { return m->hasEmission(); }
    Material* m;
};

// Triangle soup from a triangle-only OBJ (Triangle.cpp:32-75 via OBJ_Loader.hpp).
class MeshTriangle : public Object {
public:
    MeshTriangle(const std::string& filename, Material* m_ = new Material());
    std::vector<float> vertices;  // 9 floats per triangle, file face order
    uint32_t numTriangles = 0;
    bool loaded = false;
};

class Sphere : public Object {
public:
    Vector3f center;
    float radius, radius2;
    Sphere(const Vector3f& c, const float& r, Material* mt = new Material())
        : Object(mt), center(c), radius(r), radius2(r * r) {}
};

class Scene {
public:
    int width = 1280;
    int height = 960;
    double fov = 40;
    Vector3f eyePos;
    Vector3f backgroundColor = Vector3f(0.235294f, 0.67451f, 0.843137f);
    std::vector<Object*> objects;
    std::vector<Object*> m_emissionObjects;
    Scene(int w, int h) : width(w), height(h) {}
    Scene& Add(Object* object) { objects.push_back(object); return *this; }
    const std::vector<Object*>& GetObjects() const { return objects; }
    void BuildBVH();  // collects emitters; the BVH is built by tpt_upload_scene

    // Flatten into the C ABI's scene description (arrays owned by `storage`).
    struct Flat {
        std::vector<tpt_material> materials;
        std::vector<tpt_object> objects;
        std::vector<float> vertices;
        tpt_scene_desc desc;
    };
    void Flatten(Flat& storage) const;
};

struct RenderOptions {
    int device = 0;              // first HIP device
    int gpus = 1;                // >1: devices device .. device+gpus-1, pixel-sharded, one RCCL reduce (tpt_render_multi)
    std::string float_dump;      // optional raw fp32 W*H*3 dump (parity artefact)
    bool quiet = false;
    bool pt_indirect = false;    // PathTrace with the indirect bounce (TPT_MODE_PT_INDIRECT); off by default
};

class Renderer {
public:
    // Renderer.hpp:11.  thread_count is accepted for interface parity; the GPU
    // path ignores it (one lane per pixel stream).
    void Render(std::string outputFileName, const Scene& scene, int spp, int thread_count, bool bdpt);
    void Render(std::string outputFileName, const Scene& scene, int spp, int thread_count, bool bdpt,
                const RenderOptions& opt);
    std::vector<float> framebuffer;  // last render, W*H*3 (radiance + splats)
    tpt_stats stats{};
    int last_error = 0;
};

// The reference's hard-coded scenes (main.cpp:49-103) + SURVEY §8(d) variants:
// "silver" (HEAD as-is), "standard", "refractive_ball", "occlusion",
// "smooth_dielectric", "bunny".  Returns false on an unknown name / missing model.
bool BuildPresetScene(const std::string& models_dir, const std::string& name, Scene& scene);

// Film output (SceneRenderingHelper.cpp:57-70): clamp to [0,1], pow(x, 0.6), x255.
// Writes .jpg (baseline JPEG, quality 100), .ppm, or .pfm by extension.
bool SaveFloatImage(const std::vector<float>& rgb, int width, int height, const std::string& path);
