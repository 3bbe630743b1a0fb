// tpt_scene.h -- HBM layout of a flattened scene (shared by the host builder and
// the gfx950 kernels).
//
// The reference keeps a two-level BVH of heap objects (Scene::bvh over Object*,
// one BVHAccel per MeshTriangle: Scene.cpp:11-19, Triangle.cpp:74, BVH.hpp:89-104).
// Here both levels live in ONE node array:
//   nodes[0 .. ntop)          scene-level nodes, reference allocation order
//   nodes[ntop .. nnodes)     each mesh's nodes, reference allocation order
// A scene-level leaf that holds a mesh is replaced by a copy of that mesh's root
// node.  The reference tests the leaf box (MeshTriangle::bounding_box) and then the
// mesh root box (union of the triangle boxes); both are the componentwise min/max
// of the same vertices, i.e. the same box, so one test is exact.  Traversal order
// (right child popped first, BVH.cpp:129-132) and closest-hit tie breaking are
// therefore unchanged (tests/test_gpu_parity.py checks hit ordinals).
#pragma once
#include <stdint.h>

namespace tpt {

// 32 B.  a >= 0: interior (a = left, b = right).  a < 0: leaf of primitive -1-a
// (triangles [0, ntri), spheres [ntri, ntri+nsph)).  a == kEmptyLeaf: empty mesh.
struct alignas(16) DNode {
    float bmin[3];
    int32_t a;
    float bmax[3];
    int32_t b;
};
static const int32_t kEmptyLeaf = (int32_t)0x80000000;

// Threaded copy of `nodes` (same boxes, same 32-B layout, DNode with a = first,
// b = next) for stackless per-lane walks in the reference's visit order (BVH.cpp:
// 121-137 pushes left then right, so the right child is visited first):
//   a >= 0: interior, a = the right child (kSpliceBit set: the node is a scene leaf
//           replaced by its mesh's root -- entering the mesh, remember b);
//   a <  0: leaf (-1 - prim, or kEmptyLeaf);
//   b     : the node visited after this subtree (or after a box miss); kWalkEnd
//           ends the walk, kMeshExit leaves a mesh subtree for the remembered node.
// A walk therefore fetches one node per step and keeps no stack.
static const int32_t kSpliceBit = 0x40000000;
static const int32_t kWalkEnd = -1;
static const int32_t kMeshExit = -2;

// Flat queries (tpt_device.h) list at most this many primitive leaves.  A scene
// with more keeps its largest meshes out of the list as walk groups
// (tpt_scene_build.cpp: split_walk_groups).
static const int kFlatMaxLeaves = 64;

// Wide walk nodes for walk groups (tpt_device.h walk4).  A QNode4 stands for a
// binary interior node P of a mesh BVH whose box the walk has already passed; its
// kWalkW entries are P's descendants kWalkLevels binary levels down (or a shallower
// leaf itself) in the reference's visit order (right child first, BVH.cpp:129-132),
// each with its own box.  The binary boxes in between are not tested: for a ray with
// finite inv a box passing implies its enclosing boxes pass (slab monotonicity,
// tpt_device.h), so the leaves reached -- and their order -- are the reference's.
// Layout: the box coordinates SoA over the entries, then the entry codes.
#ifndef TPT_WALK_LEVELS
#define TPT_WALK_LEVELS 2  // binary levels per wide node: 2 -> 4 entries (128 B), 3 -> 8 (256 B)
#endif
static const int kWalkLevels = TPT_WALK_LEVELS;
static const int kWalkW = 1 << kWalkLevels;
struct alignas(16) QNode4 {
    float bmin[3][kWalkW];  // bmin[axis][entry]
    float bmax[3][kWalkW];
    int32_t e[kWalkW];      // >= 0: QNode index; < 0: -1 - primitive (a leaf); kQNone: unused slot
    int32_t pad[kWalkW];
};
static_assert(sizeof(QNode4) == 32 * kWalkW, "QNode4: 16-B rows");
static const int32_t kQNone = (int32_t)0x7fffffff;
// Per-lane LDS stack of the wide walk (16-bit entries): a walk group uses its wide
// tree only when its depth d satisfies (kWalkW - 1) d + 1 <= kWalkStack.
static const int kWalkStack = kWalkLevels == 2 ? 24 : 36;

// 48 B, read as three float4: (v0, n.x) (e1, n.y) (e2, n.z) -- Triangle.hpp:46-50
struct alignas(16) DTri {
    float v0[3];
    float nx;
    float e1[3];
    float ny;
    float e2[3];
    float nz;
};
// 32 B, only touched on light sampling / pdf paths: v1, v2 (Triangle::Sample uses
// the original vertices, Triangle.hpp:33), area (Triangle::pdf), material.
struct alignas(16) DTriX {
    float v1[3];
    float area;
    float v2[3];
    int32_t mat;
};
struct alignas(16) DSphere {  // Sphere.hpp:13-15
    float c[3];
    float r;
    float r2;
    float area;
    int32_t mat;
    int32_t pad;
};
struct DMat {  // Material.hpp:19-25
    int32_t type;
    float em[3];
    float ior_d;
    float ior_m[3];
    float ior_m_k[3];
    float kd[3];
    float rough;
    int32_t has_em;  // Material::hasEmission (Material.hpp:36-39)
    int32_t pad[2];
};
struct alignas(16) DObj {
    int32_t kind;         // TPT_OBJ_MESH / TPT_OBJ_SPHERE
    int32_t mat;
    int32_t root;         // mesh BVH root in nodes[] (-1 if empty)
    int32_t sphere_prim;  // global primitive id of the sphere
    float pdf;            // Object::pdf(): MeshTriangle 1/root-area (Triangle.hpp:58-60), Sphere 1/area
    float root_area;
    int32_t pad[2];
};

// Kernel argument: device pointers + constants.
struct DScene {
    const DNode* nodes;
    const float* node_area;  // BVHBuildNode::area (BVH.hpp:94), per node
    const DTri* tris;
    const DTriX* trix;
    const DSphere* sph;
    const DMat* mats;
    const DObj* objs;
    const int32_t* emitters;  // Scene::m_emissionObjects (object ids)
    const DNode* tnodes;      // threaded binary tree (stackless walks), same indices as nodes
    const DNode* leaves;      // primitive leaves in the reference's DFS order (flat queries)
    const DNode* groups;      // leaves grouped per object: box, a = first leaf, b = count;
                              // b < 0: walk group, a = first node of the mesh walk in tnodes,
                              // b <= -2: its 4-wide tree's root is qnodes[-2 - b]
    const QNode4* qnodes;     // 4-wide trees of the walk groups
    const DTri* ftris;        // triangle of flat leaf j is ftris[leaves[j].b]
    const DTri* gtris;        // `tris` in HBM, never re-pointed to LDS (the wide walks' global loads)
    const uint16_t* grank;    // walk-group triangles: rank in the reference's DFS visit order (stealing walks' ties)
    int32_t nleaf;
    int32_t ngroup;
    int32_t flat;             // flat (all-leaves) queries: kFlatShadow | kFlatHit bits, 0 = tree walks
    int32_t n_emitters;
    int32_t light_draws;  // XorShift draws of one DirectLightSampler::sample pass over all emitters
    int32_t ntri;
    int32_t nsph;
    int32_t nnodes;
    int32_t nobj;
    int32_t width;
    int32_t height;
    float scale;  // CalculateScale(fov) (SceneRenderingHelper.cpp:12-14), host-computed
    float lbox[6];     // the emitters' bounding box (min xyz, max xyz): PT shadow-cone masks
    float cone_delta;  // ... and their margin (HostScene::cone_delta)
    float eye[3];
    float bg[3];
    int32_t nmats;
    int32_t lds_bytes;  // bytes staged in LDS per workgroup (0 = read from HBM/L2)
    int32_t lds_full;   // 1: nodes + triangles + flat arrays staged; 0: only the flat arrays
    int32_t big;        // the flat list has walk groups (the kernels of small scenes fold it to 0)
    void* qs;           // device only: per-wave LDS scratch of the compacted flat queries (null: off)
    uint16_t* ws;       // device only: per-lane LDS stacks of the 4-wide walks, [slot][lane] (null: binary walks)
};

}  // namespace tpt
