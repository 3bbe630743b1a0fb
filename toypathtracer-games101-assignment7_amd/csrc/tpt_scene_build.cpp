// tpt_scene_build.cpp -- host side of tpt_upload_scene: build the reference's
// two-level BVH on the CPU and flatten it into the HBM layout of tpt_scene.h.
//
// Must reproduce the reference's trees node for node, because traversal order
// decides closest-hit ties and the per-node area sums drive light sampling:
//   Triangle ctor (e1, e2, normal, area)          Triangle.hpp:18-25
//   MeshTriangle bounding box / area sum          Triangle.cpp:46-73
//   BVHAccel::recursiveBuild (median split on the centroid axis of max extent,
//   std::sort tie order, size-2 special case,
//   pre-order allocation)                         BVH.cpp:30-99, :161-169
//   Bounds3 ctor / Union / Centroid / maxExtent   Bounds3.hpp:11-48, :117-131
//   Sphere area / bounds                          Sphere.hpp:16, Sphere.cpp:43-46
//   Scene::BuildBVH emitter list                  Scene.cpp:11-19
// The comparator sorts object indices on the same float keys in the same initial
// order with the same libstdc++ std::sort, so the permutation is identical.
// Compiled with -ffp-contract=off (the reference build has no FMA contraction).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../include/tpt.h"
#include "tpt_devmath.h"
#include "tpt_scene.h"
#include "tpt_scene_build.h"

namespace tpt {
namespace {

struct Box {
    V3 mn, mx;
};
Box empty_box() {  // Bounds3() -- Bounds3.hpp:14-20
    Box b;
    b.mn = v3s(std::numeric_limits<float>::max());
    b.mx = v3s(std::numeric_limits<float>::lowest());
    return b;
}
V3 vmin(V3 a, V3 b) { return v3(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z)); }
V3 vmax(V3 a, V3 b) { return v3(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z)); }
Box join(const Box& a, const Box& b) { return Box{vmin(a.mn, b.mn), vmax(a.mx, b.mx)}; }
Box join(const Box& a, V3 p) { return Box{vmin(a.mn, p), vmax(a.mx, p)}; }
Box box2(V3 p, V3 q) {
    return Box{v3(std::fmin(p.x, q.x), std::fmin(p.y, q.y), std::fmin(p.z, q.z)),
               v3(std::fmax(p.x, q.x), std::fmax(p.y, q.y), std::fmax(p.z, q.z))};
}
V3 centroid(const Box& b) { return mul(b.mn, 0.5f) + mul(b.mx, 0.5f); }
float axis(V3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
int max_extent(const Box& b) {
    V3 d = b.mx - b.mn;
    if (d.x > d.y && d.x > d.z) return 0;
    if (d.y > d.z) return 1;
    return 2;
}

struct BuildNode {
    Box box;
    int left = -1, right = -1;
    int item = -1;
    float area = 0.0f;
};

// BVHAccel::recursiveBuild over items with precomputed boxes / areas.
struct Builder {
    const std::vector<Box>& box;
    const std::vector<float>& area;
    std::vector<BuildNode> nodes;
    int depth = 0;
    Builder(const std::vector<Box>& b, const std::vector<float>& a) : box(b), area(a) {}

    int build(std::vector<int> items, int level) {
        depth = std::max(depth, level);
        int idx = (int)nodes.size();
        nodes.emplace_back();
        if (items.size() == 1) {
            nodes[idx].box = box[items[0]];
            nodes[idx].item = items[0];
            nodes[idx].area = area[items[0]];
            return idx;
        }
        if (items.size() == 2) {
            int l = build({items[0]}, level + 1);
            int r = build({items[1]}, level + 1);
            nodes[idx].left = l;
            nodes[idx].right = r;
            nodes[idx].box = join(nodes[l].box, nodes[r].box);
            nodes[idx].area = nodes[l].area + nodes[r].area;
            return idx;
        }
        Box cb = empty_box();
        for (int it : items) cb = join(cb, centroid(box[it]));
        int dim = max_extent(cb);
        std::sort(items.begin(), items.end(),
                  [&](int a, int b) { return axis(centroid(box[a]), dim) < axis(centroid(box[b]), dim); });
        size_t mid = items.size() / 2;
        int l = build(std::vector<int>(items.begin(), items.begin() + mid), level + 1);
        int r = build(std::vector<int>(items.begin() + mid, items.end()), level + 1);
        nodes[idx].left = l;
        nodes[idx].right = r;
        nodes[idx].box = join(nodes[l].box, nodes[r].box);
        nodes[idx].area = nodes[l].area + nodes[r].area;
        return idx;
    }
};

DNode to_dnode(const Box& b, int a, int c) {
    DNode n;
    n.bmin[0] = b.mn.x; n.bmin[1] = b.mn.y; n.bmin[2] = b.mn.z;
    n.bmax[0] = b.mx.x; n.bmax[1] = b.mx.y; n.bmax[2] = b.mx.z;
    n.a = a;
    n.b = c;
    return n;
}

}  // namespace

// Threading (tpt_scene.h, tnodes): node n's miss link is the node the reference's
// DFS pops after n's subtree.  Scene-level nodes [0, ntop) are threaded as one
// tree whose spliced mesh leaves keep their next link and point into the mesh;
// every mesh subtree is threaded on its own and ends in kMeshExit.
static void thread_tree(HostScene& hs, int n, int after, int ntop, bool scene) {
    const DNode& src = hs.nodes[n];
    DNode& t = hs.tnodes[n];
    t = src;
    t.b = after;
    if (src.a < 0) return;  // leaf: a keeps the leaf code
    const bool spliced = scene && src.a >= ntop;  // a scene leaf replaced by its mesh root
    t.a = spliced ? (src.b | kSpliceBit) : src.b;  // right child first (BVH.cpp:129-132)
    if (spliced) return;                            // the mesh is threaded by itself
    thread_tree(hs, src.b, src.a, ntop, scene);    // after the right subtree: the left child
    thread_tree(hs, src.a, after, ntop, scene);
}

// The wide tree below binary node p (tpt_scene.h QNode4): its entries are p's
// descendants kWalkLevels binary levels down -- or a shallower leaf itself -- in the
// reference's visit order, right child first (BVH.cpp:129-132).  Returns the QNode
// index; `depth` receives the tree's depth in QNodes.
static void wide_entries(const HostScene& hs, int x, int levels, std::vector<int>& ent) {
    const DNode& X = hs.nodes[x];
    if (X.a < 0) {
        if (X.a != kEmptyLeaf) ent.push_back(x);
    } else if (levels == 0) {
        ent.push_back(x);
    } else {
        wide_entries(hs, X.b, levels - 1, ent);
        wide_entries(hs, X.a, levels - 1, ent);
    }
}
static int build_qtree(HostScene& hs, int p, int& depth) {
    const int q = (int)hs.qnodes.size();
    hs.qnodes.push_back(QNode4{});
    std::vector<int> ent;  // binary node indices, visit order
    const DNode& P = hs.nodes[p];
    wide_entries(hs, P.b, kWalkLevels - 1, ent);
    wide_entries(hs, P.a, kWalkLevels - 1, ent);
    int dmax = 0;
    QNode4 Q;
    std::memset(&Q, 0, sizeof(Q));
    for (int j = 0; j < kWalkW; ++j) Q.e[j] = kQNone;
    for (size_t j = 0; j < ent.size(); ++j) {
        const DNode& E = hs.nodes[ent[j]];
        for (int k = 0; k < 3; ++k) { Q.bmin[k][j] = E.bmin[k]; Q.bmax[k][j] = E.bmax[k]; }
        if (E.a < 0) {
            Q.e[j] = E.a;  // -1 - prim
            // the walk reaches leaves in entry order, subtree by subtree: this is the
            // reference's DFS rank of the triangle within the group (BVH.cpp:129-132)
            const size_t prim = (size_t)(-1 - E.a);
            if (hs.grank.size() < hs.tris.size()) hs.grank.resize(hs.tris.size(), 0);
            if (prim < hs.grank.size()) hs.grank[prim] = (uint16_t)hs.grank_next++;
        } else {
            int d = 0;
            Q.e[j] = build_qtree(hs, ent[j], d);
            dmax = std::max(dmax, d);
        }
    }
    hs.qnodes[q] = Q;
    depth = dmax + 1;
    return q;
}

// Flat queries test every listed leaf; past kFlatMaxLeaves the largest meshes leave
// the list and become walk groups {box, a = gwalk, b = -1}: a lane whose ray passes
// the group box (the mesh root's box) walks the mesh subtree on the threaded tree,
// at the group's place in the DFS order, so the visit order is still the reference's.
static void split_walk_groups(HostScene& hs, const std::vector<int>& gwalk, const std::vector<int>& gnode) {
    int total = (int)hs.leaves.size();
    if (total <= kFlatMaxLeaves) return;
    std::vector<int> order(hs.groups.size());
    for (size_t g = 0; g < order.size(); ++g) order[g] = (int)g;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return hs.groups[x].b > hs.groups[y].b; });
    std::vector<char> walk(hs.groups.size(), 0);
    for (int g : order) {
        if (total <= kFlatMaxLeaves) break;
        if (gwalk[g] < 0) continue;
        walk[g] = 1;
        total -= hs.groups[g].b;
    }
    std::vector<DNode> leaves, groups;
    for (size_t g = 0; g < hs.groups.size(); ++g) {
        DNode G = hs.groups[g];
        if (walk[g]) {
            G.a = gwalk[g];
            G.b = -1;
            // wide tree of the mesh below the spliced root; kept when its walk stack
            // fits (kWalkW - 1 pending entries per level + the current one) and its
            // indices fit the stack's 16-bit entries
            const size_t q0 = hs.qnodes.size();
            int depth = 0;
            hs.grank_next = 0;
            const int qr = build_qtree(hs, gnode[g], depth);
            const bool fits = (kWalkW - 1) * depth + 1 <= kWalkStack && hs.qnodes.size() <= 32767 &&
                              hs.tris.size() <= 32767;
            if (fits) G.b = -2 - qr;
            else hs.qnodes.resize(q0);
        } else {
            const int a0 = G.a;
            G.a = (int)leaves.size();
            leaves.insert(leaves.end(), hs.leaves.begin() + a0, hs.leaves.begin() + a0 + G.b);
        }
        groups.push_back(G);
    }
    hs.leaves.swap(leaves);
    hs.groups.swap(groups);
}

static void build_threads(HostScene& hs, int ntop, const std::vector<int>& mesh_root) {
    hs.tnodes.assign(hs.nodes.size(), DNode{});
    hs.leaves.clear();
    if (hs.nodes.empty()) return;
    thread_tree(hs, 0, kWalkEnd, ntop, true);
    for (int r : mesh_root)
        if (r >= 0) thread_tree(hs, r, kMeshExit, ntop, false);
    // Leaves in the order a walk whose every box test passes visits them: the
    // reference's DFS order (BVH.cpp:121-137) restricted to leaves.  Any subset of
    // leaves a real ray reaches is visited in this relative order.
    // Leaves are grouped by object: a mesh's leaves are contiguous in that order and
    // its group box is the scene-level leaf box (= the mesh root box); a sphere is a
    // group of one.  groups[g] = {box, a = first leaf, b = leaf count}.
    hs.groups.clear();
    std::vector<int> gwalk;  // per group: first node of its mesh walk (the root's right child), -1 if none
    std::vector<int> gnode;  // per group: the scene node (the spliced mesh root), -1 if none
    int cur = 0, cont = kWalkEnd;
    while (cur >= 0) {
        const DNode& n = hs.tnodes[cur];
        int nxt = n.b;
        if (n.a >= 0) {
            if (n.a & kSpliceBit) {
                cont = n.b;
                nxt = n.a & ~kSpliceBit;
                DNode g = n;
                g.a = (int)hs.leaves.size();
                g.b = 0;
                hs.groups.push_back(g);
                gwalk.push_back(nxt);
                gnode.push_back(cur);
            } else {
                nxt = n.a;
            }
        } else if (n.a != kEmptyLeaf) {
            DNode l = n;
            l.b = 0;
            if (cur < ntop) {  // a leaf of the scene tree itself (sphere)
                DNode g = n;
                g.a = (int)hs.leaves.size();
                g.b = 0;
                hs.groups.push_back(g);
                gwalk.push_back(-1);
                gnode.push_back(-1);
            }
            hs.leaves.push_back(l);
            hs.groups.back().b++;
        }
        if (nxt == kMeshExit) {
            cur = cont;
            cont = kWalkEnd;
        } else {
            cur = nxt;
        }
    }
    split_walk_groups(hs, gwalk, gnode);
}

int build_host_scene(const tpt_scene_desc* d, HostScene& hs, std::string& err) {
    hs = HostScene();
    if (!d || d->width <= 0 || d->height <= 0 || d->num_materials < 0 || d->num_objects < 0) {
        err = "invalid scene description";
        return TPT_E_INVALID;
    }
    // The reference's camera and splat code assume width >= height:
    //  * the aspect ratio is an integer division, `float imageAspectRatio = width /
    //    height` (SceneRenderingHelper.cpp:17, :25), which is 0 when width < height,
    //    so RayToUV divides by zero (:26) and DrawToImage converts inf to int (:35-36);
    //  * DrawToImage writes `buffer[ix + height * iy]` (SceneRenderingHelper.cpp:50),
    //    which for height > width runs past the W*H splat buffer -- in the reference a
    //    heap overflow, on the GPU an out-of-bounds float atomic into HBM.
    // Such frames are refused instead of reproducing undefined behaviour.
    if (d->height > d->width) {
        err = "height > width is not supported: the reference's integer aspect ratio (SceneRenderingHelper.cpp:17) "
              "is 0 and its splat index ix + height*iy (SceneRenderingHelper.cpp:50) overruns the frame";
        return TPT_E_UNSUPPORTED;
    }
    for (int i = 0; i < d->num_materials; ++i) {
        const tpt_material& m = d->materials[i];
        if (m.type < 0 || m.type > 2) { err = "invalid material type"; return TPT_E_INVALID; }
        DMat dm;
        std::memset(&dm, 0, sizeof(dm));
        dm.type = m.type;
        for (int k = 0; k < 3; ++k) {
            dm.em[k] = m.emission[k];
            dm.ior_m[k] = m.ior_m[k];
            dm.ior_m_k[k] = m.ior_m_k[k];
            dm.kd[k] = m.kd[k];
        }
        dm.ior_d = m.ior_d;
        dm.rough = m.rough;
        dm.has_em = (m.emission[0] > 0.0f || m.emission[1] > 0.0f || m.emission[2] > 0.0f) ? 1 : 0;
        hs.mats.push_back(dm);
    }

    // ---- primitives: all triangles (object order, soup order), then spheres
    struct MeshRange { int first, count; };
    std::vector<MeshRange> mesh_tris(d->num_objects, MeshRange{0, 0});
    std::vector<float> mesh_area(d->num_objects, 0.0f);
    std::vector<Box> mesh_box(d->num_objects, empty_box());
    for (int o = 0; o < d->num_objects; ++o) {
        const tpt_object& ob = d->objects[o];
        if (ob.material < 0 || ob.material >= d->num_materials) { err = "object material out of range"; return TPT_E_INVALID; }
        if (ob.kind != TPT_OBJ_MESH) continue;
        if (ob.first_triangle < 0 || ob.num_triangles < 0 ||
            3 * ((int64_t)ob.first_triangle + ob.num_triangles) > d->num_vertices) {
            err = "mesh triangle range out of bounds";
            return TPT_E_INVALID;
        }
        mesh_tris[o].first = (int)hs.tris.size();
        mesh_tris[o].count = ob.num_triangles;
        V3 mn = v3s(std::numeric_limits<float>::max()), mx = v3s(-std::numeric_limits<float>::max());
        for (int t = 0; t < ob.num_triangles; ++t) {
            V3 v[3];
            for (int j = 0; j < 3; ++j) {
                const float* p = d->vertices + 3 * (3 * ((int64_t)ob.first_triangle + t) + j);
                v[j] = v3(p[0], p[1], p[2]);
                mn = v3(std::min(mn.x, v[j].x), std::min(mn.y, v[j].y), std::min(mn.z, v[j].z));
                mx = v3(std::max(mx.x, v[j].x), std::max(mx.y, v[j].y), std::max(mx.z, v[j].z));
            }
            V3 e1 = v[1] - v[0], e2 = v[2] - v[0];
            V3 n = normalized(cross(e1, e2));
            V3 c = cross(e1, e2);
            float area = std::sqrt(c.x * c.x + c.y * c.y + c.z * c.z) * 0.5f;
            DTri dt;
            dt.v0[0] = v[0].x; dt.v0[1] = v[0].y; dt.v0[2] = v[0].z;
            dt.e1[0] = e1.x; dt.e1[1] = e1.y; dt.e1[2] = e1.z;
            dt.e2[0] = e2.x; dt.e2[1] = e2.y; dt.e2[2] = e2.z;
            dt.nx = n.x; dt.ny = n.y; dt.nz = n.z;
            DTriX dx;
            dx.v1[0] = v[1].x; dx.v1[1] = v[1].y; dx.v1[2] = v[1].z;
            dx.v2[0] = v[2].x; dx.v2[1] = v[2].y; dx.v2[2] = v[2].z;
            dx.area = area;
            dx.mat = ob.material;
            hs.tris.push_back(dt);
            hs.trix.push_back(dx);
            hs.tri_object.push_back(o);
            mesh_area[o] += area;  // MeshTriangle::area, sequential (Triangle.cpp:70-73)
        }
        mesh_box[o] = box2(mn, mx);
    }
    const int ntri = (int)hs.tris.size();
    std::vector<int> sphere_prim(d->num_objects, -1);
    for (int o = 0; o < d->num_objects; ++o) {
        const tpt_object& ob = d->objects[o];
        if (ob.kind == TPT_OBJ_MESH) continue;
        if (ob.kind != TPT_OBJ_SPHERE) { err = "invalid object kind"; return TPT_E_INVALID; }
        DSphere s;
        std::memset(&s, 0, sizeof(s));
        s.c[0] = ob.center[0]; s.c[1] = ob.center[1]; s.c[2] = ob.center[2];
        s.r = ob.radius;
        s.r2 = ob.radius * ob.radius;
        s.area = 4 * kPi * ob.radius * ob.radius;  // Sphere.hpp:16
        s.mat = ob.material;
        sphere_prim[o] = ntri + (int)hs.sph.size();
        hs.sph.push_back(s);
    }

    // ---- per-mesh BVHs (each mesh's BVHAccel, Triangle.cpp:74)
    std::vector<Box> tri_box(ntri);
    std::vector<float> tri_area(ntri);
    for (int t = 0; t < ntri; ++t) {
        V3 v0 = v3(hs.tris[t].v0[0], hs.tris[t].v0[1], hs.tris[t].v0[2]);
        V3 v1 = v3(hs.trix[t].v1[0], hs.trix[t].v1[1], hs.trix[t].v1[2]);
        V3 v2 = v3(hs.trix[t].v2[0], hs.trix[t].v2[1], hs.trix[t].v2[2]);
        tri_box[t] = join(box2(v0, v1), v2);  // Triangle::GetBounds, Triangle.hpp:29
        tri_area[t] = hs.trix[t].area;
    }
    struct MeshTree { std::vector<BuildNode> nodes; int depth = 0; };
    std::vector<MeshTree> mtree(d->num_objects);
    for (int o = 0; o < d->num_objects; ++o) {
        if (d->objects[o].kind != TPT_OBJ_MESH || mesh_tris[o].count == 0) continue;
        Builder b(tri_box, tri_area);
        std::vector<int> items;
        for (int t = 0; t < mesh_tris[o].count; ++t) items.push_back(mesh_tris[o].first + t);
        b.build(items, 1);
        mtree[o].nodes = std::move(b.nodes);
        mtree[o].depth = b.depth;
    }

    // ---- scene-level BVH (Scene::BuildBVH, Scene.cpp:11-13)
    std::vector<Box> obj_box(d->num_objects);
    std::vector<float> obj_area(d->num_objects);
    for (int o = 0; o < d->num_objects; ++o) {
        if (d->objects[o].kind == TPT_OBJ_MESH) {
            obj_box[o] = mesh_box[o];
            obj_area[o] = mesh_area[o];
        } else {
            const DSphere& s = hs.sph[sphere_prim[o] - ntri];
            obj_box[o] = box2(v3(s.c[0] - s.r, s.c[1] - s.r, s.c[2] - s.r), v3(s.c[0] + s.r, s.c[1] + s.r, s.c[2] + s.r));
            obj_area[o] = s.area;
        }
    }
    Builder top(obj_box, obj_area);
    if (d->num_objects > 0) {
        std::vector<int> items;
        for (int o = 0; o < d->num_objects; ++o) items.push_back(o);
        top.build(items, 1);
    }

    // ---- flatten: scene-level nodes first, then each mesh's nodes
    const int ntop = (int)top.nodes.size();
    std::vector<int> mesh_base(d->num_objects, -1);
    int total = ntop;
    for (int o = 0; o < d->num_objects; ++o)
        if (!mtree[o].nodes.empty()) { mesh_base[o] = total; total += (int)mtree[o].nodes.size(); }
    hs.nodes.resize(total);
    hs.node_area.assign(total, 0.0f);
    for (int o = 0; o < d->num_objects; ++o) {
        if (mesh_base[o] < 0) continue;
        const std::vector<BuildNode>& mn = mtree[o].nodes;
        for (size_t k = 0; k < mn.size(); ++k) {
            const BuildNode& n = mn[k];
            int gi = mesh_base[o] + (int)k;
            if (n.item >= 0) hs.nodes[gi] = to_dnode(n.box, -1 - n.item, -1);
            else hs.nodes[gi] = to_dnode(n.box, mesh_base[o] + n.left, mesh_base[o] + n.right);
            hs.node_area[gi] = n.area;
        }
    }
    for (int k = 0; k < ntop; ++k) {
        const BuildNode& n = top.nodes[k];
        if (n.item < 0) {
            hs.nodes[k] = to_dnode(n.box, n.left, n.right);
            hs.node_area[k] = n.area;
            continue;
        }
        int o = n.item;
        if (d->objects[o].kind == TPT_OBJ_MESH) {
            if (mesh_base[o] < 0) hs.nodes[k] = to_dnode(n.box, kEmptyLeaf, -1);
            else {
                DNode root = hs.nodes[mesh_base[o]];
                hs.nodes[k] = to_dnode(n.box, root.a, root.b);  // identical box, see tpt_scene.h
            }
        } else {
            hs.nodes[k] = to_dnode(n.box, -1 - sphere_prim[o], -1);
        }
        hs.node_area[k] = n.area;
    }
    build_threads(hs, ntop, mesh_base);

    // ---- objects and emitters
    for (int o = 0; o < d->num_objects; ++o) {
        DObj ob;
        std::memset(&ob, 0, sizeof(ob));
        ob.kind = d->objects[o].kind;
        ob.mat = d->objects[o].material;
        ob.root = mesh_base[o];
        ob.sphere_prim = sphere_prim[o];
        if (ob.kind == TPT_OBJ_MESH) {
            ob.root_area = mesh_base[o] >= 0 ? hs.node_area[mesh_base[o]] : 0.0f;
            ob.pdf = 1.0f / ob.root_area;  // MeshTriangle::pdf
        } else {
            ob.root_area = hs.sph[sphere_prim[o] - ntri].area;
            ob.pdf = 1.0f / ob.root_area;  // Sphere::pdf
        }
        hs.objs.push_back(ob);
        if (hs.mats[ob.mat].has_em) hs.emitters.push_back(o);
    }
    hs.width = d->width;
    hs.height = d->height;
    for (int k = 0; k < 3; ++k) { hs.eye[k] = d->eye[k]; hs.bg[k] = d->background[k]; }
    hs.fov = d->fov;
    // PT shadow-cone masks (pt_cone_mask, tpt_device.h): the emitters' box and the margin
    double cmax = 0.0;
    for (int k = 0; k < 3; ++k) cmax = std::max(cmax, (double)std::fabs(hs.eye[k]));
    for (size_t t = 0; t < hs.tris.size(); ++t)
        for (int k = 0; k < 3; ++k)
            cmax = std::max({cmax, (double)std::fabs(hs.tris[t].v0[k]), (double)std::fabs(hs.trix[t].v1[k]),
                             (double)std::fabs(hs.trix[t].v2[k])});
    for (const DSphere& sp : hs.sph)
        for (int k = 0; k < 3; ++k) cmax = std::max(cmax, (double)std::fabs(sp.c[k]) + std::fabs(sp.r));
#ifndef TPT_CONE_DELTA_LOG2
// cone_delta = C 2^-16.  What it must cover, with C the largest coordinate magnitude:
// the origin (a float hit point on the emitter, ~C 2^-22 off the exact one), the
// direction (normalized in float: the ray passes within L 2^-21 <= C 2^-20 of x), the
// counting hit point (C 2^-23) and the float edges of Moller-Trumbore's triangles
// against their vertex boxes (C 2^-23, emitter and blocker): together < C 2^-19, so the
// margin is ~11x.  2^-12 (the first form) kept the ceiling, 0.1 above the light, in
// every cone: Standard PT 43.4 -> 42.4 ms with 2^-16.
#define TPT_CONE_DELTA_LOG2 (-16)
#endif
    hs.cone_delta = (float)std::max(std::ldexp(cmax, TPT_CONE_DELTA_LOG2), 0x1p-60);
    float lb[6] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
                   std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(),
                   -std::numeric_limits<float>::max(), -std::numeric_limits<float>::max()};
    auto grow = [&](const float* p) {
        for (int k = 0; k < 3; ++k) {
            lb[k] = std::min(lb[k], p[k]);
            lb[3 + k] = std::max(lb[3 + k], p[k]);
        }
    };
    for (int o : hs.emitters) {
        if (d->objects[o].kind == TPT_OBJ_MESH) {
            for (int t = mesh_tris[o].first; t < mesh_tris[o].first + mesh_tris[o].count; ++t) {
                grow(hs.tris[t].v0);
                grow(hs.trix[t].v1);
                grow(hs.trix[t].v2);
            }
        } else {
            const DSphere& sp = hs.sph[sphere_prim[o] - ntri];
            const float lo[3] = {sp.c[0] - sp.r, sp.c[1] - sp.r, sp.c[2] - sp.r};
            const float hi[3] = {sp.c[0] + sp.r, sp.c[1] + sp.r, sp.c[2] + sp.r};
            grow(lo);
            grow(hi);
        }
    }
    for (int k = 0; k < 6; ++k) hs.lbox[k] = lb[k];
    return TPT_OK;
}

}  // namespace tpt
