// tpt_scene_build.h -- host-side flattened scene (input to the HBM upload).
#pragma once
#include <string>
#include <vector>

#include "../../include/tpt.h"
#include "tpt_scene.h"

namespace tpt {

struct HostScene {
    std::vector<DNode> nodes;
    std::vector<DNode> tnodes;
    std::vector<DNode> leaves;  // primitive leaves in the reference's visit order (flat queries)
    std::vector<DNode> groups;  // per object: its box, first leaf (a) and leaf count (b); b < 0: walk group
    std::vector<DTri> ftris;    // flat-only LDS mode: the triangle of each flat leaf, in leaf order
    std::vector<QNode4> qnodes; // 4-wide trees of the walk groups
    std::vector<uint16_t> grank; // per triangle: rank of its leaf in its walk group's DFS visit order
    int grank_next = 0;          // (build_qtree's counter, reset per walk group)
    std::vector<float> node_area;
    std::vector<DTri> tris;
    std::vector<DTriX> trix;
    std::vector<int> tri_object;
    std::vector<DSphere> sph;
    std::vector<DMat> mats;
    std::vector<DObj> objs;
    std::vector<int32_t> emitters;
    // the emitters' bounding box (every emitter's triangle vertices and sphere bounds) and
    // the margin of the PT shadow-cone masks (pt_cone_mask): C * 2^-16, C bounding every
    // scene and eye coordinate
    float lbox[6] = {0, 0, 0, 0, 0, 0};
    float cone_delta = 0.0f;
    int width = 0, height = 0;
    float eye[3] = {0, 0, 0};
    float bg[3] = {0, 0, 0};
    double fov = 40.0;
};

int build_host_scene(const tpt_scene_desc* d, HostScene& hs, std::string& err);

}  // namespace tpt
