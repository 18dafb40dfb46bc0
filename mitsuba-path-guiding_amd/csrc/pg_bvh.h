// Host-side binned-SAH BVH2 builder producing the GPU layouts of pg_layout.h:
// 64-B nodes (both child boxes in the parent), 48-B Woop unit-triangle records, and the
// BVH-order triangle permutation.  Replaces the reference's SAH kd-tree build
// (include/mitsuba/render/sahkdtree3.h, gkdtree.h) — only the closest-hit contract is kept.
#pragma once
#include <stdint.h>

#include <vector>

namespace pgh {

struct BvhOut {
    std::vector<float> nodes;     // 16 floats per node
    std::vector<float> woop;      // 12 floats per triangle (BVH order)
    std::vector<uint32_t> order;  // BVH-order -> original triangle id
    uint32_t max_depth = 0;
    float lo[3], hi[3];
};

// positions: 3*nv floats, indices: 3*nt.  Returns false if the tree would exceed max_depth.
bool buildBvh(const float *positions, const uint32_t *indices, uint32_t nt, uint32_t stack_limit, BvhOut &out);

}  // namespace pgh
