// Host-side BVH builders producing the GPU layouts of pg_layout.h from one binned-SAH binary build
// (leaves <= 3 triangles): a 4-wide BVH (128-B nodes; binary 64-B nodes with PG_BVH4 = 0) for closest-hit rays, and an 8-wide BVH with
// quantised child boxes (80-B nodes, collapsed SAH-optimally from the same tree) for shadow rays,
// which it traverses with 28 % less time.  Both index one array of 48-B triangle records (pg_layout.h PG_TRIACCEL).  Replaces the reference's SAH kd-tree build
// (include/mitsuba/render/sahkdtree3.h, gkdtree.h) — only the closest-hit contract is kept.
#pragma once
#include <stdint.h>

#include <vector>

namespace pgh {

struct BvhOut {
    // closest-hit structure: 4-wide BVH, 4 * PG_QNODE_F4 floats per node (binary: 16), leaves index `order`
    std::vector<float> nodes;
    std::vector<float> tris;      // 12 floats per triangle (BVH order, pg_layout.h PG_TRIACCEL), shared by both BVHs
    std::vector<uint32_t> order;  // BVH-order -> original triangle id
    uint32_t max_depth = 0;
    uint32_t top_nodes = 0;       // nodes [0, top_nodes): the top PG_BVH_TOP_LEVELS levels, breadth first
    // any-hit structure: 8-wide BVH, 4 * PG_WIDE_NODE_F4 floats per node (root = node 0), over the
    // same triangle order
    std::vector<float> wnodes;
    uint32_t wide_depth = 0;
    float lo[3], hi[3];
};

// positions: 3*nv floats, indices: 3*nt.  Returns false if either tree is deeper than
// stack_limit - 1 (the traversal stacks hold at most one entry per level).
bool buildBvh(const float *positions, const uint32_t *indices, uint32_t nt, uint32_t stack_limit, BvhOut &out);

}  // namespace pgh
