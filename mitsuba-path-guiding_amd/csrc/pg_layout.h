// GPU record layouts shared by the host driver (pg_host.cpp) and the kernels (pg_kernels.hip).
// Sizes are static_asserted; DESIGN.md §"Data layout in HBM" documents them.
#pragma once
#include <stdint.h>

#include "../../include/pg_capi.h"

// Material record: 128 B (8 x 16 B), derived constants precomputed on the host (BSDF::configure()).
struct GMat {
    uint32_t model, dist, flags, type;  // pg BSDF model, microfacet distribution, PG_MAT_* flags, EBSDFType bits
    float alpha_u, alpha_v, eta, invEta;
    float invEta2, fdrInt, specWeight, wbound;  // wbound: max channel of BSDF::getAlbedo (guide-fraction bound)
    float diff[4];
    float spec[4];
    float trans[4];
    union {
        float ceta[4];
        struct {
            const float *rtrans;  // roughplastic: external rough-transmittance table (device)
            float pad1[2];
        };
    };
    float ck[4];
};
static_assert(sizeof(GMat) == 128, "GMat layout");

// Area emitter record: 32 B.  Triangles of emitter e are em_tri[tri_begin, tri_begin + tri_count),
// each with its normalized area-CDF entry em_cdf[tri_begin + 1 + i] (em_cdf[tri_begin] = 0 slot
// lives at index tri_begin + e, see pg_host.cpp: cdf arrays are stored with one leading zero each).
struct GEmitter {
    uint32_t tri_begin;   // into em_tri
    uint32_t tri_count;
    uint32_t cdf_begin;   // into em_cdf (tri_count + 1 entries)
    float inv_area;
    float radiance[4];
};
static_assert(sizeof(GEmitter) == 32, "GEmitter layout");

// Environment emitter record: 128 B (EnvironmentMap, envmap.cpp:260-329).  texels: width x height
// float4 (rgb rounded to half precision, as the reference's SpectrumHalf MIP level 0; w = 0), row
// y = theta.  cdf_rows: height + 1 marginal CDF entries; cdf_cols: height rows of width + 1
// conditional CDF entries; row_weights: sin((y + 0.5) pi / height).  R: toWorld rotation,
// row-major (world = R local, local = R^T world).  center/radius: the scene's bounding sphere
// enlarged by 1.5 (EnvironmentMap::createShape, envmap.cpp:331-356).
struct GEnv {
    const float *texels;  // float4 per texel
    const float *cdf_rows;
    const float *cdf_cols;
    const float *row_weights;
    uint32_t width, height;
    float scale, normalization;
    float pixel_size[2];
    float radius, pad0;
    float center[3], pad1;
    float R[9];
    float pad2[3];
};
static_assert(sizeof(GEnv) == 128, "GEnv layout");

// Heterogeneous medium record: 128 B (volpath).  World -> grid is g = p * gs + go
// (gridvolume.cpp:186-198); invMax = 1 / (scale * maxFloatValue), maxFloatValue = 1
// (gridvolume.cpp:583-585, heterogeneous.cpp:236-242).  density: res x*y*z floats, x fastest.
// maj: the majorant grid, mx*my*mz cells of PG_MAJORANT_CELL^3 voxels, each scale * the maximum
// voxel over the cell extended by one voxel per side.
// With PG_DENSITY_BRICKS = 1 the density is stored in 4x4x4-voxel bricks of 256 B (bricks x fastest,
// bx * by bricks per z layer; inside a brick x, then y, then z): the 2x2x2 corners of a trilinear
// lookup then touch ~2.3 cache lines instead of 4 rows of the linear layout.
#ifndef PG_MAJORANT_CELL
#define PG_MAJORANT_CELL 16  // voxels per majorant cell and axis (oracle: orc_medium.h kCell)
#endif
#ifndef PG_DENSITY_CORNERS
#define PG_DENSITY_CORNERS 1  // corner-packed density (below); 0: linear voxels (or bricks)
#endif
#ifndef PG_DENSITY_BRICKS
#define PG_DENSITY_BRICKS 0  // measured: no gain over the linear layout (DESIGN.md "Volumes")
#endif
#if PG_DENSITY_BRICKS  // bricks replace the corner packing
#undef PG_DENSITY_CORNERS
#define PG_DENSITY_CORNERS 0
#endif
struct GMedium {
    const float *density;
    uint32_t resx, resy;
    uint32_t resz;
    float scale, invMax, g;
    float lo[3];
    uint32_t mx;
    float hi[3];
    uint32_t my;
    float gs[3];
    uint32_t mz;
    float go[3];
    uint32_t bx;  // bricks along x (PG_DENSITY_BRICKS)
    float albedo[3];
    uint32_t by;  // bricks along y
    const float *maj;
    uint32_t pad4, pad5;
};
static_assert(sizeof(GMedium) == 128, "GMedium layout");
// Corner-packed density (PG_DENSITY_CORNERS, the default build; the layout is a compile-time choice of
// lookupDensity, there is no runtime fallback, and an upload that cannot hold it fails with PG_ERR_OOM): cell (x, y, z) of the
// (rx-1)(ry-1)(rz-1) cells between voxel centres stores its 8 corner voxels, 32 B in lookup order
// (z, y, x bits: d000 d001 d010 d011 | d100 d101 d110 d111), so a trilinear lookup is two aligned
// 16-B loads instead of eight scattered 4-B loads over four cache lines.  8x the memory of the grid
// (530 MB for 256^3): a trade the 288 GB of HBM3E affords.

// Triangle records of both BVHs (48 B = 3 x float4 per BVH-order triangle).  PG_TRIACCEL (default): the
// reference's own triangle test, TriAccel (include/mitsuba/render/triaccel.h:37-157; the oracle's
// orc_scene.h TriAccel): (n_u, n_v, n_d, bits(k)), (a_u, a_v, b_nu, b_nv), (c_nu, c_nv, bits(original
// triangle id), 0), built in fp32 as TriAccel::load builds it and tested with contraction off, so a hit's
// t and barycentrics are the oracle's bit for bit; k = 3 marks a degenerate triangle (NaN plane: never
// hit).  PG_TRIACCEL = 0: Woop unit-triangle rows (rows of [e0 e1 n]^-1 in double; A/B).
#ifndef PG_TRIACCEL
#define PG_TRIACCEL 1
#endif
// PG_TRI_BLOCKED: the records in blocks of 8 BVH-order triangles (384 B, three 128-B lines): the 8 first rows,
// then the 8 (row 1, row 2) pairs.  A leaf's first-row loads share one line, and rows 1-2, loaded only for
// triangles whose plane distance passes, never straddle a line.  0: three consecutive rows per triangle.
#ifndef PG_TRI_BLOCKED
#define PG_TRI_BLOCKED 0
#endif
// float4 index of row r (0-2) of BVH-order triangle tr; PG_TRI_F4(nt) float4 for nt triangles
#if PG_TRI_BLOCKED
#define PG_TRI_ROW(tr, r) (24u * ((uint32_t)(tr) >> 3) + ((r) == 0 ? ((uint32_t)(tr) & 7u) : 7u + 2u * ((uint32_t)(tr) & 7u) + (r)))
#define PG_TRI_F4(nt) (24u * (((uint32_t)(nt) + 7u) >> 3))
#else
#define PG_TRI_ROW(tr, r) (3u * (uint32_t)(tr) + (r))
#define PG_TRI_F4(nt) (3u * (uint32_t)(nt))
#endif

// Volumetric flight order key (pg_volpath.hip flightKey): 0 = 16^3 cells (4096 sort bins), 1 = direction
// octant + 8^3 cells (4096), 2 = 8^3 cells (512 bins: an eighth of the counting sort's per-tile atomics)
#ifndef PG_VOL_SORT_KEY
#define PG_VOL_SORT_KEY 2
#endif
#define PG_VOL_SORT_BINS (PG_VOL_SORT_KEY == 2 ? 512u : 4096u)

// Per-triangle shading record (5 x float4 = 80 B), indexed by BVH-order triangle id:
//   [0] p0.xyz, bits(material | (emitter + 1) << 16)
//   [1] p1.xyz, n2.z
//   [2] p2.xyz, bits(original triangle id)
//   [3] n0.xyz, n1.x
//   [4] n1.y, n1.z, n2.x, n2.y
// The same layout is used for the compact emitter-triangle array.
#define PG_TRI_SHADE_F4 5
// float4 per triangle in the BVH-order array (tshade); 8 pads a record to one 128-B line (A/B: half of the
// 80-B records straddle two).  The emitter-triangle array keeps PG_TRI_SHADE_F4.
#ifndef PG_TRI_SHADE_STRIDE
#define PG_TRI_SHADE_STRIDE PG_TRI_SHADE_F4
#endif

// Binary BVH node for closest-hit rays (PG_BVH4 = 0 builds; 4 x float4 = 64 B):
//   [0] c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y   [1] c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y
//   [2] c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z   [3] bits(child0), bits(child1), 0, 0
// child >= 0: inner node index; child < 0: leaf, ~child = (first_tri << 4) | count (count <= 15).
#define PG_BVH_NODE_F4 4
#define PG_LEAF_MAX 3  // the binary tree is the one the 8-wide BVH collapses (PG_WIDE_LEAF_MAX)
// The inner nodes of the top PG_BVH_TOP_LEVELS levels come first, in breadth-first order (the rest
// in depth-first order): k_trace stages nodes [0, SceneDev.top_nodes) in LDS once per block.
#define PG_BVH_TOP_LEVELS 5
#define PG_BVH_TOP_NODES 31

// 4-wide BVH node for closest-hit rays (default, PG_BVH4 = 1; 8 x float4 = 128 B, one L2 line), collapsed
// from the same binary tree by opening the largest-area inner child until four slots are used
// (C3 +1.5 %, kitchen +6.9 %, C5 +3.1 % over the binary nodes, identical results; profiles/r03za_bvh4_ab):
//   [0] lo.x[4]  [1] hi.x[4]  [2] lo.y[4]  [3] hi.y[4]  [4] lo.z[4]  [5] hi.z[4]   (slot order)
//   [6] bits(child[4]) with the binary node's encoding (>= 0 inner, < 0 leaf), PG_QNODE_EMPTY unused
//   [7] 0
#ifndef PG_BVH4
#define PG_BVH4 1
#endif
// PG_QNODE_QUANT = 1: the same tree in 64-B nodes (4 x float4) with child boxes quantised to bytes in the
// node's frame (as the 8-wide shadow nodes):
//   [0] origin.xyz (the node box's lo corner), bits((e_x + 127) | (e_y + 127) << 8 | (e_z + 127) << 16)
//   [1] bits(child[4])
//   [2] u32 lo.x, hi.x, lo.y, hi.y  [3] u32 lo.z, hi.z, 0, 0   -- byte s of each word: slot s's plane
// plane = origin + q * 2^e, rounded outward (floor / ceil, checked against the fp32 reconstruction);
// an empty slot has lo = 255, hi = 0 (an inverted box) and the PG_QNODE_EMPTY ref
#ifndef PG_QNODE_QUANT
#define PG_QNODE_QUANT 1
#endif
#if PG_QNODE_QUANT
#define PG_QNODE_F4 4
#else
#define PG_QNODE_F4 8
#endif
#define PG_QNODE_EMPTY 0x7ffffffe
// The 4-wide nodes of the top PG_BVH4_TOP_LEVELS + 1 levels come first, breadth first (round 5; the rest
// depth first): k_rays / k_trace stage nodes [0, SceneDev.top_nodes) in LDS with PG_RAYS_LDS_TOP (A/B).
// 1 + 4 + 16 = 21 nodes, 1.3 KiB of quantised nodes.
#ifndef PG_BVH4_TOP_LEVELS
#define PG_BVH4_TOP_LEVELS 2
#endif
#define PG_BVH4_TOP_NODES 21
// closest-hit stack entries a 4-wide traversal may need (the builder checks its trees against it;
// the global overflow ring already holds PG_QSTACK_DEPTH - LDS_STACK words per thread)
#define PG_QSTACK_DEPTH 96
// host-side accessors of a 4-wide node (either layout; tests/csrc/bvh_shim.cpp): slot s's ref and box
inline int32_t pg_qnode_ref(const float *node, int s) {
    int32_t r;
    __builtin_memcpy(&r, node + (PG_QNODE_QUANT ? 4 : 24) + s, 4);
    return r;
}
inline void pg_qnode_box(const float *node, int s, float lo[3], float hi[3]) {
#if PG_QNODE_QUANT
    uint32_t e, w[6];
    __builtin_memcpy(&e, node + 3, 4);
    __builtin_memcpy(w, node + 8, 24);
    for (int a = 0; a < 3; ++a) {
        uint32_t eb = ((e >> (8 * a)) & 0xFFu) << 23;
        float scale;
        __builtin_memcpy(&scale, &eb, 4);
        lo[a] = node[a] + (float)((w[2 * a] >> (8 * s)) & 0xFFu) * scale;
        hi[a] = node[a] + (float)((w[2 * a + 1] >> (8 * s)) & 0xFFu) * scale;
    }
#else
    for (int a = 0; a < 3; ++a) {
        lo[a] = node[8 * a + s];
        hi[a] = node[8 * a + 4 + s];
    }
#endif
}

// 8-wide BVH node for shadow rays, with quantised child boxes (5 x float4 = 80 B; after Ylitie et al. 2017):
//   [0] p.xyz (quantisation origin = node box min), bits(ex | ey << 8 | ez << 16 | imask << 24)
//       child box coordinate = p + q * 2^(e - 127) per axis; imask bit s: slot s is an inner node
//   [1] child_base (inner children are consecutive nodes, in slot order), tri_base (leaf triangles
//       are consecutive BVH-order triangles, in slot order), meta[8] (bytes): leaf slot s =
//       offset from tri_base | count << 5 (count 1..3), 0 = empty slot
//   [2] qlo.x[8] qlo.y[8]   [3] qlo.z[8] qhi.x[8]   [4] qhi.y[8] qhi.z[8]   (uint8, slot order)
// Slot s holds the child that rays of direction octant s (bit a = negative along axis a) should
// visit first, so traversal orders hits by slot ^ (7 - octant) without sorting.
// PG_WIDE_NODE_F4: float4 per node; 8 pads a node to one 128-B line (A/B: half of the 80-B nodes straddle two)
#ifndef PG_WIDE_NODE_F4
#define PG_WIDE_NODE_F4 5
#endif
#define PG_WIDE_LEAF_MAX 3

// Material classes of the per-bounce shading queues (k_classify -> k_shade<MODEL>)
#define PG_CLASS_DIFFUSE 0
#define PG_CLASS_ROUGHCONDUCTOR 1
#define PG_CLASS_ROUGHDIELECTRIC 2
#define PG_CLASS_PLASTIC 3
#define PG_CLASS_ROUGHPLASTIC 4
#define PG_CLASS_DELTA 5
#define PG_NUM_CLASSES 6

// Path-state flags (pinfo.z high bits)
#define PF_SCATTERED 0x1u
#define PF_EMITTED_QUERY 0x2u
#define PF_PREV_DELTA 0x4u

// Kernel-side constants of one render context.
struct GParams {
    // camera
    float cam_o[3], cam_left[3], cam_up[3], cam_dir[3];
    float tan_half, aspect, near_clip, far_clip;
    uint32_t width, height;
    // integrator
    int32_t max_depth, rr_depth, use_nee, hide_emitters, strict_normals, guiding, record, max_vertices;
    float max_component_value, bsdf_fraction;
    uint32_t seed, num_emitters, num_materials, depth_cap;  // num_emitters counts the environment emitter
    int32_t fraction_bound;  // pg_config.bsdf_fraction_bound (PG_FRACTION_*)
    int32_t exact_mis;       // pg_config.volpath_exact_mis
    int32_t glossy_prior;    // pg_config.glossy_prior
};
