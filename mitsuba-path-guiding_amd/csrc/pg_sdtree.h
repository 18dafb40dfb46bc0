// Host side of the SD-tree (Mueller et al. 2017): the topology refit that runs in the
// postprogression slot (src/librender/progressiveintegrator.cpp:314-317) and the flat device
// layout it uploads.  The per-sample work (lookup, sample, pdf, splat) runs on the GPU
// (pg_device.h / pg_kernels.hip); this refit is a few ms per training iteration on the host.
// Spec: DESIGN.md §"SD-tree" (restated from the paper; parity unpinned against the reference,
// which does not contain the guiding code).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace pgh {

struct SdNodeS {  // sampling quadtree node
    float sum[4] = {0, 0, 0, 0};
    uint32_t child[4] = {0, 0, 0, 0};  // tree-local, 0 = leaf
};
struct SdNodeB {  // building quadtree node
    uint64_t sum[4] = {0, 0, 0, 0};    // 2^-24 fixed point
    uint32_t child[4] = {0, 0, 0, 0};
};
// learned BSDF-sampling fraction (PG_FRACTION_LEARNED, pg_device.h fracStat): candidates and the
// number of u64 statistics per leaf (one cross-entropy sum per candidate + the guided-record count)
constexpr int kFracCandidates = 10;
constexpr int kFracStats = kFracCandidates + 1;
constexpr uint64_t kFracMinRecords = 64;  // fewer guided records: the leaf keeps its fraction
inline float fracCandidate(int k) { return 0.05f + 0.1f * (float)k; }

struct SdLeaf {  // D-tree pair attached to one S-tree leaf
    std::vector<SdNodeS> sampling{SdNodeS{}};
    float total = 0;
    float alpha = 0;  // learned BSDF-sampling fraction (0: not learned, pg_config.bsdf_sampling_fraction)
    std::vector<SdNodeB> building{SdNodeB{}};
    uint32_t count = 0;
    uint64_t frac[kFracStats] = {};  // building statistics of the fraction (two's complement sums)
};

struct SdTree {
    float lo[3] = {0, 0, 0}, extent = 1;
    std::vector<uint32_t> snode;  // 2 words per node: child0 (0xFFFFFFFF = leaf), child1 / leaf index
    std::vector<SdLeaf> leaves;
    bool built = false;

    void reset(const float bmin[3], const float bmax[3]);
    // learn: pick each leaf's BSDF-sampling fraction from its statistics (PG_FRACTION_LEARNED)
    void refit(uint32_t iteration, float s_threshold, float rho, int max_depth, bool learn = false);
    std::vector<uint8_t> serialize() const;
    bool deserialize(const uint8_t *p, size_t n);

    // the device layout (pg_kernels.h SDDev), written in place (e.g. into a pinned staging buffer)
    static constexpr int kJumpBits = 6;
    struct Layout {
        uint32_t *snodes;  // 2 per S-tree node
        uint32_t *meta;    // 4 per leaf: sampling base, building base, bits(alpha), bits(total)
        uint32_t *qnode;   // 8 per sampling node: f32 sum[4], u32 child[4] (absolute, 0 = leaf)
        uint32_t *bchild;  // 4 per building node (absolute)
        uint64_t *bsum;    // 4 per building node
        uint64_t *count;   // per leaf
        uint32_t *jump;    // (2^kJumpBits)^3 S-tree node ids or 0x80000000 | D-tree id inside one leaf, index (z * R + y) * R + x (nullptr: skipped)
        uint64_t *frac;    // kFracStats per leaf
    };
    void flattenInto(const Layout &d) const;
    // the same layout in owned arrays (wire format, tests)
    struct Flat {
        std::vector<uint32_t> snodes, meta, qnode, bchild, jump;
        std::vector<uint64_t> bsum, count, frac;
    };
    void flatten(Flat &f) const;
    // absorb device-side building sums/counts/fraction statistics (same absolute layout as flatten())
    void absorb(const uint64_t *bsum, const uint32_t *count, const uint64_t *frac);
    size_t samplingNodes() const;
    size_t buildingNodes() const;
};

}  // namespace pgh
