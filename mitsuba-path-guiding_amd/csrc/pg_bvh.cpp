// Binned-SAH BVH2 builder (host) — see pg_bvh.h.
#include "pg_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

#include "pg_layout.h"

namespace pgh {
namespace {

struct Box {
    float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                   std::numeric_limits<float>::infinity()};
    float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                   -std::numeric_limits<float>::infinity()};
    void grow(const float *p) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a]);
            hi[a] = std::max(hi[a], p[a]);
        }
    }
    void grow(const Box &b) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    float area() const {
        float e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
        if (!(e0 >= 0)) return 0.0f;
        return 2.0f * (e0 * e1 + e1 * e2 + e2 * e0);
    }
};

struct BNode {
    Box box;
    int32_t child[2] = {-1, -1};  // build-node indices (inner)
    uint32_t first = 0, count = 0;
    bool leaf = false;
};

constexpr int kBins = 32;
constexpr uint32_t kLeafTarget = 4;

}  // namespace

bool buildBvh(const float *P, const uint32_t *I, uint32_t nt, uint32_t stack_limit, BvhOut &out) {
    std::vector<Box> tb(nt);
    std::vector<float> cen(3 * (size_t)nt);
    Box all;
    for (uint32_t t = 0; t < nt; ++t) {
        for (int j = 0; j < 3; ++j) tb[t].grow(P + 3 * (size_t)I[3 * (size_t)t + j]);
        for (int a = 0; a < 3; ++a) cen[3 * (size_t)t + a] = 0.5f * (tb[t].lo[a] + tb[t].hi[a]);
        all.grow(tb[t]);
    }
    for (int a = 0; a < 3; ++a) {
        out.lo[a] = all.lo[a];
        out.hi[a] = all.hi[a];
    }
    std::vector<uint32_t> ord(nt);
    for (uint32_t t = 0; t < nt; ++t) ord[t] = t;
    std::vector<BNode> bn;
    bn.reserve(nt ? 2 * (size_t)nt / kLeafTarget + 8 : 8);
    struct Job { int32_t node; uint32_t first, count, depth; };
    std::vector<Job> st;
    bn.emplace_back();
    st.push_back({0, 0, nt, 0});
    uint32_t maxDepth = 0;
    while (!st.empty()) {
        Job j = st.back();
        st.pop_back();
        maxDepth = std::max(maxDepth, j.depth);
        Box box, cb;
        for (uint32_t i = j.first; i < j.first + j.count; ++i) {
            box.grow(tb[ord[i]]);
            cb.grow(&cen[3 * (size_t)ord[i]]);
        }
        bn[j.node].box = box;
        uint32_t mid = 0;
        bool leaf = j.count <= kLeafTarget;
        if (!leaf) {
            int bestAxis = -1, bestBin = -1;
            float bestCost = std::numeric_limits<float>::infinity();
            const bool median = j.depth >= 32;  // bound the depth: object-median splits from here on
            if (!median) {
                for (int ax = 0; ax < 3; ++ax) {
                    float lo = cb.lo[ax], hi = cb.hi[ax];
                    if (!(hi > lo)) continue;
                    float k = kBins / (hi - lo);
                    Box bb[kBins];
                    uint32_t bc[kBins] = {0};
                    for (uint32_t i = j.first; i < j.first + j.count; ++i) {
                        int b = std::min(kBins - 1, std::max(0, (int)((cen[3 * (size_t)ord[i] + ax] - lo) * k)));
                        bb[b].grow(tb[ord[i]]);
                        bc[b]++;
                    }
                    float la[kBins];
                    uint32_t lc[kBins];
                    Box acc;
                    uint32_t n = 0;
                    for (int b = 0; b < kBins; ++b) {
                        acc.grow(bb[b]);
                        n += bc[b];
                        la[b] = acc.area();
                        lc[b] = n;
                    }
                    acc = Box();
                    n = 0;
                    for (int b = kBins - 1; b > 0; --b) {
                        acc.grow(bb[b]);
                        n += bc[b];
                        if (lc[b - 1] == 0 || n == 0) continue;
                        float cost = la[b - 1] * lc[b - 1] + acc.area() * n;
                        if (cost < bestCost) {
                            bestCost = cost;
                            bestAxis = ax;
                            bestBin = b;
                        }
                    }
                }
                float leafCost = box.area() * (float)j.count;
                float splitCost = box.area() * 1.0f + bestCost;  // traversal cost ~ 1 triangle test
                if (bestAxis >= 0 && splitCost >= leafCost && j.count <= PG_LEAF_MAX) leaf = true;
            }
            if (!leaf) {
                if (bestAxis >= 0 && !median) {
                    float lo = cb.lo[bestAxis], hi = cb.hi[bestAxis];
                    float k = kBins / (hi - lo);
                    auto it = std::partition(ord.begin() + j.first, ord.begin() + j.first + j.count, [&](uint32_t t) {
                        int b = std::min(kBins - 1, std::max(0, (int)((cen[3 * (size_t)t + bestAxis] - lo) * k)));
                        return b < bestBin;
                    });
                    mid = (uint32_t)(it - ord.begin());
                }
                if (bestAxis < 0 || median || mid == j.first || mid == j.first + j.count) {
                    if (j.count <= 15 && bestAxis < 0 && !median) {
                        leaf = true;  // coincident centroids, small enough
                    } else {
                        int ax = 0;
                        float ext = -1;
                        for (int a = 0; a < 3; ++a)
                            if (cb.hi[a] - cb.lo[a] > ext) {
                                ext = cb.hi[a] - cb.lo[a];
                                ax = a;
                            }
                        mid = j.first + j.count / 2;
                        std::nth_element(ord.begin() + j.first, ord.begin() + mid, ord.begin() + j.first + j.count,
                                         [&](uint32_t a, uint32_t b) {
                                             return cen[3 * (size_t)a + ax] < cen[3 * (size_t)b + ax];
                                         });
                    }
                }
            }
        }
        if (leaf) {
            bn[j.node].leaf = true;
            bn[j.node].first = j.first;
            bn[j.node].count = j.count;
        } else {
            int32_t l = (int32_t)bn.size();
            bn.emplace_back();
            bn.emplace_back();
            bn[j.node].child[0] = l;
            bn[j.node].child[1] = l + 1;
            st.push_back({l + 1, mid, j.first + j.count - mid, j.depth + 1});
            st.push_back({l, j.first, mid - j.first, j.depth + 1});
        }
    }
    out.max_depth = maxDepth;
    if (maxDepth + 1 > stack_limit) return false;

    // ---- pack: inner nodes get GPU indices in DFS order; a leaf root gets a synthetic parent
    out.order = ord;
    out.woop.assign(12 * (size_t)nt, 0.0f);
    for (uint32_t k = 0; k < nt; ++k) {
        uint32_t t = ord[k];
        const float *v0 = P + 3 * (size_t)I[3 * (size_t)t], *v1 = P + 3 * (size_t)I[3 * (size_t)t + 1],
                    *v2 = P + 3 * (size_t)I[3 * (size_t)t + 2];
        double e0[3], e1[3], n[3];
        for (int a = 0; a < 3; ++a) {
            e0[a] = (double)v0[a] - v2[a];
            e1[a] = (double)v1[a] - v2[a];
        }
        n[0] = e0[1] * e1[2] - e0[2] * e1[1];
        n[1] = e0[2] * e1[0] - e0[0] * e1[2];
        n[2] = e0[0] * e1[1] - e0[1] * e1[0];
        // M = [e0 e1 n] (columns); rows of M^-1 map (p - v2) -> (a, b, c)
        double m[3][3] = {{e0[0], e1[0], n[0]}, {e0[1], e1[1], n[1]}, {e0[2], e1[2], n[2]}};
        double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) - m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                     m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
        float *w = &out.woop[12 * (size_t)k];
        if (!(std::fabs(det) > 0) || !std::isfinite(det)) continue;  // degenerate: never hit (NaN t)
        double inv[3][3];
        inv[0][0] = (m[1][1] * m[2][2] - m[1][2] * m[2][1]) / det;
        inv[0][1] = (m[0][2] * m[2][1] - m[0][1] * m[2][2]) / det;
        inv[0][2] = (m[0][1] * m[1][2] - m[0][2] * m[1][1]) / det;
        inv[1][0] = (m[1][2] * m[2][0] - m[1][0] * m[2][2]) / det;
        inv[1][1] = (m[0][0] * m[2][2] - m[0][2] * m[2][0]) / det;
        inv[1][2] = (m[0][2] * m[1][0] - m[0][0] * m[1][2]) / det;
        inv[2][0] = (m[1][0] * m[2][1] - m[1][1] * m[2][0]) / det;
        inv[2][1] = (m[0][1] * m[2][0] - m[0][0] * m[2][1]) / det;
        inv[2][2] = (m[0][0] * m[1][1] - m[0][1] * m[1][0]) / det;
        auto rowdot = [&](int r) { return inv[r][0] * v2[0] + inv[r][1] * v2[1] + inv[r][2] * v2[2]; };
        // w0: c(p) = r2.p - r2.v2 ; stored as (r2, r2.v2) so that t = (w0.w - r2.o) / r2.d
        w[0] = (float)inv[2][0];
        w[1] = (float)inv[2][1];
        w[2] = (float)inv[2][2];
        w[3] = (float)rowdot(2);
        w[4] = (float)inv[0][0];
        w[5] = (float)inv[0][1];
        w[6] = (float)inv[0][2];
        w[7] = (float)(-rowdot(0));
        w[8] = (float)inv[1][0];
        w[9] = (float)inv[1][1];
        w[10] = (float)inv[1][2];
        w[11] = (float)(-rowdot(1));
    }

    std::vector<int32_t> gpuIndex(bn.size(), -1);
    std::vector<int32_t> innerOrder;
    {
        std::vector<int32_t> s{0};
        while (!s.empty()) {
            int32_t n = s.back();
            s.pop_back();
            if (bn[n].leaf) continue;
            gpuIndex[n] = (int32_t)innerOrder.size();
            innerOrder.push_back(n);
            s.push_back(bn[n].child[1]);
            s.push_back(bn[n].child[0]);
        }
    }
    auto ref = [&](int32_t n) -> int32_t {
        if (bn[n].leaf) return (int32_t)(~((bn[n].first << 4) | bn[n].count));
        return gpuIndex[n];
    };
    auto putNode = [&](float *o, const Box &b0, int32_t r0, const Box &b1, int32_t r1) {
        o[0] = b0.lo[0]; o[1] = b0.hi[0]; o[2] = b0.lo[1]; o[3] = b0.hi[1];
        o[4] = b1.lo[0]; o[5] = b1.hi[0]; o[6] = b1.lo[1]; o[7] = b1.hi[1];
        o[8] = b0.lo[2]; o[9] = b0.hi[2]; o[10] = b1.lo[2]; o[11] = b1.hi[2];
        std::memcpy(&o[12], &r0, 4);
        std::memcpy(&o[13], &r1, 4);
        o[14] = 0;
        o[15] = 0;
    };
    if (innerOrder.empty()) {  // the root is a leaf: synthetic inner root + empty far-away leaf
        out.nodes.assign(16, 0.0f);
        Box far;
        for (int a = 0; a < 3; ++a) far.lo[a] = far.hi[a] = 1e30f;
        int32_t empty = (int32_t)(~0u << 4);  // ~((0 << 4) | 0) with count 0
        empty = ~(int32_t)0;                  // first 0, count 0
        putNode(&out.nodes[0], bn[0].box, ref(0), far, empty);
        return true;
    }
    out.nodes.assign(16 * innerOrder.size(), 0.0f);
    for (size_t i = 0; i < innerOrder.size(); ++i) {
        const BNode &n = bn[innerOrder[i]];
        putNode(&out.nodes[16 * i], bn[n.child[0]].box, ref(n.child[0]), bn[n.child[1]].box, ref(n.child[1]));
    }
    return true;
}

}  // namespace pgh
