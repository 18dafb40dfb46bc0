// Binned-SAH BVH2 builder (host) — see pg_bvh.h.
#include "pg_bvh.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
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
// SAH constants: leaves of at most kLeafTarget triangles are never split; a triangle test costs
// kTriCost node traversals.  PG_BVH_LEAF_TARGET / PG_BVH_TRI_COST override them (A/B measurements).
uint32_t leafTarget() {
    const char *e = std::getenv("PG_BVH_LEAF_TARGET");
    return e ? (uint32_t)std::atoi(e) : 2u;
}
float triCost() {
    const char *e = std::getenv("PG_BVH_TRI_COST");
    return e ? (float)std::atof(e) : 1.0f;
}

}  // namespace

// Binned-SAH binary build: nodes bn (bn[0] = root), triangle permutation ord, leaves of at most
// maxLeaf triangles (SAH leaf/split decision, object median past depth 32).
static void buildBinary(const float *P, const uint32_t *I, uint32_t nt, uint32_t maxLeaf, std::vector<BNode> &bn,
                 std::vector<uint32_t> &ord, uint32_t &maxDepth, Box &all) {
    std::vector<Box> tb(nt);
    std::vector<float> cen(3 * (size_t)nt);
    all = Box();
    for (uint32_t t = 0; t < nt; ++t) {
        for (int j = 0; j < 3; ++j) tb[t].grow(P + 3 * (size_t)I[3 * (size_t)t + j]);
        for (int a = 0; a < 3; ++a) cen[3 * (size_t)t + a] = 0.5f * (tb[t].lo[a] + tb[t].hi[a]);
        all.grow(tb[t]);
    }
    ord.assign(nt, 0);
    for (uint32_t t = 0; t < nt; ++t) ord[t] = t;
    bn.clear();
    const uint32_t kLeafTarget = std::max(1u, leafTarget());
    const float kTri = triCost();
    bn.reserve(nt ? 2 * (size_t)nt / kLeafTarget + 8 : 8);
    struct Job { int32_t node; uint32_t first, count, depth; };
    std::vector<Job> st;
    bn.emplace_back();
    st.push_back({0, 0, nt, 0});
    maxDepth = 0;
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
        bool leaf = j.count <= std::min(kLeafTarget, maxLeaf);
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
                float leafCost = box.area() * (float)j.count * kTri;
                float splitCost = box.area() * 1.0f + bestCost * kTri;  // one node visit + the children's tests
                if (bestAxis >= 0 && splitCost >= leafCost && j.count <= maxLeaf) leaf = true;
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
                    if (j.count <= maxLeaf && bestAxis < 0 && !median) {
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
}

// Woop unit-triangle record (3 x float4) of triangle t: rows of the inverse of [e0 e1 n] in double.
static void woopRecord(const float *P, const uint32_t *I, uint32_t t, float *w) {
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
    for (int k = 0; k < 12; ++k) w[k] = 0.0f;
    if (!(std::fabs(det) > 0) || !std::isfinite(det)) return;  // degenerate: never hit (NaN t)
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

// TriAccel record of triangle t (TriAccel::load, triaccel.h:37-94, in fp32 as the reference computes
// it; this file builds with -ffp-contract=off): 12 floats, pg_layout.h PG_TRIACCEL
static void triAccelRecord(const float *P, const uint32_t *I, uint32_t t, float *w) {
    static const int waldModulo[4] = {1, 2, 0, 1};
    const float *A = P + 3 * (size_t)I[3 * (size_t)t], *B = P + 3 * (size_t)I[3 * (size_t)t + 1],
                *C = P + 3 * (size_t)I[3 * (size_t)t + 2];
    const float b[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]}, c[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
    const float N[3] = {c[1] * b[2] - c[2] * b[1], c[2] * b[0] - c[0] * b[2], c[0] * b[1] - c[1] * b[0]};  // cross(c, b)
    int k = 0;
    for (int j = 0; j < 3; ++j)
        if (std::fabs(N[j]) > std::fabs(N[k])) k = j;
    const int u = waldModulo[k], v = waldModulo[k + 1];
    const float n_k = N[k], denom = b[u] * c[v] - b[v] * c[u];
    for (int i = 0; i < 12; ++i) w[i] = 0.0f;
    uint32_t kk = (uint32_t)k;
    if (denom == 0) {  // degenerate: k = 3, a NaN plane that no t passes
        w[0] = w[1] = w[2] = std::numeric_limits<float>::quiet_NaN();
        kk = 3;
    } else {
        w[0] = N[u] / n_k;                                          // n_u
        w[1] = N[v] / n_k;                                          // n_v
        w[2] = (A[0] * N[0] + A[1] * N[1] + A[2] * N[2]) / n_k;    // n_d = dot(A, N) / n_k
        w[4] = A[u];                                                // a_u
        w[5] = A[v];                                                // a_v
        w[6] = b[u] / denom;                                        // b_nu
        w[7] = -b[v] / denom;                                       // b_nv
        w[8] = c[v] / denom;                                        // c_nu
        w[9] = -c[u] / denom;                                       // c_nv
    }
    std::memcpy(&w[3], &kk, 4);
    std::memcpy(&w[10], &t, 4);  // the original triangle id
}

namespace {

// Child-slot assignment by ray octant: slot s holds the child a ray of octant s (bit a set =
// negative direction along axis a) should visit first, i.e. the child minimising
// dot(centroid - parent centroid, diag(s)).  Greedy over the sorted (cost, child, slot) table.
void assignSlots(const Box &parent, const std::vector<Box> &cb, int slotOf[8]) {
    const int k = (int)cb.size();
    float pc[3];
    for (int a = 0; a < 3; ++a) pc[a] = 0.5f * (parent.lo[a] + parent.hi[a]);
    struct C { float cost; int child, slot; };
    std::vector<C> tab;
    for (int i = 0; i < k; ++i) {
        float v[3];
        for (int a = 0; a < 3; ++a) v[a] = 0.5f * (cb[i].lo[a] + cb[i].hi[a]) - pc[a];
        for (int sl = 0; sl < 8; ++sl) {
            float c = 0;
            for (int a = 0; a < 3; ++a) c += ((sl >> a) & 1) ? -v[a] : v[a];
            tab.push_back({c, i, sl});
        }
    }
    std::stable_sort(tab.begin(), tab.end(), [](const C &x, const C &y) { return x.cost < y.cost; });
    bool usedSlot[8] = {false};
    for (int i = 0; i < k; ++i) slotOf[i] = -1;
    for (const C &c : tab) {
        if (slotOf[c.child] >= 0 || usedSlot[c.slot]) continue;
        slotOf[c.child] = c.slot;
        usedSlot[c.slot] = true;
    }
}

// power-of-two scale exponent with 255 * 2^e >= extent
int quantExponent(float extent) {
    if (!(extent > 0)) return -126;
    int e;
    std::frexp((double)extent / 255.0, &e);  // extent/255 = m * 2^e, m in [0.5, 1)
    return std::max(-126, std::min(127, e));
}

}  // namespace

// 8-wide BVH (for any-hit queries), collapsed from the binary tree (bn, ord); its leaf slots copy the
// binary leaves' triangle ranges contiguously, and that copy order (out.order) is the one triangle
// order of both BVHs: posOf[i] = the position of ord[i] in it.
static bool buildWide(const float *P, const uint32_t *I, uint32_t nt, uint32_t stack_limit, const std::vector<BNode> &bn,
                      const std::vector<uint32_t> &ord, BvhOut &out, std::vector<uint32_t> &posOf) {
    // ---- collapse to 8-wide nodes, SAH-optimal over the binary tree (dynamic programming after
    // Ylitie et al. 2017): dist[n][j] = cheapest way to spread subtree n over at most j slots of
    // one wide node; a slot is a leaf (subtree of <= PG_WIDE_LEAF_MAX triangles, one contiguous
    // range of `ord`) or an inner wide node.
    const size_t nb = bn.size();
    constexpr float kCostNode = 1.0f, kCostTri = 0.3f;
    constexpr float kInf = std::numeric_limits<float>::infinity();
    std::vector<uint32_t> rFirst(nb), rCount(nb);
    std::vector<std::array<float, 9>> dist(nb);
    std::vector<float> cWide(nb, kInf), cLeaf(nb, kInf);
    std::vector<std::array<uint8_t, 9>> splitK(nb);  // best left share for dist[n][j], 0 = n as one slot
    {
        std::vector<int32_t> post;
        std::vector<int32_t> s{0};
        while (!s.empty()) {
            int32_t n = s.back();
            s.pop_back();
            post.push_back(n);
            if (!bn[n].leaf) {
                s.push_back(bn[n].child[0]);
                s.push_back(bn[n].child[1]);
            }
        }
        for (size_t i = post.size(); i-- > 0;) {
            const int32_t n = post[i];
            const float A = bn[n].box.area();
            splitK[n].fill(0);
            if (bn[n].leaf) {
                rFirst[n] = bn[n].first;
                rCount[n] = bn[n].count;
                cLeaf[n] = kCostTri * A * (float)bn[n].count;
                for (int j = 1; j <= 8; ++j) dist[n][j] = cLeaf[n];
                continue;
            }
            const int32_t L = bn[n].child[0], R = bn[n].child[1];
            rFirst[n] = std::min(rFirst[L], rFirst[R]);
            rCount[n] = rCount[L] + rCount[R];
            if (rCount[n] <= PG_WIDE_LEAF_MAX) cLeaf[n] = kCostTri * A * (float)rCount[n];
            // n opened as a wide node: its children spread over 8 slots
            float best = kInf;
            for (int k = 1; k < 8; ++k) best = std::min(best, dist[L][k] + dist[R][8 - k]);
            cWide[n] = kCostNode * A + best;
            dist[n][1] = std::min(cLeaf[n], cWide[n]);
            for (int j = 2; j <= 8; ++j) {
                dist[n][j] = dist[n][1];
                for (int k = 1; k < j; ++k) {
                    const float c = dist[L][k] + dist[R][j - k];
                    if (c < dist[n][j]) {
                        dist[n][j] = c;
                        splitK[n][j] = (uint8_t)k;
                    }
                }
            }
        }
    }
    // slots of wide node n: children of n spread over 8 slots along the DP's choices
    auto collect = [&](int32_t n, std::vector<int32_t> &out) {
        std::vector<std::pair<int32_t, int>> s;
        int bestK = 1;
        float best = kInf;
        for (int k = 1; k < 8; ++k) {
            const float c = dist[bn[n].child[0]][k] + dist[bn[n].child[1]][8 - k];
            if (c < best) {
                best = c;
                bestK = k;
            }
        }
        s.push_back({bn[n].child[1], 8 - bestK});
        s.push_back({bn[n].child[0], bestK});
        while (!s.empty()) {
            auto [m, j] = s.back();
            s.pop_back();
            const int k = bn[m].leaf ? 0 : splitK[m][j];
            if (k == 0) {
                out.push_back(m);
            } else {
                s.push_back({bn[m].child[1], j - k});
                s.push_back({bn[m].child[0], k});
            }
        }
    };
    // a slot is a leaf when the subtree fits one and a leaf is not costlier than a wide node
    auto isLeafSlot = [&](int32_t m) { return bn[m].leaf || cLeaf[m] <= cWide[m]; };

    struct WTask { int32_t bnode; uint32_t wide; uint32_t depth; };
    std::vector<WTask> work{{0, 0, 1}};
    std::vector<float> nodes(PG_WIDE_NODE_F4 * 4, 0.0f);
    std::vector<uint32_t> order;
    posOf.assign(nt, 0);
    order.reserve(nt);
    uint32_t wideDepth = 0;
    for (size_t w = 0; w < work.size(); ++w) {
        const WTask task = work[w];
        wideDepth = std::max(wideDepth, task.depth);
        std::vector<int32_t> ch;
        if (isLeafSlot(task.bnode)) ch.push_back(task.bnode);  // tiny scene: the root is one leaf
        else collect(task.bnode, ch);
        std::vector<Box> cb;
        Box parent;
        for (int32_t c : ch) {
            cb.push_back(bn[c].box);
            parent.grow(bn[c].box);
        }
        int slotOf[8];
        assignSlots(parent, cb, slotOf);
        int childAt[8];
        for (int sl = 0; sl < 8; ++sl) childAt[sl] = -1;
        for (size_t i = 0; i < ch.size(); ++i) childAt[slotOf[i]] = (int)i;
        // quantisation frame of this node
        int ex[3];
        float scale[3];
        for (int a = 0; a < 3; ++a) {
            ex[a] = quantExponent(parent.hi[a] - parent.lo[a]);
            scale[a] = std::ldexp(1.0f, ex[a]);
        }
        uint32_t imask = 0, childBase = (uint32_t)(nodes.size() / (PG_WIDE_NODE_F4 * 4)),
                 triBase = (uint32_t)order.size(), nInner = 0;
        uint8_t meta[8] = {0}, q[6][8];
        for (int a = 0; a < 6; ++a)
            for (int sl = 0; sl < 8; ++sl) q[a][sl] = 0;
        for (int sl = 0; sl < 8; ++sl) {
            const int i = childAt[sl];
            if (i < 0) continue;
            const int32_t cn = ch[i];
            const BNode &c = bn[cn];
            for (int a = 0; a < 3; ++a) {
                // conservative: floor / ceil in double, then checked against the float reconstruction
                double lo = std::floor(((double)c.box.lo[a] - parent.lo[a]) / scale[a]);
                double hi = std::ceil(((double)c.box.hi[a] - parent.lo[a]) / scale[a]);
                lo = std::max(0.0, std::min(255.0, lo));
                hi = std::max(0.0, std::min(255.0, hi));
                while (lo > 0 && parent.lo[a] + (float)lo * scale[a] > c.box.lo[a]) lo -= 1;
                while (hi < 255 && parent.lo[a] + (float)hi * scale[a] < c.box.hi[a]) hi += 1;
                q[a][sl] = (uint8_t)lo;
                q[3 + a][sl] = (uint8_t)hi;
            }
            if (isLeafSlot(cn)) {
                const uint32_t off = (uint32_t)order.size() - triBase;
                for (uint32_t k = 0; k < rCount[cn]; ++k) {
                    posOf[rFirst[cn] + k] = (uint32_t)order.size();
                    order.push_back(ord[rFirst[cn] + k]);
                }
                meta[sl] = (uint8_t)(off | (rCount[cn] << 5));  // count 1..3 in bits 5-6 (0 = empty slot)
            } else {
                imask |= 1u << sl;
                work.push_back({cn, childBase + nInner, task.depth + 1});
                ++nInner;
            }
        }
        nodes.resize(nodes.size() + (size_t)nInner * PG_WIDE_NODE_F4 * 4, 0.0f);
        float *o = &nodes[(size_t)task.wide * PG_WIDE_NODE_F4 * 4];
        uint32_t w0 = (uint32_t)(ex[0] + 127) | ((uint32_t)(ex[1] + 127) << 8) | ((uint32_t)(ex[2] + 127) << 16) |
                      (imask << 24);
        o[0] = parent.lo[0];
        o[1] = parent.lo[1];
        o[2] = parent.lo[2];
        std::memcpy(&o[3], &w0, 4);
        uint32_t w1[4] = {childBase, triBase, 0, 0};
        std::memcpy(&w1[2], meta, 8);
        std::memcpy(&o[4], w1, 16);
        // [2] qlo.x qlo.y  [3] qlo.z qhi.x  [4] qhi.y qhi.z   (8 bytes each, slot order)
        std::memcpy(&o[8], q[0], 8);
        std::memcpy(&o[10], q[1], 8);
        std::memcpy(&o[12], q[2], 8);
        std::memcpy(&o[14], q[3], 8);
        std::memcpy(&o[16], q[4], 8);
        std::memcpy(&o[18], q[5], 8);
    }
    out.wnodes.swap(nodes);
    out.wide_depth = wideDepth;
    if (wideDepth + 1 > stack_limit || order.size() != nt) return false;
    out.order.swap(order);
    out.tris.assign(4 * (size_t)PG_TRI_F4(nt), 0.0f);
    for (uint32_t k = 0; k < nt; ++k) {
        float rec[12];
        (PG_TRIACCEL ? triAccelRecord : woopRecord)(P, I, out.order[k], rec);
        for (uint32_t r = 0; r < 3; ++r) std::memcpy(&out.tris[4 * (size_t)PG_TRI_ROW(k, r)], rec + 4 * r, 16);
    }
    return true;
}

// binary BVH (for closest-hit queries) over the same tree: nodes whose leaves index the shared
// triangle order (posOf: a binary leaf's triangles lie inside one wide leaf slot, so they stay
// contiguous)
static bool buildBinaryBvh(const std::vector<BNode> &bn, uint32_t maxDepth, const std::vector<uint32_t> &posOf,
                           uint32_t stack_limit, BvhOut &out) {
    out.max_depth = maxDepth;
    if (maxDepth + 1 > stack_limit) return false;
    // ---- pack: the inner nodes of the top PG_BVH_TOP_LEVELS levels first, breadth first (k_trace
    // stages them in LDS), then the rest depth first; a leaf root gets a synthetic parent
    std::vector<int32_t> gpuIndex(bn.size(), -1);
    std::vector<int32_t> innerOrder;
    {
        std::vector<std::pair<int32_t, int>> level{{0, 0}};
        std::vector<int32_t> frontier;  // children below the top levels, left to right
        for (size_t k = 0; k < level.size(); ++k) {
            const auto [n, d] = level[k];
            if (bn[n].leaf) continue;
            if (d >= PG_BVH_TOP_LEVELS) {
                frontier.push_back(n);
                continue;
            }
            gpuIndex[n] = (int32_t)innerOrder.size();
            innerOrder.push_back(n);
            level.push_back({bn[n].child[0], d + 1});
            level.push_back({bn[n].child[1], d + 1});
        }
        out.top_nodes = (uint32_t)innerOrder.size();
        std::vector<int32_t> s(frontier.rbegin(), frontier.rend());
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
        if (bn[n].leaf) return (int32_t)(~((posOf[bn[n].first] << 4) | bn[n].count));
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
        out.top_nodes = 1;
        return true;
    }
    out.nodes.assign(16 * innerOrder.size(), 0.0f);
    for (size_t i = 0; i < innerOrder.size(); ++i) {
        const BNode &n = bn[innerOrder[i]];
        putNode(&out.nodes[16 * i], bn[n.child[0]].box, ref(n.child[0]), bn[n.child[1]].box, ref(n.child[1]));
    }
    return true;
}

// one 4-wide node (pg_layout.h PG_QNODE_*): child boxes box[2a][s] / box[2a+1][s] (lo / hi along axis
// a) of the first `used` slots, refs r[4]; full-precision planes, or (PG_QNODE_QUANT) bytes in the
// node's frame rounded outward as the 8-wide nodes' are
static void putQuadNode(float *o, const float box[6][4], const int32_t r[4], int used) {
#if PG_QNODE_QUANT
    Box parent;
    if (used == 0)
        for (int a = 0; a < 3; ++a) parent.lo[a] = parent.hi[a] = 0.0f;
    for (int s = 0; s < used; ++s)
        for (int a = 0; a < 3; ++a) {
            parent.lo[a] = std::min(parent.lo[a], box[2 * a][s]);
            parent.hi[a] = std::max(parent.hi[a], box[2 * a + 1][s]);
        }
    uint32_t e = 0, w[6] = {0, 0, 0, 0, 0, 0};
    for (int a = 0; a < 3; ++a) {
        const int ex = quantExponent(parent.hi[a] - parent.lo[a]);
        const float scale = std::ldexp(1.0f, ex);
        e |= (uint32_t)(ex + 127) << (8 * a);
        o[a] = parent.lo[a];
        for (int s = 0; s < 4; ++s) {
            double lo = 255, hi = 0;  // empty slot: an inverted box
            if (s < used) {
                lo = std::floor(((double)box[2 * a][s] - parent.lo[a]) / scale);
                hi = std::ceil(((double)box[2 * a + 1][s] - parent.lo[a]) / scale);
                lo = std::max(0.0, std::min(255.0, lo));
                hi = std::max(0.0, std::min(255.0, hi));
                while (lo > 0 && parent.lo[a] + (float)lo * scale > box[2 * a][s]) lo -= 1;
                while (hi < 255 && parent.lo[a] + (float)hi * scale < box[2 * a + 1][s]) hi += 1;
            }
            w[2 * a] |= (uint32_t)lo << (8 * s);
            w[2 * a + 1] |= (uint32_t)hi << (8 * s);
        }
    }
    std::memcpy(&o[3], &e, 4);
    std::memcpy(&o[4], r, 16);
    std::memcpy(&o[8], w, 24);
    o[14] = o[15] = 0.0f;
#else
    (void)used;
    for (int a = 0; a < 6; ++a)
        for (int s = 0; s < 4; ++s) o[4 * a + s] = box[a][s];
    std::memcpy(&o[24], r, 16);
#endif
}

// 4-wide BVH (PG_BVH4, closest hit) over the same tree; its leaves are the binary leaves (same refs).
// Which binary nodes a 4-wide node absorbs is the SAH-optimal choice (the 8-wide collapse's dynamic
// programme with 4 slots and the leaves fixed: it minimises the summed surface area of the opened
// nodes, i.e. the expected node visits); PG_BVH4_GREEDY=1 opens the largest-area inner child
// instead (A/B).  Siblings are stored consecutively, nodes depth first.  Fails if a root-to-leaf walk
// could hold more than PG_QSTACK_DEPTH stack entries (the siblings pushed at every level).
static bool buildQuadBvh(const std::vector<BNode> &bn, const std::vector<uint32_t> &posOf, BvhOut &out) {
    const bool greedy = std::getenv("PG_BVH4_GREEDY") && std::atoi(std::getenv("PG_BVH4_GREEDY")) != 0;
    const size_t nb = bn.size();
    constexpr float kInf = std::numeric_limits<float>::infinity();
    // dist[n][j]: least summed area of opened nodes to spread subtree n over at most j slots
    std::vector<std::array<float, 5>> dist(nb);
    std::vector<std::array<uint8_t, 5>> splitK(nb);
    {
        std::vector<int32_t> post, s{0};
        while (!s.empty()) {
            const int32_t n = s.back();
            s.pop_back();
            post.push_back(n);
            if (!bn[n].leaf) {
                s.push_back(bn[n].child[0]);
                s.push_back(bn[n].child[1]);
            }
        }
        for (size_t i = post.size(); i-- > 0;) {
            const int32_t n = post[i];
            splitK[n].fill(0);
            if (bn[n].leaf) {
                dist[n].fill(0.0f);
                continue;
            }
            const int32_t L = bn[n].child[0], R = bn[n].child[1];
            float best = kInf;
            for (int k = 1; k < 4; ++k) best = std::min(best, dist[L][k] + dist[R][4 - k]);
            dist[n][1] = bn[n].box.area() + best;  // n as one slot: an opened 4-wide node
            for (int j = 2; j <= 4; ++j) {
                dist[n][j] = dist[n][1];
                for (int k = 1; k < j; ++k) {
                    const float c = dist[L][k] + dist[R][j - k];
                    if (c < dist[n][j]) {
                        dist[n][j] = c;
                        splitK[n][j] = (uint8_t)k;
                    }
                }
            }
        }
    }
    // the slots of opened node n along the programme's choices
    auto collect = [&](int32_t n, std::vector<int32_t> &ch) {
        int bestK = 1;
        float best = kInf;
        for (int k = 1; k < 4; ++k) {
            const float c = dist[bn[n].child[0]][k] + dist[bn[n].child[1]][4 - k];
            if (c < best) {
                best = c;
                bestK = k;
            }
        }
        std::vector<std::pair<int32_t, int>> s{{bn[n].child[1], 4 - bestK}, {bn[n].child[0], bestK}};
        while (!s.empty()) {
            auto [m, j] = s.back();
            s.pop_back();
            const int k = bn[m].leaf ? 0 : splitK[m][j];
            if (k == 0) {
                ch.push_back(m);
            } else {
                s.push_back({bn[m].child[1], j - k});
                s.push_back({bn[m].child[0], k});
            }
        }
    };
    auto ref = [&](int32_t n, int32_t inner) -> int32_t {
        if (bn[n].leaf) return (int32_t)(~((posOf[bn[n].first] << 4) | bn[n].count));
        return inner;
    };
    struct QTask { int32_t bnode; uint32_t qnode; uint32_t stackNeed; };
    std::vector<float> nodes;
    std::vector<QTask> st;
    uint32_t maxNeed = 0;
    auto alloc = [&]() {
        const uint32_t q = (uint32_t)(nodes.size() / (4 * PG_QNODE_F4));
        nodes.resize(nodes.size() + 4 * PG_QNODE_F4, 0.0f);
        return q;
    };
    out.top_nodes = 0;  // set below: the 4-wide nodes of the breadth-first top levels
    if (bn[0].leaf) {  // the root is a leaf: one node with one leaf slot
        out.top_nodes = 1;
        const uint32_t q = alloc();
        float *o = &nodes[(size_t)q * 4 * PG_QNODE_F4];
        int32_t r[4] = {ref(0, 0), PG_QNODE_EMPTY, PG_QNODE_EMPTY, PG_QNODE_EMPTY};
        float box[6][4] = {};
        for (int a = 0; a < 3; ++a) {
            box[2 * a][0] = bn[0].box.lo[a];
            box[2 * a + 1][0] = bn[0].box.hi[a];
        }
        putQuadNode(o, box, r, 1);
        out.nodes.swap(nodes);
        return true;
    }
    // the top PG_BVH4_TOP_LEVELS levels' nodes are processed breadth first, so their children -- the
    // nodes of depths <= PG_BVH4_TOP_LEVELS -- take the first indices (k_rays' LDS tile); the rest depth
    // first.  Node contents and refs do not depend on the order: walks return the same hits.
    std::vector<QTask> bfs{{0, alloc(), 1}};
    std::vector<uint32_t> depthOf{0};
    size_t head = 0;
    auto depth = [&](uint32_t q) { return q < depthOf.size() ? depthOf[q] : 0xFFFFFFFFu; };
    while (true) {
        QTask t;
        if (head < bfs.size()) {
            t = bfs[head++];
        } else if (!st.empty()) {
            t = st.back();
            st.pop_back();
        } else {
            break;
        }
        const uint32_t td = depth(t.qnode);
        std::vector<int32_t> ch;
        if (!greedy) collect(t.bnode, ch);
        else ch = {bn[t.bnode].child[0], bn[t.bnode].child[1]};
        while (greedy && ch.size() < 4) {
            int best = -1;
            float bestA = -1.0f;
            for (size_t i = 0; i < ch.size(); ++i)
                if (!bn[ch[i]].leaf && bn[ch[i]].box.area() > bestA) {
                    bestA = bn[ch[i]].box.area();
                    best = (int)i;
                }
            if (best < 0) break;
            const int32_t m = ch[best];
            ch[best] = bn[m].child[0];
            ch.insert(ch.begin() + best + 1, bn[m].child[1]);
        }
        const uint32_t need = t.stackNeed + (uint32_t)ch.size() - 1;
        maxNeed = std::max(maxNeed, need);
        int32_t r[4] = {PG_QNODE_EMPTY, PG_QNODE_EMPTY, PG_QNODE_EMPTY, PG_QNODE_EMPTY};
        float box[6][4];
        for (int a = 0; a < 6; ++a)
            for (int s = 0; s < 4; ++s) box[a][s] = 0.0f;
        for (size_t s = 0; s < ch.size(); ++s) {
            const BNode &c = bn[ch[s]];
            for (int a = 0; a < 3; ++a) {
                box[2 * a][s] = c.box.lo[a];
                box[2 * a + 1][s] = c.box.hi[a];
            }
            if (c.leaf) {
                r[s] = ref(ch[s], 0);
            } else {
                const uint32_t q = alloc();
                r[s] = (int32_t)q;
                if (td != 0xFFFFFFFFu && td + 1 < (uint32_t)PG_BVH4_TOP_LEVELS) {  // breadth-first top levels
                    depthOf.resize(q + 1, 0xFFFFFFFFu);
                    depthOf[q] = td + 1;
                    bfs.push_back({ch[s], q, need});
                } else {
                    st.push_back({ch[s], q, need});
                }
            }
        }
        float *o = &nodes[(size_t)t.qnode * 4 * PG_QNODE_F4];
        putQuadNode(o, box, r, (int)ch.size());
        if (head == bfs.size() && out.top_nodes == 0) out.top_nodes = (uint32_t)(nodes.size() / (4 * PG_QNODE_F4));
    }
    out.nodes.swap(nodes);
    return maxNeed <= PG_QSTACK_DEPTH;
}

bool buildBvh(const float *P, const uint32_t *I, uint32_t nt, uint32_t stack_limit, BvhOut &out) {
    if (nt == 0) {  // every ray misses: an inner root with two empty far-away leaves; a childless wide node
        out.nodes.assign(16, 0.0f);
        for (int k = 0; k < 4; ++k) out.nodes[k] = out.nodes[4 + k] = 1e30f;
        out.nodes[8] = out.nodes[9] = out.nodes[10] = out.nodes[11] = 1e30f;
        int32_t empty = ~(int32_t)0;
        std::memcpy(&out.nodes[12], &empty, 4);
        std::memcpy(&out.nodes[13], &empty, 4);
        if (PG_BVH4) {  // one node without children
            out.nodes.assign(4 * PG_QNODE_F4, 0.0f);
            const int32_t r[4] = {PG_QNODE_EMPTY, PG_QNODE_EMPTY, PG_QNODE_EMPTY, PG_QNODE_EMPTY};
            const float box[6][4] = {};
            putQuadNode(out.nodes.data(), box, r, 0);
        }
        out.wnodes.assign(PG_WIDE_NODE_F4 * 4, 0.0f);
        out.order.clear();
        out.tris.clear();
        out.max_depth = out.wide_depth = 1;
        out.top_nodes = 1;
        for (int a = 0; a < 3; ++a) out.lo[a] = out.hi[a] = 0.0f;
        return true;
    }
    // one binary build (leaves <= PG_WIDE_LEAF_MAX triangles) serves both BVHs, and both walk one
    // triangle array in one order (the L2 of an XCD then holds one copy of the triangles)
    std::vector<BNode> bn;
    std::vector<uint32_t> ord, posOf;
    uint32_t maxDepth = 0;
    Box all;
    buildBinary(P, I, nt, PG_WIDE_LEAF_MAX, bn, ord, maxDepth, all);
    for (int a = 0; a < 3; ++a) {
        out.lo[a] = all.lo[a];
        out.hi[a] = all.hi[a];
    }
    if (!buildWide(P, I, nt, stack_limit, bn, ord, out, posOf)) return false;
    if (PG_BVH4) {
        out.max_depth = maxDepth;
        return buildQuadBvh(bn, posOf, out);
    }
    return buildBinaryBvh(bn, maxDepth, posOf, stack_limit, out);
}

}  // namespace pgh
