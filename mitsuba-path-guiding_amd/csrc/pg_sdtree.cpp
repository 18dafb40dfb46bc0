// SD-tree host refit + wire format (see pg_sdtree.h and DESIGN.md §"SD-tree").
#include "pg_sdtree.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace pgh {
namespace {

constexpr uint32_t kMagic = 0x44534750u;  // 'PGSD'
constexpr uint32_t kLeafMark = 0xFFFFFFFFu;

inline float fixedToFloat(uint64_t x) { return (float)std::ldexp((double)x, -24); }

// f(i) for i in [0, n) on up to 16 host threads, in blocks of 8 leaves.  Every D-tree is refit,
// rebuilt and flattened independently of the others, so the result does not depend on the split.
// The workers persist across calls (a refit makes four parallel passes; spawning 15 threads per pass
// cost ~1 ms); a caller that finds the pool busy (another context refitting concurrently) runs inline.
class Pool {
public:
    static Pool &get() {
        static Pool p;
        return p;
    }
    template <class F>
    bool run(size_t n, size_t threads, F &f) {
        std::unique_lock<std::mutex> own(use_, std::try_to_lock);
        if (!own.owns_lock()) return false;
        {
            std::lock_guard<std::mutex> lk(m_);
            while (workers_.size() + 1 < threads) workers_.emplace_back([this] { loop(); });
            job_ = [&f](size_t i) { f(i); };
            n_ = n;
            next_.store(0);
            active_ = std::min(threads, workers_.size() + 1) - 1;
            pending_ = active_;
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
        return true;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }

private:
    void work() {
        for (size_t b; (b = next_.fetch_add(8)) < n_;)
            for (size_t i = b, e = std::min(n_, b + 8); i < e; ++i) job_(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return stop_ || (gen_ != seen && active_ > 0); });
            if (stop_) return;
            seen = gen_;
            --active_;  // this worker takes part in generation gen_
            lk.unlock();
            work();
            lk.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex use_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    std::function<void(size_t)> job_;
    std::atomic<size_t> next_{0};
    size_t n_ = 0, active_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

template <class F>
void parallelFor(size_t n, F &&f) {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t T = std::min<size_t>(std::min(hw, 16u), (n + 63) / 64);
    if (T <= 1 || !Pool::get().run(n, T, f))
        for (size_t i = 0; i < n; ++i) f(i);
}
inline float total4(const float *s) { return ((s[0] + s[1]) + s[2]) + s[3]; }

// bottom-up quadrant sums of a building tree (integer, exact below 2^64; saturating above, as the
// oracle's buildSums: a D-tree's total is the sum of all its records over every rank)
uint64_t propagate(std::vector<SdNodeB> &b, uint32_t n) {
    uint64_t tot = 0;
    for (int q = 0; q < 4; ++q) {
        if (b[n].child[q]) b[n].sum[q] = propagate(b, b[n].child[q]);
        tot = (tot + b[n].sum[q] < tot) ? ~0ull : tot + b[n].sum[q];
    }
    return tot;
}

// New building topology: refine every quadrant of the (just built) tree whose energy fraction
// exceeds rho, below max_depth; quadrants of leaves keep refining with sum/4 estimates.
void rebuildTopology(SdLeaf &L, int maxDepth, float rho) {
    struct Tmp { float s[4]; uint32_t c[4]; };
    struct Item { uint32_t dst; uint32_t src; bool prev; int depth; };
    // per-thread scratch reused across leaves (no allocation per D-tree)
    thread_local std::vector<Tmp> nodes;
    thread_local std::vector<Item> stack;
    nodes.assign(1, Tmp{{0, 0, 0, 0}, {0, 0, 0, 0}});
    stack.assign(1, Item{0, 0, true, 1});
    const float total = L.total;
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        float ss[4];
        uint32_t sc[4];
        if (it.prev) {
            for (int q = 0; q < 4; ++q) {
                ss[q] = L.sampling[it.src].sum[q];
                sc[q] = L.sampling[it.src].child[q];
            }
        } else {
            for (int q = 0; q < 4; ++q) {
                ss[q] = nodes[it.src].s[q];
                sc[q] = 0;
            }
        }
        for (int q = 0; q < 4; ++q) {
            float frac = total > 0 ? (ss[q] / total) : std::pow(0.25f, (float)it.depth);
            if (!(it.depth < maxDepth && frac > rho)) continue;
            uint32_t c = (uint32_t)nodes.size();
            nodes[it.dst].c[q] = c;
            Tmp t;
            for (int k = 0; k < 4; ++k) {
                t.s[k] = ss[q] / 4;
                t.c[k] = 0;
            }
            nodes.push_back(t);
            if (it.prev && sc[q]) stack.push_back({c, sc[q], true, it.depth + 1});
            else stack.push_back({c, c, false, it.depth + 1});
        }
    }
    L.building.assign(nodes.size(), SdNodeB{});
    for (size_t i = 0; i < nodes.size(); ++i)
        for (int q = 0; q < 4; ++q) L.building[i].child[q] = nodes[i].c[q];
    L.count = 0;
    for (uint64_t &f : L.frac) f = 0;
}

}  // namespace

void SdTree::reset(const float bmin[3], const float bmax[3]) {
    float m = std::max(bmax[0] - bmin[0], std::max(bmax[1] - bmin[1], bmax[2] - bmin[2]));
    for (int a = 0; a < 3; ++a) lo[a] = bmin[a];
    extent = m;
    snode = {kLeafMark, 0u};
    leaves.assign(1, SdLeaf{});
    built = false;
}

void SdTree::refit(uint32_t iteration, float sThreshold, float rho, int maxDepth, bool learn) {
    // 1. build: building -> sampling (fp32 from the exact integer sums); the learned fraction: the
    //    candidate of the largest cross-entropy estimate (ties: the larger fraction) when the leaf saw
    //    enough guided records (pg_device.h fracStat; oracle SDTree::learnedFraction)
    parallelFor(leaves.size(), [&](size_t li) {
        SdLeaf &L = leaves[li];
        if (learn && L.frac[kFracCandidates] >= kFracMinRecords) {
            int best = 0;
            for (int k = 1; k < kFracCandidates; ++k)
                if ((int64_t)L.frac[k] >= (int64_t)L.frac[best]) best = k;
            L.alpha = fracCandidate(best);
        }
        propagate(L.building, 0);
        L.sampling.assign(L.building.size(), SdNodeS{});
        for (size_t i = 0; i < L.building.size(); ++i)
            for (int q = 0; q < 4; ++q) {
                L.sampling[i].sum[q] = fixedToFloat(L.building[i].sum[q]);
                L.sampling[i].child[q] = L.building[i].child[q];
            }
        L.total = total4(L.sampling[0].sum);
    });
    // 2. refine the S-tree: split leaves whose record count exceeds c * sqrt(2^k); children copy
    //    the D-trees and halve the count; recursion continues into the children (DFS, child0 first)
    const double thr = (double)sThreshold * std::sqrt(std::pow(2.0, (double)iteration));
    std::vector<uint32_t> stack{0};
    while (!stack.empty()) {
        uint32_t n = stack.back();
        stack.pop_back();
        if (snode[2 * n] == kLeafMark && (double)leaves[snode[2 * n + 1]].count > thr) {
            uint32_t l0 = snode[2 * n + 1];
            leaves[l0].count /= 2;
            uint32_t l1 = (uint32_t)leaves.size();
            leaves.push_back(leaves[l0]);
            uint32_t c0 = (uint32_t)(snode.size() / 2);
            snode.push_back(kLeafMark);
            snode.push_back(l0);
            snode.push_back(kLeafMark);
            snode.push_back(l1);
            snode[2 * n] = c0;
            snode[2 * n + 1] = c0 + 1;
        }
        if (snode[2 * n] != kLeafMark) {
            stack.push_back(snode[2 * n + 1]);
            stack.push_back(snode[2 * n]);
        }
    }
    // 3. reset the building trees
    parallelFor(leaves.size(), [&](size_t li) { rebuildTopology(leaves[li], maxDepth, rho); });
    built = true;
}

size_t SdTree::samplingNodes() const {
    size_t n = 0;
    for (auto &L : leaves) n += L.sampling.size();
    return n;
}
size_t SdTree::buildingNodes() const {
    size_t n = 0;
    for (auto &L : leaves) n += L.building.size();
    return n;
}

// Jump grid for the device lookup: cell (x, y, z) of a 2^k grid -> the S-tree node reached after
// following the cell's bits for 3k axis-cycling levels (or the leaf met on the way).
static void fillJump(const std::vector<uint32_t> &sn, uint32_t node, int depth, int k, uint32_t x0, uint32_t y0,
                     uint32_t z0, uint32_t sx, uint32_t sy, uint32_t sz, uint32_t *jump) {
    const uint32_t R = 1u << k;
    if (sn[2 * node] == kLeafMark || depth == 3 * k) {
        // k_sd_jump's encoding: a leaf's cells hold its D-tree id, flagged
        const uint32_t v = sn[2 * node] == kLeafMark ? (0x80000000u | sn[2 * node + 1]) : node;
        for (uint32_t z = z0; z < z0 + sz; ++z)
            for (uint32_t y = y0; y < y0 + sy; ++y)
                for (uint32_t x = x0; x < x0 + sx; ++x) jump[((size_t)z * R + y) * R + x] = v;
        return;
    }
    const int axis = depth % 3;
    uint32_t c0 = sn[2 * node], c1 = sn[2 * node + 1];
    if (axis == 0) {
        fillJump(sn, c0, depth + 1, k, x0, y0, z0, sx / 2, sy, sz, jump);
        fillJump(sn, c1, depth + 1, k, x0 + sx / 2, y0, z0, sx / 2, sy, sz, jump);
    } else if (axis == 1) {
        fillJump(sn, c0, depth + 1, k, x0, y0, z0, sx, sy / 2, sz, jump);
        fillJump(sn, c1, depth + 1, k, x0, y0 + sy / 2, z0, sx, sy / 2, sz, jump);
    } else {
        fillJump(sn, c0, depth + 1, k, x0, y0, z0, sx, sy, sz / 2, jump);
        fillJump(sn, c1, depth + 1, k, x0, y0, z0 + sz / 2, sx, sy, sz / 2, jump);
    }
}

void SdTree::flattenInto(const Layout &d) const {
    std::memcpy(d.snodes, snode.data(), 4 * snode.size());
    const uint32_t R = 1u << kJumpBits;
    if (d.jump) fillJump(snode, 0, 0, kJumpBits, 0, 0, 0, R, R, R, d.jump);  // nullptr: built on the device
    std::vector<uint32_t> sbase(leaves.size()), bbase(leaves.size());
    for (size_t i = 0, sb = 0, bb = 0; i < leaves.size(); ++i) {
        sbase[i] = (uint32_t)sb;
        bbase[i] = (uint32_t)bb;
        sb += leaves[i].sampling.size();
        bb += leaves[i].building.size();
    }
    parallelFor(leaves.size(), [&](size_t i) {
        const SdLeaf &L = leaves[i];
        const uint32_t sb = sbase[i], bb = bbase[i];
        d.meta[4 * i + 0] = sb;
        d.meta[4 * i + 1] = bb;
        std::memcpy(&d.meta[4 * i + 2], &L.alpha, 4);
        std::memcpy(&d.meta[4 * i + 3], &L.total, 4);
        for (int k = 0; k < kFracStats; ++k) d.frac[(size_t)kFracStats * i + k] = L.frac[k];
        for (size_t k = 0; k < L.sampling.size(); ++k) {
            uint32_t *q = d.qnode + 8 * (sb + k);
            std::memcpy(q, L.sampling[k].sum, 16);
            for (int j = 0; j < 4; ++j) q[4 + j] = L.sampling[k].child[j] ? L.sampling[k].child[j] + sb : 0;
        }
        for (size_t k = 0; k < L.building.size(); ++k)
            for (int q = 0; q < 4; ++q) {
                d.bchild[4 * (bb + k) + q] = L.building[k].child[q] ? L.building[k].child[q] + bb : 0;
                d.bsum[4 * (bb + k) + q] = L.building[k].sum[q];
            }
        d.count[i] = L.count;
    });
}

void SdTree::flatten(Flat &f) const {
    const size_t R = (size_t)1 << kJumpBits;
    f.snodes.resize(snode.size());
    f.meta.resize(4 * leaves.size());
    f.qnode.resize(8 * samplingNodes());
    f.bchild.resize(4 * buildingNodes());
    f.bsum.resize(4 * buildingNodes());
    f.count.resize(leaves.size());
    f.jump.resize(R * R * R);
    f.frac.resize((size_t)kFracStats * leaves.size());
    flattenInto(Layout{f.snodes.data(), f.meta.data(), f.qnode.data(), f.bchild.data(), f.bsum.data(), f.count.data(),
                       f.jump.data(), f.frac.data()});
}

void SdTree::absorb(const uint64_t *bsum, const uint32_t *count, const uint64_t *frac) {
    std::vector<size_t> bbase(leaves.size());
    for (size_t i = 0, bb = 0; i < leaves.size(); ++i) {
        bbase[i] = bb;
        bb += leaves[i].building.size();
    }
    parallelFor(leaves.size(), [&](size_t i) {
        SdLeaf &L = leaves[i];
        for (size_t k = 0; k < L.building.size(); ++k)
            for (int q = 0; q < 4; ++q) L.building[k].sum[q] = bsum[4 * (bbase[i] + k) + q];
        L.count = count[i];
        for (int k = 0; k < kFracStats; ++k) L.frac[k] = frac[(size_t)kFracStats * i + k];
    });
}

// Wire format (little endian), shared with the oracle's golden vectors:
//   u32 magic 'PGSD', u32 version 2, u32 built, u32 0
//   f32 lo.xyz, 0, hi.xyz, 0            (cube)
//   u32 num_snodes, num_dtrees, num_sampling_nodes, num_building_nodes
//   num_snodes x {u32 child0, u32 child1}
//   num_dtrees x {u32 sampling_base, building_base, sampling_count, building_count, f32 total, u32 count,
//                 f32 alpha (learned BSDF-sampling fraction, 0 = none), 0}
//   sampling nodes x {f32 sum[4], u32 child[4] (absolute, 0 = leaf)}
//   building nodes x {u64 sum[4], u32 child[4] (absolute, 0 = leaf)}
//   num_dtrees x {u64 frac[kFracStats]}  (learned-fraction building statistics)
std::vector<uint8_t> SdTree::serialize() const {
    std::vector<uint8_t> out;
    auto put = [&](const void *p, size_t n) {
        const uint8_t *b = (const uint8_t *)p;
        out.insert(out.end(), b, b + n);
    };
    uint32_t hdr[4] = {kMagic, 2u, built ? 1u : 0u, 0u};
    put(hdr, 16);
    float box[8] = {lo[0], lo[1], lo[2], extent, lo[0] + extent, lo[1] + extent, lo[2] + extent, 0};
    put(box, 32);
    Flat f;
    flatten(f);
    uint32_t cnt[4] = {(uint32_t)(snode.size() / 2), (uint32_t)leaves.size(), (uint32_t)(f.qnode.size() / 8),
                       (uint32_t)(f.bchild.size() / 4)};
    put(cnt, 16);
    put(snode.data(), 4 * snode.size());
    for (size_t i = 0; i < leaves.size(); ++i) {
        uint32_t m[8] = {f.meta[4 * i], f.meta[4 * i + 1], (uint32_t)leaves[i].sampling.size(),
                         (uint32_t)leaves[i].building.size(), f.meta[4 * i + 3], leaves[i].count, f.meta[4 * i + 2], 0};
        put(m, 32);
    }
    put(f.qnode.data(), 4 * f.qnode.size());  // {f32 sum[4], u32 child[4]} per node
    for (size_t k = 0; k < f.bchild.size() / 4; ++k) {
        put(&f.bsum[4 * k], 32);
        put(&f.bchild[4 * k], 16);
    }
    put(f.frac.data(), 8 * f.frac.size());
    return out;
}

bool SdTree::deserialize(const uint8_t *p, size_t n) {
    size_t off = 0;
    auto get = [&](void *d, size_t k) {
        if (off + k > n) return false;
        std::memcpy(d, p + off, k);
        off += k;
        return true;
    };
    uint32_t hdr[4], cnt[4];
    float box[8];
    if (!get(hdr, 16) || hdr[0] != kMagic || hdr[1] != 2 || !get(box, 32) || !get(cnt, 16)) return false;
    built = hdr[2] != 0;
    for (int a = 0; a < 3; ++a) lo[a] = box[a];
    extent = box[3];
    snode.assign(2 * (size_t)cnt[0], 0);
    if (!get(snode.data(), 8 * (size_t)cnt[0])) return false;
    leaves.assign(cnt[1], SdLeaf{});
    std::vector<uint32_t> sb(cnt[1]), bb(cnt[1]);
    for (uint32_t i = 0; i < cnt[1]; ++i) {
        uint32_t m[8];
        if (!get(m, 32)) return false;
        sb[i] = m[0];
        bb[i] = m[1];
        leaves[i].sampling.assign(m[2], SdNodeS{});
        leaves[i].building.assign(m[3], SdNodeB{});
        std::memcpy(&leaves[i].total, &m[4], 4);
        leaves[i].count = m[5];
        std::memcpy(&leaves[i].alpha, &m[6], 4);
    }
    for (uint32_t i = 0; i < cnt[1]; ++i)
        for (auto &nd : leaves[i].sampling) {
            if (!get(nd.sum, 16) || !get(nd.child, 16)) return false;
            for (int q = 0; q < 4; ++q)
                if (nd.child[q]) nd.child[q] -= sb[i];
        }
    for (uint32_t i = 0; i < cnt[1]; ++i)
        for (auto &nd : leaves[i].building) {
            if (!get(nd.sum, 32) || !get(nd.child, 16)) return false;
            for (int q = 0; q < 4; ++q)
                if (nd.child[q]) nd.child[q] -= bb[i];
        }
    for (uint32_t i = 0; i < cnt[1]; ++i)
        if (!get(leaves[i].frac, 8 * kFracStats)) return false;
    return off == n;
}

}  // namespace pgh
