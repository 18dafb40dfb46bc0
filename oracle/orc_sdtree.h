// ORACLE — test infrastructure only.  CPU restatement of the SD-tree of Mueller, Gross, Novak,
// "Practical Path Guiding for Efficient Light-Transport Simulation" (EGSR 2017) — the guiding
// data structure the fork's scaffolding is built for but which is ABSENT from the
// reference snapshot.  PARITY UNPINNED: no reference test or fixture covers it; the spec below
// (DESIGN.md "SD-tree") is restated from the paper and both this oracle and the HIP path follow it.
//
// Hook points in the reference: postprogression (src/librender/progressiveintegrator.cpp:314-317)
// runs splat + refit; RadianceQueryRecord::pixelId (include/mitsuba/render/integrator.h:313-317).
//
//  * S-tree: binary tree over the scene AABB enlarged to a cube; axis = depth % 3; midpoint splits.
//    After iteration k a leaf splits when its record count > c * sqrt(2^k) (c = sTreeThreshold);
//    both children copy the leaf's D-trees and get half its count (integer halving).
//  * D-tree: quadtree over the cylindrical square (u = (cos theta + 1)/2, v = phi / 2pi), node =
//    4 quadrant energies + 4 child links (0 = leaf).  Records add radiance/woPdf into the leaf
//    quadrant of the building tree as 2^-24 fixed point (u64, order-independent => bit-identical
//    across devices/ranks).  Build: sums propagate bottom-up; sampling tree := building tree (fp32).
//    Reset: new building topology refining every quadrant whose energy fraction > rho (depth < max);
//    sums cleared.  Sampling descends quadrants proportional to energy; pdf = prod 4 E_q / E_node / 4pi.
#pragma once
#include <mutex>
#include <vector>

#include "orc_math.h"

namespace orc {

constexpr float kFixedScale = 16777216.0f;  // 2^24
// per-record cap of the fixed-point value, 2^48 (radiance / woPdf <= 2^24).  A leaf quadrant's u64 sum
// (device atomics, all records and ranks of one iteration) wraps only past 2^40 value units, e.g. 2^16
// records at the cap; interior sums saturate instead of wrapping (buildSums)
constexpr float kSplatCap = 281474976710656.0f;
constexpr uint32_t kSdMagic = 0x44534750u;    // 'PGSD'

struct SNode {
    uint32_t child[2];  // child[0] == 0xFFFFFFFF -> leaf, child[1] = dtree index
    bool leaf() const { return child[0] == 0xFFFFFFFFu; }
};
struct QNode {  // sampling node
    float sum[4] = {0, 0, 0, 0};
    uint32_t child[4] = {0, 0, 0, 0};
};
struct BNode {  // building node
    uint64_t sum[4] = {0, 0, 0, 0};
    uint32_t child[4] = {0, 0, 0, 0};
};
// ---- learned BSDF-sampling fraction per S-tree leaf (PG_FRACTION_LEARNED; kernels: pg_device.h
// fracStat, k_splat, pg_sdtree.cpp refit).  After Mueller 2019 ("Practical Path Guiding in
// Production": the selection probability optimised per spatial cell against the KL divergence from
// f * L_i), restated as a batch choice: every training iteration estimates the cross-entropy
// E_{p*}[log2 q_k] of the candidate mixtures q_k = a_k p_bsdf + (1 - a_k) p_guide, a_k = 0.05 + 0.1 k,
// from its guided records with importance weights w = f L_i / q0, as 2^-16 fixed-point sums; the
// refit keeps the candidate with the largest sum (ties: the larger fraction) once a leaf has 64 guided
// records.  No libm: pgLog2 is a fixed polynomial, bit-identical with the device.
constexpr int kFracCandidates = 10;
constexpr int kFracStats = kFracCandidates + 1;
constexpr uint64_t kFracMinRecords = 64;
constexpr float kFracFixedScale = 65536.0f;
constexpr float kFracCap = 70368744177664.0f;  // 2^46
inline float fracCandidate(int k) { return 0.05f + 0.1f * (float)k; }
inline float pgLog2(float x) {
    if (!(x > 1.17549435e-38f)) return -126.0f;
    uint32_t b;
    std::memcpy(&b, &x, 4);
    const float e = (float)((int)((b >> 23) & 0xFFu) - 127);
    const uint32_t mb = (b & 0x7FFFFFu) | 0x3F800000u;
    float m;
    std::memcpy(&m, &mb, 4);
    const float t = (m - 1.0f) / (m + 1.0f), t2 = t * t;
    const float s = t * (1.0f + t2 * (0.333333343f + t2 * (0.2f + t2 * (0.142857149f + t2 * 0.111111112f))));
    return e + s * 2.88539004f;
}
inline uint64_t fracStat(float w, float pb, float pg, float q0, int k) {
    const float a = fracCandidate(k);
    const float qk = a * pb + (1.0f - a) * pg;
    float v = w * pgLog2(qk / q0) * kFracFixedScale;
    if (v > kFracCap) v = kFracCap;
    if (v < -kFracCap) v = -kFracCap;
    return (uint64_t)(int64_t)v;
}

struct DTreeW {
    std::vector<QNode> sampling{QNode{}};
    float samplingTotal = 0;
    float alpha = 0;  // learned fraction (0: not learned, pg_config.bsdf_sampling_fraction)
    std::vector<BNode> building{BNode{}};
    uint32_t count = 0;
    uint64_t frac[kFracStats] = {};
};

inline void dirToCanonical(V3 d, float &u, float &v) {
    float cosTheta = std::min(std::max(d.z, -1.0f), 1.0f);
    float phi = std::atan2(d.y, d.x);
    if (phi < 0) phi += 2 * kPi;
    u = (cosTheta + 1) * 0.5f;
    v = phi * (1.0f / (2 * kPi));
    if (!(u >= 0)) u = 0;
    if (!(u < 1)) u = 0.99999994f;
    if (!(v >= 0)) v = 0;
    if (!(v < 1)) v = 0.99999994f;
}
inline V3 canonicalToDir(float u, float v) {
    float cosTheta = 2 * u - 1;
    float phi = 2 * kPi * v;
    float sinTheta = safe_sqrt(1 - cosTheta * cosTheta);
    return {sinTheta * std::cos(phi), sinTheta * std::sin(phi), cosTheta};
}
inline uint32_t packCanonical(float u, float v) {
    uint32_t a = std::min<uint32_t>(65535u, (uint32_t)(u * 65536.0f));
    uint32_t b = std::min<uint32_t>(65535u, (uint32_t)(v * 65536.0f));
    return a | (b << 16);
}
inline void unpackCanonical(uint32_t w, float &u, float &v) {
    u = ((float)(w & 0xFFFFu) + 0.5f) * (1.0f / 65536.0f);
    v = ((float)(w >> 16) + 0.5f) * (1.0f / 65536.0f);
}
// quadrant of p in the unit square, rescaling p into the child's square
inline int childIndex(float &u, float &v) {
    int q = 0;
    if (u >= 0.5f) { q |= 1; u = u * 2 - 1; } else { u = u * 2; }
    if (v >= 0.5f) { q |= 2; v = v * 2 - 1; } else { v = v * 2; }
    return q;
}
inline float nodeTotal(const float *s) { return ((s[0] + s[1]) + s[2]) + s[3]; }

struct SDTree {
    V3 lo, hi;  // cube: hi = lo + extent
    float extent = 1;
    std::vector<SNode> snodes{SNode{{0xFFFFFFFFu, 0u}}};
    std::vector<DTreeW> dtrees{DTreeW{}};
    bool built = false;
    std::mutex mtx;
    std::vector<pg_record> pending;

    void init(V3 bmin, V3 bmax) {
        V3 size = bmax - bmin;
        float m = std::max(size.x, std::max(size.y, size.z));
        lo = bmin;
        extent = m;
        hi = bmin + V3(m);
        snodes.assign(1, SNode{{0xFFFFFFFFu, 0u}});
        dtrees.assign(1, DTreeW{});  // one S-tree leaf, D-trees = a single root node
        built = false;
    }

    uint32_t lookup(V3 p) const {
        float q[3];
        for (int a = 0; a < 3; ++a) {
            float x = (p[a] - lo[a]) / extent;
            q[a] = std::min(std::max(x, 0.0f), 1.0f);
        }
        uint32_t n = 0;
        int depth = 0;
        while (!snodes[n].leaf()) {
            int ax = depth % 3;
            if (q[ax] < 0.5f) {
                q[ax] = q[ax] * 2;
                n = snodes[n].child[0];
            } else {
                q[ax] = q[ax] * 2 - 1;
                n = snodes[n].child[1];
            }
            ++depth;
        }
        return snodes[n].child[1];
    }

    // ---- sampling-tree queries (pdf w.r.t. solid angle)
    static float pdfDir(const DTreeW &dt, V3 d) {
        if (!(dt.samplingTotal > 0)) return kInvFourPi;
        float u, v;
        dirToCanonical(d, u, v);
        return pdfCanon(dt, u, v);
    }
    // pdf = prod_l 4 E_q(l) / E_node(l) / 4pi, telescoped to 4^d E_leafquadrant / E_root / 4pi
    static float telescopedPdf(float leafEnergy, float rootTotal, int depth) {
        if (!(leafEnergy > 0)) return 0.0f;
        return std::ldexp(leafEnergy / rootTotal, 2 * depth) * kInvFourPi;
    }
    static float pdfCanon(const DTreeW &dt, float u, float v) {
        if (!(dt.samplingTotal > 0)) return kInvFourPi;
        uint32_t n = 0;
        int depth = 1;
        for (;;) {
            const QNode &nd = dt.sampling[n];
            int q = childIndex(u, v);
            if (nd.child[q] == 0) return telescopedPdf(nd.sum[q], dt.samplingTotal, depth);
            n = nd.child[q];
            ++depth;
        }
    }
    // returns world direction; pdf computed along the sampled path
    static V3 sampleDir(const DTreeW &dt, float u, float v, float &pdf) {
        float cu, cv;
        sampleCanon(dt, u, v, cu, cv, pdf);
        return canonicalToDir(cu, cv);
    }
    static void sampleCanon(const DTreeW &dt, float px, float py, float &cu, float &cv, float &pdf) {
        if (!(dt.samplingTotal > 0)) {
            cu = px;
            cv = py;
            pdf = kInvFourPi;
            return;
        }
        uint32_t n = 0;
        float ox = 0, oy = 0, scale = 1;
        int depth = 0;
        float parentEnergy = dt.samplingTotal;
        for (;;) {
            const QNode &nd = dt.sampling[n];
            float total = nodeTotal(nd.sum);
            if (!(total > 0)) {  // degenerate node: uniform inside it
                cu = ox + scale * px;
                cv = oy + scale * py;
                pdf = telescopedPdf(parentEnergy, dt.samplingTotal, depth);
                return;
            }
            float partial = nd.sum[0] + nd.sum[2];
            float boundary = partial / total;
            int q = 0;
            float qx = 0, qy = 0;
            if (px < boundary) {
                px = px / boundary;
                boundary = nd.sum[0] / partial;
            } else {
                partial = total - partial;
                qx = 0.5f;
                px = (px - boundary) / (1.0f - boundary);
                boundary = nd.sum[1] / partial;
                q |= 1;
            }
            if (py < boundary) {
                py = py / boundary;
            } else {
                qy = 0.5f;
                py = (py - boundary) / (1.0f - boundary);
                q |= 2;
            }
            px = std::min(std::max(px, 0.0f), 0.99999994f);
            py = std::min(std::max(py, 0.0f), 0.99999994f);
            ox = ox + scale * qx;
            oy = oy + scale * qy;
            scale = scale * 0.5f;
            ++depth;
            if (nd.child[q] == 0) {
                cu = ox + scale * px;
                cv = oy + scale * py;
                pdf = telescopedPdf(nd.sum[q], dt.samplingTotal, depth);
                return;
            }
            parentEnergy = nd.sum[q];
            n = nd.child[q];
        }
    }

    // ---- training: splat records into the building trees
    static bool recordValue(const pg_record &r, uint64_t &fixed) {
        if (!(r.wo_pdf > 0)) return false;
        float val = r.radiance / r.wo_pdf;
        if (!(val >= 0) || !(val < 1e30f)) return false;
        float s = val * kFixedScale;
        if (s >= kSplatCap) s = kSplatCap;  // kernels: k_splat
        fixed = (uint64_t)s;
        return true;
    }
    bool learned = false;  // PG_FRACTION_LEARNED: splat also gathers the fraction statistics
    float alpha0 = 0.5f;   // pg_config.bsdf_sampling_fraction
    void splat(const pg_record *recs, size_t n) {
        for (size_t i = 0; i < n; ++i) {
            const pg_record &r = recs[i];
            uint64_t fx;
            if (!recordValue(r, fx)) continue;
            DTreeW &dt = dtrees[lookup(V3(r.pos[0], r.pos[1], r.pos[2]))];
            dt.count += 1;
            if (learned && r.weight >= 0.0f && r.product > 0.0f && r.product < 1e30f) {
                const float a0 = dt.alpha > 0 ? dt.alpha : alpha0;
                const float pb = std::max((r.wo_pdf - (1.0f - a0) * r.weight) / a0, 0.0f);
                for (int k = 0; k < kFracCandidates; ++k) dt.frac[k] += fracStat(r.product, pb, r.weight, r.wo_pdf, k);
                dt.frac[kFracCandidates] += 1;
            }
            float u, v;
            unpackCanonical(r.dir, u, v);
            uint32_t nidx = 0;
            for (;;) {
                BNode &nd = dt.building[nidx];
                int q = childIndex(u, v);
                if (nd.child[q] == 0) {
                    nd.sum[q] += fx;
                    break;
                }
                nidx = nd.child[q];
            }
        }
    }

    // ---- refit after training iteration `iter`
    static uint64_t buildSums(std::vector<BNode> &b, uint32_t n) {
        uint64_t tot = 0;
        for (int q = 0; q < 4; ++q) {
            if (b[n].child[q] != 0) b[n].sum[q] = buildSums(b, b[n].child[q]);
            tot = (tot + b[n].sum[q] < tot) ? ~0ull : tot + b[n].sum[q];  // saturating (pg_sdtree.cpp propagate)
        }
        return tot;
    }
    static float fixedToFloat(uint64_t x) { return (float)std::ldexp((double)x, -24); }

    static void resetBuilding(DTreeW &dt, int maxDepth, float rho) {
        // topology from the current sampling tree's energies (= the just-built building tree)
        const std::vector<QNode> &prev = dt.sampling;
        float total = dt.samplingTotal;
        std::vector<QNode> tmp;  // new nodes with temporary sums
        tmp.emplace_back();
        struct St { uint32_t ni; bool fromPrev; uint32_t src; int depth; };
        std::vector<St> st;
        st.push_back({0, true, 0, 1});
        while (!st.empty()) {
            St s = st.back();
            st.pop_back();
            QNode srcNode = s.fromPrev ? prev[s.src] : tmp[s.src];
            for (int i = 0; i < 4; ++i) {
                float fraction = total > 0 ? (srcNode.sum[i] / total) : std::pow(0.25f, (float)s.depth);
                if (s.depth < maxDepth && fraction > rho) {
                    uint32_t c = (uint32_t)tmp.size();
                    tmp[s.ni].child[i] = c;
                    QNode nn;
                    for (int j = 0; j < 4; ++j) nn.sum[j] = srcNode.sum[i] / 4;
                    tmp.push_back(nn);
                    if (s.fromPrev && srcNode.child[i] != 0) st.push_back({c, true, srcNode.child[i], s.depth + 1});
                    else st.push_back({c, false, c, s.depth + 1});
                }
            }
        }
        dt.building.assign(tmp.size(), BNode{});
        for (size_t i = 0; i < tmp.size(); ++i)
            for (int q = 0; q < 4; ++q) dt.building[i].child[q] = tmp[i].child[q];
        dt.count = 0;
        for (uint64_t &f : dt.frac) f = 0;
    }

    void refit(uint32_t iter, float sThreshold, float rho, int maxDepth) {
        // 1. build: building -> sampling; the learned fraction from this iteration's statistics
        for (auto &dt : dtrees) {
            if (learned && dt.frac[kFracCandidates] >= kFracMinRecords) {
                int best = 0;
                for (int k = 1; k < kFracCandidates; ++k)
                    if ((int64_t)dt.frac[k] >= (int64_t)dt.frac[best]) best = k;
                dt.alpha = fracCandidate(best);
            }
            buildSums(dt.building, 0);
            dt.sampling.assign(dt.building.size(), QNode{});
            for (size_t i = 0; i < dt.building.size(); ++i)
                for (int q = 0; q < 4; ++q) {
                    dt.sampling[i].sum[q] = fixedToFloat(dt.building[i].sum[q]);
                    dt.sampling[i].child[q] = dt.building[i].child[q];
                }
            dt.samplingTotal = nodeTotal(dt.sampling[0].sum);
        }
        // 2. refine the S-tree
        double thr = (double)sThreshold * std::sqrt(std::pow(2.0, (double)iter));
        std::vector<uint32_t> st{0};
        while (!st.empty()) {
            uint32_t n = st.back();
            st.pop_back();
            if (snodes[n].leaf() && (double)dtrees[snodes[n].child[1]].count > thr) {
                uint32_t d0 = snodes[n].child[1];
                uint32_t d1 = (uint32_t)dtrees.size();
                dtrees[d0].count /= 2;
                dtrees.push_back(dtrees[d0]);
                uint32_t c0 = (uint32_t)snodes.size();
                snodes.push_back(SNode{{0xFFFFFFFFu, d0}});
                snodes.push_back(SNode{{0xFFFFFFFFu, d1}});
                snodes[n].child[0] = c0;
                snodes[n].child[1] = c0 + 1;
            }
            if (!snodes[n].leaf()) {
                st.push_back(snodes[n].child[1]);
                st.push_back(snodes[n].child[0]);
            }
        }
        // 3. reset building trees
        for (auto &dt : dtrees) resetBuilding(dt, maxDepth, rho);
        built = true;
    }

    // ---- serialization (DESIGN.md "SD-tree wire format")
    std::vector<uint8_t> serialize() const {
        std::vector<uint8_t> out;
        auto put = [&](const void *p, size_t n) {
            const uint8_t *b = (const uint8_t *)p;
            out.insert(out.end(), b, b + n);
        };
        uint32_t nsamp = 0, nbuild = 0;
        for (auto &dt : dtrees) {
            nsamp += (uint32_t)dt.sampling.size();
            nbuild += (uint32_t)dt.building.size();
        }
        uint32_t hdr[4] = {kSdMagic, 2u, built ? 1u : 0u, 0u};
        put(hdr, sizeof hdr);
        float box[8] = {lo.x, lo.y, lo.z, extent, hi.x, hi.y, hi.z, 0};
        put(box, sizeof box);
        uint32_t cnt[4] = {(uint32_t)snodes.size(), (uint32_t)dtrees.size(), nsamp, nbuild};
        put(cnt, sizeof cnt);
        for (auto &s : snodes) put(s.child, 8);
        uint32_t sbase = 0, bbase = 0;
        for (auto &dt : dtrees) {
            uint32_t meta[8] = {sbase, bbase, (uint32_t)dt.sampling.size(), (uint32_t)dt.building.size(), 0, dt.count, 0, 0};
            std::memcpy(&meta[4], &dt.samplingTotal, 4);
            std::memcpy(&meta[6], &dt.alpha, 4);
            put(meta, sizeof meta);
            sbase += (uint32_t)dt.sampling.size();
            bbase += (uint32_t)dt.building.size();
        }
        sbase = 0;
        for (auto &dt : dtrees) {
            for (auto &n : dt.sampling) {
                put(n.sum, 16);
                uint32_t ch[4];
                for (int q = 0; q < 4; ++q) ch[q] = n.child[q] ? n.child[q] + sbase : 0;
                put(ch, 16);
            }
            sbase += (uint32_t)dt.sampling.size();
        }
        bbase = 0;
        for (auto &dt : dtrees) {
            for (auto &n : dt.building) {
                put(n.sum, 32);
                uint32_t ch[4];
                for (int q = 0; q < 4; ++q) ch[q] = n.child[q] ? n.child[q] + bbase : 0;
                put(ch, 16);
            }
            bbase += (uint32_t)dt.building.size();
        }
        for (auto &dt : dtrees) put(dt.frac, 8 * kFracStats);
        return out;
    }
    bool deserialize(const uint8_t *p, size_t n) {
        size_t off = 0;
        auto get = [&](void *dst, size_t k) {
            if (off + k > n) return false;
            std::memcpy(dst, p + off, k);
            off += k;
            return true;
        };
        uint32_t hdr[4];
        float box[8];
        uint32_t cnt[4];
        if (!get(hdr, 16) || hdr[0] != kSdMagic || hdr[1] != 2 || !get(box, 32) || !get(cnt, 16)) return false;
        built = hdr[2] != 0;
        lo = V3(box[0], box[1], box[2]);
        extent = box[3];
        hi = V3(box[4], box[5], box[6]);
        snodes.resize(cnt[0]);
        for (auto &s : snodes)
            if (!get(s.child, 8)) return false;
        dtrees.assign(cnt[1], DTreeW{});
        std::vector<uint32_t> sb(cnt[1]), bb(cnt[1]);
        for (uint32_t i = 0; i < cnt[1]; ++i) {
            uint32_t meta[8];
            if (!get(meta, 32)) return false;
            sb[i] = meta[0];
            bb[i] = meta[1];
            dtrees[i].sampling.resize(meta[2]);
            dtrees[i].building.resize(meta[3]);
            std::memcpy(&dtrees[i].samplingTotal, &meta[4], 4);
            dtrees[i].count = meta[5];
            std::memcpy(&dtrees[i].alpha, &meta[6], 4);
        }
        for (uint32_t i = 0; i < cnt[1]; ++i)
            for (auto &nd : dtrees[i].sampling) {
                if (!get(nd.sum, 16) || !get(nd.child, 16)) return false;
                for (int q = 0; q < 4; ++q)
                    if (nd.child[q]) nd.child[q] -= sb[i];
            }
        for (uint32_t i = 0; i < cnt[1]; ++i)
            for (auto &nd : dtrees[i].building) {
                if (!get(nd.sum, 32) || !get(nd.child, 16)) return false;
                for (int q = 0; q < 4; ++q)
                    if (nd.child[q]) nd.child[q] -= bb[i];
            }
        for (uint32_t i = 0; i < cnt[1]; ++i)
            if (!get(dtrees[i].frac, 8 * kFracStats)) return false;
        return off == n;
    }
};

}  // namespace orc
