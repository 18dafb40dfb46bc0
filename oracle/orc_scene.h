// ORACLE — test infrastructure only.  CPU restatement of the reference's ray casting, hit-record
// fill, area-light sampling and pinhole camera:
//   ShapeKDTree::rayIntersect (adaptive epsilon, AABB clip)  src/librender/skdtree.cpp:112-142,207-227
//   TriAccel::load / rayIntersect                             include/mitsuba/render/triaccel.h:37-157
//   fillIntersectionRecord<true> + computeShadingFrame         include/mitsuba/render/skdtree.h:343-430
//   Scene::sampleEmitterDirect / pdfEmitterDirect              src/librender/scene.cpp:871-895,992-995
//   AreaLight::sampleDirect / pdfDirect / eval                 src/emitters/area.cpp:158-183
//   Shape::sampleDirect / pdfDirect                            src/librender/shape.cpp:102-126
//   TriMesh::samplePosition, Triangle::sample                  src/librender/trimesh.cpp:412-423, src/libcore/triangle.cpp:24-60
//   DiscreteDistribution::sampleReuse                          include/mitsuba/core/pmf.h:124-188
//   PerspectiveCamera::sampleRay + Transform::lookAt           src/sensors/perspective.cpp:271-298, transform.cpp:191-214
//   EnvironmentMap configure / evalEnvironment / sampleDirect / pdfDirect
//                                                              src/emitters/envmap.cpp:260-356,380-410,516-663
//   TMIPMap level 0: half storage, evalTexel, evalBilinear     include/mitsuba/render/mipmap.h:225-240,503-596
//   solveQuadratic / BSphere::rayIntersect                     src/libcore/util.cpp, include/mitsuba/core/bsphere.h
// The kd-tree (sahkdtree3.h) is replaced by a binned-SAH BVH: only the closest hit matters.
#pragma once
#include <limits>
#include <vector>

#include "orc_bsdf.h"
#include "orc_medium.h"

namespace orc {

constexpr float kInf = std::numeric_limits<float>::infinity();

struct Ray {
    V3 o, d;
    float mint, maxt;
};

struct TriAccel {
    uint32_t k;
    float n_u, n_v, n_d, a_u, a_v, b_nu, b_nv, c_nu, c_nv;
    uint32_t prim;
    int load(V3 A, V3 B, V3 C) {
        static const int waldModulo[4] = {1, 2, 0, 1};
        V3 b = C - A, c = B - A, N = cross(c, b);
        k = 0;
        for (int j = 0; j < 3; j++)
            if (std::fabs(N[j]) > std::fabs(N[(int)k])) k = j;
        int u = waldModulo[k], v = waldModulo[k + 1];
        float n_k = N[(int)k], denom = b[u] * c[v] - b[v] * c[u];
        if (denom == 0) {
            k = 3;
            return 1;
        }
        n_u = N[u] / n_k;
        n_v = N[v] / n_k;
        n_d = dot(A, N) / n_k;
        b_nu = b[u] / denom;
        b_nv = -b[v] / denom;
        a_u = A[u];
        a_v = A[v];
        c_nu = c[v] / denom;
        c_nv = -c[u] / denom;
        return 0;
    }
    bool intersect(const Ray &r, float mint, float maxt, float &u, float &v, float &t) const {
        float o_u, o_v, o_k, d_u, d_v, d_k;
        switch (k) {
            case 0: o_u = r.o.y; o_v = r.o.z; o_k = r.o.x; d_u = r.d.y; d_v = r.d.z; d_k = r.d.x; break;
            case 1: o_u = r.o.z; o_v = r.o.x; o_k = r.o.y; d_u = r.d.z; d_v = r.d.x; d_k = r.d.y; break;
            case 2: o_u = r.o.x; o_v = r.o.y; o_k = r.o.z; d_u = r.d.x; d_v = r.d.y; d_k = r.d.z; break;
            default: return false;
        }
        t = (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
        if (!(t >= mint && t <= maxt)) return false;
        float hu = o_u + t * d_u - a_u, hv = o_v + t * d_v - a_v;
        u = hv * b_nu + hu * b_nv;
        v = hu * c_nu + hv * c_nv;
        return u >= 0 && v >= 0 && u + v <= 1.0f;
    }
};

struct AABB {
    V3 lo{kInf, kInf, kInf}, hi{-kInf, -kInf, -kInf};
    void expand(V3 p) {
        lo = V3(std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z));
        hi = V3(std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z));
    }
    void expand(const AABB &b) {  // component-wise, so an empty b (lo = +inf, hi = -inf) is a no-op
        lo = V3(std::min(lo.x, b.lo.x), std::min(lo.y, b.lo.y), std::min(lo.z, b.lo.z));
        hi = V3(std::max(hi.x, b.hi.x), std::max(hi.y, b.hi.y), std::max(hi.z, b.hi.z));
    }
    float area() const {
        V3 e = hi - lo;
        if (e.x < 0) return 0;
        return 2 * (e.x * e.y + e.y * e.z + e.z * e.x);
    }
    // AABB::rayIntersect (include/mitsuba/core/aabb.h): slab test, returns near/far (may be < 0)
    bool rayIntersect(const Ray &r, float &nearT, float &farT) const {
        nearT = -kInf;
        farT = kInf;
        for (int i = 0; i < 3; i++) {
            float o = r.o[i], d = r.d[i], mn = lo[i], mx = hi[i];
            if (d == 0) {
                if (o < mn || o > mx) return false;
            } else {
                float t1 = (mn - o) / d, t2 = (mx - o) / d;
                if (t1 > t2) std::swap(t1, t2);
                nearT = std::max(t1, nearT);
                farT = std::min(t2, farT);
                if (!(nearT <= farT)) return false;
            }
        }
        return true;
    }
};

struct Its {
    bool valid = false;
    float t = kInf;
    V3 p, geoN, uv;
    Frame sh;
    V3 wi;
    uint32_t prim = 0, shape = 0;
    V3 toLocal(V3 v) const { return sh.toLocal(v); }
    V3 toWorld(V3 v) const { return sh.toWorld(v); }
};

struct BvhNode {
    AABB box;
    uint32_t left_or_first, count;  // count > 0 -> leaf
};

struct Camera {
    V3 o, left, up, dir;
    float tanHalf, aspect, nearC, farC;
    uint32_t W, H;
};

// binary16 round-to-nearest-even (the MIP map's SpectrumHalf texel storage), as a float
inline float halfRound(float f) {
    if (!std::isfinite(f) || f == 0.0f) return f;
    const float a = std::fabs(f);
    if (a >= 65520.0f) return std::copysign(kInf, f);
    float q;
    if (a < 6.103515625e-05f) {
        q = 5.9604644775390625e-08f;
    } else {
        int e;
        std::frexp(a, &e);
        q = std::ldexp(1.0f, e - 11);
    }
    return std::copysign(std::nearbyint(a / q) * q, f);
}
// Environment emitter (EnvironmentMap, envmap.cpp) restated on the latitude-longitude level 0
struct Env {
    bool valid = false;
    int W = 0, H = 0;
    std::vector<V3> tex;  // half-rounded, negatives clamped (mipmap.h:232-240)
    std::vector<float> cdfRows, cdfCols, rowWeights;
    float normalization = 0, pixelSize[2] = {0, 0}, scale = 1, radius = 0;
    V3 center;
    float R[9];

    V3 texel(int x, int y) const {  // evalTexel: ERepeat in u, EClamp in v
        if (x < 0 || x >= W) {
            x %= W;
            if (x < 0) x += W;
        }
        y = std::min(std::max(y, 0), H - 1);
        return tex[(size_t)y * W + x];
    }
    V3 toLocal(V3 d) const {
        return V3(R[0] * d.x + R[3] * d.y + R[6] * d.z, R[1] * d.x + R[4] * d.y + R[7] * d.z,
                  R[2] * d.x + R[5] * d.y + R[8] * d.z);
    }
    V3 toWorld(V3 d) const {
        return V3(R[0] * d.x + R[1] * d.y + R[2] * d.z, R[3] * d.x + R[4] * d.y + R[5] * d.z,
                  R[6] * d.x + R[7] * d.y + R[8] * d.z);
    }
    static float safeAcos(float v) { return std::acos(std::min(1.0f, std::max(-1.0f, v))); }

    // EnvironmentMap::configure (envmap.cpp:260-329) + createShape's bounding sphere (:331-356)
    void build(const pg_envmap &e, const AABB &box) {
        W = (int)e.width;
        H = (int)e.height;
        scale = e.scale;
        for (int k = 0; k < 9; ++k) R[k] = e.to_world[k];
        tex.resize((size_t)W * H);
        for (size_t i = 0; i < (size_t)W * H; ++i)
            tex[i] = V3(halfRound(std::max(e.rgb[3 * i], 0.0f)), halfRound(std::max(e.rgb[3 * i + 1], 0.0f)),
                        halfRound(std::max(e.rgb[3 * i + 2], 0.0f)));
        cdfCols.assign((size_t)(W + 1) * H, 0.0f);
        cdfRows.assign(H + 1, 0.0f);
        rowWeights.assign(H, 0.0f);
        size_t colPos = 0, rowPos = 0;
        float rowSum = 0.0f;
        cdfRows[rowPos++] = 0;
        for (int y = 0; y < H; ++y) {
            float colSum = 0;
            cdfCols[colPos++] = 0;
            for (int x = 0; x < W; ++x) {
                colSum += luminance(tex[(size_t)y * W + x]);
                cdfCols[colPos++] = colSum;
            }
            if (colSum > 0) {
                float normalization_ = 1.0f / colSum;
                for (int x = 1; x < W; ++x) cdfCols[colPos - x - 1] *= normalization_;
            } else {  // black row: zero marginal mass; uniform conditional (the reference divides by 0)
                for (int x = 1; x < W; ++x) cdfCols[colPos - x - 1] = (float)(W - x) / (float)W;
            }
            cdfCols[colPos - 1] = 1.0f;
            float weight = (float)std::sin((y + 0.5f) * M_PI / H);
            rowWeights[y] = weight;
            rowSum += colSum * weight;
            cdfRows[rowPos++] = rowSum;
        }
        float normalization_ = 1.0f / rowSum;
        for (int y = 1; y < H; ++y) cdfRows[rowPos - y - 1] *= normalization_;
        cdfRows[rowPos - 1] = 1.0f;
        normalization = (float)(1.0f / (rowSum * (2 * M_PI / W) * (M_PI / H)));
        pixelSize[0] = (float)(2 * M_PI / W);
        pixelSize[1] = (float)(M_PI / H);
        center = (box.lo + box.hi) * 0.5f;
        radius = std::max(kEpsilon, length(box.hi - center) * 1.5f);
        valid = true;
    }
    // evalEnvironment without differentials -> evalBilinear(0, uv) * scale (envmap.cpp:380-410)
    V3 eval(V3 dWorld) const {
        V3 v = toLocal(dWorld);
        float ux = std::atan2(v.x, -v.z) * (0.5f * kInvPi), uy = safeAcos(v.y) * kInvPi;
        if (!std::isfinite(ux) || !std::isfinite(uy)) return V3(0.f);
        float u = ux * W - 0.5f, w = uy * H - 0.5f;
        int xPos = (int)std::floor(u), yPos = (int)std::floor(w);
        float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = w - yPos, dy2 = 1.0f - dy1;
        V3 r = texel(xPos, yPos) * dx2 * dy2 + texel(xPos, yPos + 1) * dx2 * dy1 + texel(xPos + 1, yPos) * dx1 * dy2 +
               texel(xPos + 1, yPos + 1) * dx1 * dy1;
        return r * scale;
    }
    // internalPdfDirection (envmap.cpp:603-633) of a local direction
    float pdfLocal(V3 d) const {
        float ux = std::atan2(d.x, -d.z) * (0.5f * kInvPi), uy = safeAcos(d.y) * kInvPi;
        if (!std::isfinite(ux) || !std::isfinite(uy)) return 0.0f;
        float u = ux * W - 0.5f, w = uy * H - 0.5f;
        int xPos = (int)std::floor(u), yPos = (int)std::floor(w);
        float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = w - yPos, dy2 = 1.0f - dy1;
        V3 v1 = texel(xPos, yPos) * dx2 * dy2 + texel(xPos + 1, yPos) * dx1 * dy2;
        V3 v2 = texel(xPos, yPos + 1) * dx2 * dy1 + texel(xPos + 1, yPos + 1) * dx1 * dy1;
        float sinTheta = safe_sqrt(1 - d.y * d.y);
        return (luminance(v1) * rowWeights[std::min(std::max(yPos, 0), H - 1)] +
                luminance(v2) * rowWeights[std::min(std::max(yPos + 1, 0), H - 1)]) *
               normalization / std::max(std::fabs(sinTheta), kEpsilon);
    }
    float pdf(V3 dWorld) const { return pdfLocal(toLocal(dWorld)); }
    // sampleReuse (envmap.cpp:658-663)
    static uint32_t sampleReuse(const float *cdf, uint32_t size, float &s) {
        const float *entry = std::lower_bound(cdf, cdf + size + 1, s);
        uint32_t index = std::min((uint32_t)std::max((ptrdiff_t)0, entry - cdf - 1), size - 1);
        s = (s - cdf[index]) / (cdf[index + 1] - cdf[index]);
        return index;
    }
    static float intervalToTent(float s) {  // warp.cpp:143-155
        float sign;
        if (s < 0.5f) {
            sign = 1;
            s *= 2;
        } else {
            sign = -1;
            s = 2 * (s - 0.5f);
        }
        return sign * (1 - std::sqrt(s));
    }
    // internalSampleDirection (envmap.cpp:567-600)
    V3 sampleLocal(float sx, float sy, V3 &value, float &pdfOut) const {
        uint32_t row = sampleReuse(cdfRows.data(), (uint32_t)H, sy);
        uint32_t col = sampleReuse(cdfCols.data() + (size_t)row * (W + 1), (uint32_t)W, sx);
        float px = (float)col + intervalToTent(sx), py = (float)row + intervalToTent(sy);
        int xPos = (int)std::floor(px), yPos = (int)std::floor(py);
        float dx1 = px - xPos, dx2 = 1.0f - dx1, dy1 = py - yPos, dy2 = 1.0f - dy1;
        V3 v1 = texel(xPos, yPos) * dx2 * dy2 + texel(xPos + 1, yPos) * dx1 * dy2;
        V3 v2 = texel(xPos, yPos + 1) * dx2 * dy1 + texel(xPos + 1, yPos + 1) * dx1 * dy1;
        value = (v1 + v2) * scale;
        pdfOut = (luminance(v1) * rowWeights[std::min(std::max(yPos, 0), H - 1)] +
                  luminance(v2) * rowWeights[std::min(std::max(yPos + 1, 0), H - 1)]) *
                 normalization;
        float sinPhi = std::sin(pixelSize[0] * (px + 0.5f)), cosPhi = std::cos(pixelSize[0] * (px + 0.5f));
        float sinTheta = std::sin(pixelSize[1] * (py + 0.5f)), cosTheta = std::cos(pixelSize[1] * (py + 0.5f));
        pdfOut /= std::max(std::fabs(sinTheta), kEpsilon);
        return V3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    }
    // sampleDirect (envmap.cpp:516-543): value / pdf; pdf = 0 on failure
    V3 sampleDirect(V3 ref, float sx, float sy, V3 &d, float &dist, float &pdfOut) const {
        V3 value;
        float pdf;
        d = toWorld(sampleLocal(sx, sy, value, pdf));
        pdfOut = 0;
        if (isZero(value) || pdf == 0) return V3(0.f);
        V3 o = ref - center;
        float A = dot(d, d), B = 2 * dot(o, d), C = dot(o, o) - radius * radius;
        float disc = B * B - 4.0f * A * C;
        if (disc < 0) return V3(0.f);
        float sq = std::sqrt(disc), temp = (B < 0) ? -0.5f * (B - sq) : -0.5f * (B + sq);
        float x0 = temp / A, x1 = C / temp;
        if (x0 > x1) std::swap(x0, x1);
        if (x0 >= 0 || x1 <= 0) return V3(0.f);
        dist = x1;
        pdfOut = pdf;
        return value / pdf;
    }
};

// Debug log of the rays one path casts (oracle_path_rays, tools/diverge_c3.py): when set, every
// closest-hit and shadow query appends (kind 0 / 1, o.xyz, mint, d.xyz, maxt, t or occluded, prim).
inline thread_local std::vector<float> *g_rayLog = nullptr;

struct Scene {
    std::vector<V3> pos, nrm;
    std::vector<uint32_t> idx;
    std::vector<uint32_t> triShape;
    std::vector<pg_shape> shapes;
    std::vector<Material> mats;
    std::vector<pg_emitter> emitters;
    std::vector<std::vector<float>> emCdf;  // per emitter: normalized triangle-area CDF
    std::vector<float> emArea;
    std::vector<TriAccel> accel;  // in BVH order
    std::vector<BvhNode> nodes;
    AABB bounds;
    Camera cam;
    Env env;  // the last emitter of the uniform pick when valid
    uint32_t numEmitters() const { return (uint32_t)emitters.size() + (env.valid ? 1u : 0u); }
    std::vector<Medium> media;
    int camMedium = -1;

    void build(const pg_scene_desc &d);
    bool intersect(const Ray &ray, Its &its) const {
        const bool h = intersectImpl(ray, its);
        logRay(0, ray, h ? its.t : 0.0f, h ? its.prim : 0xFFFFFFFFu);
        return h;
    }
    bool occluded(const Ray &ray) const {
        const bool o = occludedImpl(ray);
        logRay(1, ray, o ? 1.0f : 0.0f, 0u);
        return o;
    }
    bool intersectImpl(const Ray &ray, Its &its) const;
    bool occludedImpl(const Ray &ray) const;
    bool intersectRaw(const Ray &ray, float &t, uint32_t &prim) const;
    bool traverse(const Ray &r, float mint, float maxt, bool any, float &t, float &u, float &v, uint32_t &prim) const;
    bool bruteForce(const Ray &r, float mint, float maxt, float &t, float &u, float &v, uint32_t &prim) const;
    static void logRay(int kind, const Ray &r, float res, uint32_t prim) {
        if (!g_rayLog) return;
        float pb;
        std::memcpy(&pb, &prim, 4);
        g_rayLog->insert(g_rayLog->end(), {(float)kind, r.o.x, r.o.y, r.o.z, r.mint, r.d.x, r.d.y, r.d.z, r.maxt, res, pb});
    }
    void fill(const Ray &r, float t, float u, float v, uint32_t prim, Its &its) const;
    Ray cameraRay(float sx, float sy) const;
};

inline Ray Scene::cameraRay(float px, float py) const {
    // sampleToCamera for fovAxis=x: screen = (1 - 2 sx, (1 - 2 sy)/aspect) scaled by tan(fov/2)
    float sx = px / (float)cam.W, sy = py / (float)cam.H;
    V3 nearP((1.0f - 2.0f * sx) * cam.tanHalf, (1.0f - 2.0f * sy) / cam.aspect * cam.tanHalf, 1.0f);
    V3 d = normalize(nearP);
    float invZ = 1.0f / d.z;
    Ray r;
    r.mint = cam.nearC * invZ;
    r.maxt = cam.farC * invZ;
    r.o = cam.o;
    r.d = cam.left * d.x + cam.up * d.y + cam.dir * d.z;
    return r;
}

inline void Scene::build(const pg_scene_desc &d) {
    pos.resize(d.num_vertices);
    for (uint32_t i = 0; i < d.num_vertices; ++i) pos[i] = V3(d.positions[3 * i], d.positions[3 * i + 1], d.positions[3 * i + 2]);
    if (d.normals) {
        nrm.resize(d.num_vertices);
        for (uint32_t i = 0; i < d.num_vertices; ++i) nrm[i] = V3(d.normals[3 * i], d.normals[3 * i + 1], d.normals[3 * i + 2]);
    }
    idx.assign(d.indices, d.indices + 3 * (size_t)d.num_triangles);
    shapes.assign(d.shapes, d.shapes + d.num_shapes);
    triShape.assign(d.num_triangles, 0);
    for (uint32_t s = 0; s < d.num_shapes; ++s)
        for (uint32_t t = 0; t < shapes[s].tri_count; ++t) triShape[shapes[s].tri_begin + t] = s;
    for (uint32_t m = 0; m < d.num_materials; ++m) mats.push_back(makeMaterial(d.materials[m]));
    emitters.assign(d.emitters, d.emitters + d.num_emitters);
    media.resize(d.num_media);
    for (uint32_t m = 0; m < d.num_media; ++m) media[m].init(d.media[m]);
    camMedium = d.camera_medium;
    for (auto &e : emitters) {
        const pg_shape &sh = shapes[e.shape];
        // area CDF: double accumulation of fp32 triangle areas, normalized, stored as fp32
        std::vector<float> cdf(sh.tri_count + 1, 0.0f);
        double acc = 0;
        std::vector<double> cd(sh.tri_count + 1, 0.0);
        for (uint32_t t = 0; t < sh.tri_count; ++t) {
            uint32_t tri = sh.tri_begin + t;
            V3 a = pos[idx[3 * tri]], b = pos[idx[3 * tri + 1]], c = pos[idx[3 * tri + 2]];
            acc += (double)(0.5f * length(cross(b - a, c - a)));
            cd[t + 1] = acc;
        }
        for (uint32_t t = 0; t <= sh.tri_count; ++t) cdf[t] = (float)(cd[t] / acc);
        cdf[sh.tri_count] = 1.0f;
        emCdf.push_back(cdf);
        emArea.push_back((float)acc);
    }
    // camera (Transform::lookAt)
    const pg_camera &c = d.camera;
    V3 o(c.origin[0], c.origin[1], c.origin[2]), tg(c.target[0], c.target[1], c.target[2]), up(c.up[0], c.up[1], c.up[2]);
    cam.o = o;
    cam.dir = normalize(tg - o);
    cam.left = normalize(cross(up, cam.dir));
    cam.up = cross(cam.dir, cam.left);
    cam.tanHalf = std::tan(c.fov_x_deg * kPi / 360.0f);
    cam.W = c.width;
    cam.H = c.height;
    cam.aspect = (float)c.width / (float)c.height;
    cam.nearC = c.near_clip;
    cam.farC = c.far_clip;

    // ---- binned SAH BVH over triangle bounds
    uint32_t nt = d.num_triangles;
    std::vector<AABB> tb(nt);
    std::vector<V3> cen(nt);
    for (uint32_t t = 0; t < nt; ++t) {
        for (int j = 0; j < 3; ++j) tb[t].expand(pos[idx[3 * t + j]]);
        bounds.expand(tb[t]);
        cen[t] = (tb[t].lo + tb[t].hi) * 0.5f;
    }
    // the kd-tree's slightly enlarged scene AABB (gkdtree.h:1213-1220, MTS_KD_AABB_EPSILON = 1e-3)
    {
        const float eps = 1e-3f;
        bounds.lo = bounds.lo - ((bounds.hi - bounds.lo) * eps + V3(eps));
        bounds.hi = bounds.hi + ((bounds.hi - bounds.lo) * eps + V3(eps));
    }
    if (d.envmap) env.build(*d.envmap, bounds);
    std::vector<uint32_t> order(nt);
    for (uint32_t t = 0; t < nt; ++t) order[t] = t;
    nodes.clear();
    nodes.reserve(2 * (size_t)nt + 1);
    struct Job { uint32_t node, first, count; };
    std::vector<Job> stack;
    nodes.push_back(BvhNode{});
    stack.push_back({0, 0, nt});
    while (!stack.empty()) {
        Job j = stack.back();
        stack.pop_back();
        AABB box, cb;
        for (uint32_t i = j.first; i < j.first + j.count; ++i) {
            box.expand(tb[order[i]]);
            cb.expand(cen[order[i]]);
        }
        nodes[j.node].box = box;
        bool leaf = j.count <= 4;
        uint32_t mid = 0;
        if (!leaf) {
            const int B = 16;
            float best = kInf;
            int bestAxis = -1, bestBin = -1;
            for (int ax = 0; ax < 3; ++ax) {
                float lo = cb.lo[ax], hi = cb.hi[ax];
                if (!(hi > lo)) continue;
                AABB bb[B];
                uint32_t bc[B] = {0};
                for (uint32_t i = j.first; i < j.first + j.count; ++i) {
                    int b = (int)((cen[order[i]][ax] - lo) / (hi - lo) * B);
                    b = std::min(std::max(b, 0), B - 1);
                    bb[b].expand(tb[order[i]]);
                    bc[b]++;
                }
                AABB la[B];
                uint32_t lc[B];
                AABB acc;
                uint32_t n = 0;
                for (int b = 0; b < B; ++b) {
                    acc.expand(bb[b]);
                    n += bc[b];
                    la[b] = acc;
                    lc[b] = n;
                }
                acc = AABB();
                n = 0;
                for (int b = B - 1; b > 0; --b) {
                    acc.expand(bb[b]);
                    n += bc[b];
                    float cost = la[b - 1].area() * lc[b - 1] + acc.area() * n;
                    if (lc[b - 1] > 0 && n > 0 && cost < best) {
                        best = cost;
                        bestAxis = ax;
                        bestBin = b;
                    }
                }
            }
            // SAH with a traversal cost of one triangle test per node visit; leaves hold <= 8
            if (bestAxis < 0 || box.area() + best >= box.area() * j.count) {
                if (j.count <= 8 || bestAxis < 0) {
                    leaf = true;
                    if (bestAxis < 0 && j.count > 8) {  // all centroids equal: split in the middle
                        leaf = false;
                        mid = j.first + j.count / 2;
                    }
                }
            }
            if (!leaf && bestAxis >= 0) {
                float lo = cb.lo[bestAxis], hi = cb.hi[bestAxis];
                auto it = std::partition(order.begin() + j.first, order.begin() + j.first + j.count, [&](uint32_t t) {
                    int b = (int)((cen[t][bestAxis] - lo) / (hi - lo) * B);
                    b = std::min(std::max(b, 0), B - 1);
                    return b < bestBin;
                });
                mid = (uint32_t)(it - order.begin());
                if (mid == j.first || mid == j.first + j.count) mid = j.first + j.count / 2;
            }
        }
        if (leaf) {
            nodes[j.node].left_or_first = j.first;
            nodes[j.node].count = j.count;
        } else {
            uint32_t l = (uint32_t)nodes.size();
            nodes.push_back(BvhNode{});
            nodes.push_back(BvhNode{});
            nodes[j.node].left_or_first = l;
            nodes[j.node].count = 0;
            stack.push_back({l, j.first, mid - j.first});
            stack.push_back({l + 1, mid, j.first + j.count - mid});
        }
    }
    accel.resize(nt);
    for (uint32_t i = 0; i < nt; ++i) {
        uint32_t t = order[i];
        accel[i].load(pos[idx[3 * t]], pos[idx[3 * t + 1]], pos[idx[3 * t + 2]]);
        accel[i].prim = t;
    }
}

// Closest hit over the BVH with the same contract as a brute-force loop over every TriAccel: the
// smallest t in [mint, maxt], equal distances (shared edges, coplanar triangles) to the lower
// original triangle index, so the hit depends on neither the tree nor the visiting order (the
// kd-tree of skdtree.cpp:112-142 finds every triangle its TriAccel test accepts).  Box tests are made
// robust to rounding as the kernels' walk is (pg_trace.h slabRay): each axis's slab is padded by
// 2^-21 |o_a / d_a| (the rounding of (plane - o) / d far from the origin), intervals are compared as
// t0 <= t1 (1 + 2^-21), and boxes are culled against the current hit distance widened by its own
// rounding, so a box holding a tie is still visited.  Without this a ray grazing a box edge far from
// the origin could miss a hit inside it (tests/test_oracle_kat.py: strip geometry).
inline bool Scene::traverse(const Ray &r, float mint, float maxt, bool any, float &tBest, float &uBest, float &vBest,
                            uint32_t &prim) const {
    if (nodes.empty()) return false;
    const float eps = 1e-30f;  // as the kernels: no infinite reciprocals, so no inf - inf below
    const V3 inv(1.0f / (std::fabs(r.d.x) > eps ? r.d.x : std::copysign(eps, r.d.x)),
                 1.0f / (std::fabs(r.d.y) > eps ? r.d.y : std::copysign(eps, r.d.y)),
                 1.0f / (std::fabs(r.d.z) > eps ? r.d.z : std::copysign(eps, r.d.z)));
    const float kPad = 4.76837158e-7f, kRel = 1.000000477f;  // 2^-21, 1 + 2^-21
    V3 pad;
    float oidMax = 0.0f;
    for (int a = 0; a < 3; ++a) {
        const float oid = std::fabs(r.o[a] * inv[a]);
        pad[a] = kPad * oid;
        oidMax = std::max(oidMax, oid);
    }
    const float tslack = 1e-6f * oidMax;
    bool hit = false;
    float far = maxt;
    auto cull = [&]() { return hit ? far * 1.000001f + tslack : far; };
    // slab test of node n against [mint, cull()]; returns the entry distance or +inf on a miss
    auto enter = [&](const BvhNode &n) {
        float t0 = mint, t1 = cull();
        for (int a = 0; a < 3; ++a) {
            float ta = (n.box.lo[a] - r.o[a]) * inv[a], tb = (n.box.hi[a] - r.o[a]) * inv[a];
            if (ta > tb) std::swap(ta, tb);
            if (std::isnan(ta) || std::isnan(tb)) continue;  // degenerate slab with o on the plane
            t0 = std::max(t0, ta - pad[a]);
            t1 = std::min(t1, tb + pad[a]);
        }
        return t0 <= t1 * kRel ? t0 : kInf;
    };
    // near-first traversal: stack entries carry their entry distance, culled against the widened far
    std::vector<std::pair<uint32_t, float>> stack;
    stack.reserve(64);
    if (enter(nodes[0]) < kInf) stack.push_back({0u, 0.0f});
    while (!stack.empty()) {
        auto [ni, tin] = stack.back();
        stack.pop_back();
        if (tin > cull()) continue;
        const BvhNode &n = nodes[ni];
        if (n.count > 0) {
            for (uint32_t i = n.left_or_first; i < n.left_or_first + n.count; ++i) {
                float u, v, t;
                if (accel[i].intersect(r, mint, far, u, v, t) && (!hit || t < far || accel[i].prim < prim)) {
                    if (any) return true;
                    far = t;
                    tBest = t;
                    uBest = u;
                    vBest = v;
                    prim = accel[i].prim;
                    hit = true;
                }
            }
        } else {
            const uint32_t c0 = n.left_or_first, c1 = n.left_or_first + 1;
            const float t0 = enter(nodes[c0]), t1 = enter(nodes[c1]);
            if (t0 <= t1) {
                if (t1 < kInf) stack.push_back({c1, t1});
                if (t0 < kInf) stack.push_back({c0, t0});
            } else {
                if (t0 < kInf) stack.push_back({c0, t0});
                if (t1 < kInf) stack.push_back({c1, t1});
            }
        }
    }
    return hit;
}

// every TriAccel with traverse()'s accept rule (smallest t, ties to the lower original index): the
// walk's contract, checked in tests/test_oracle_kat.py
inline bool Scene::bruteForce(const Ray &r, float mint, float maxt, float &tBest, float &uBest, float &vBest,
                              uint32_t &prim) const {
    bool hit = false;
    float far = maxt;
    for (const TriAccel &a : accel) {
        float u, v, t;
        if (a.intersect(r, mint, far, u, v, t) && (!hit || t < far || a.prim < prim)) {
            far = tBest = t;
            uBest = u;
            vBest = v;
            prim = a.prim;
            hit = true;
        }
    }
    return hit;
}

inline void Scene::fill(const Ray &r, float t, float u, float v, uint32_t prim, Its &its) const {
    uint32_t i0 = idx[3 * prim], i1 = idx[3 * prim + 1], i2 = idx[3 * prim + 2];
    V3 p0 = pos[i0], p1 = pos[i1], p2 = pos[i2];
    float b0 = 1 - u - v, b1 = u, b2 = v;
    its.valid = true;
    its.t = t;
    its.p = p0 * b0 + p1 * b1 + p2 * b2;
    V3 side1 = p1 - p0, side2 = p2 - p0;
    V3 fn = cross(side1, side2);
    float len = length(fn);
    if (!isZero(fn)) fn = fn / len;
    V3 shn;
    if (!nrm.empty()) {
        shn = normalize(nrm[i0] * b0 + nrm[i1] * b1 + nrm[i2] * b2);
        if (dot(fn, shn) < 0) fn = -fn;
    } else {
        shn = fn;
    }
    its.geoN = fn;
    its.sh = shadingFrame(shn, side1);
    its.prim = prim;
    its.shape = triShape[prim];
    its.wi = its.sh.toLocal(-r.d);
}

// ShapeKDTree::rayIntersect(ray, its): AABB clip + adaptive epsilon (skdtree.cpp:112-142)
inline bool Scene::intersectImpl(const Ray &ray, Its &its) const {
    its.valid = false;
    float mint, maxt;
    if (!bounds.rayIntersect(ray, mint, maxt)) return false;
    float rayMinT = ray.mint;
    if (rayMinT == kEpsilon)
        rayMinT *= std::max(std::max(std::max(std::fabs(ray.o.x), std::fabs(ray.o.y)), std::fabs(ray.o.z)), kEpsilon);
    if (rayMinT > mint) mint = rayMinT;
    if (ray.maxt < maxt) maxt = ray.maxt;
    if (!(maxt > mint)) return false;
    float t, u, v;
    uint32_t prim;
    if (!traverse(ray, mint, maxt, false, t, u, v, prim)) return false;
    fill(ray, t, u, v, prim, its);
    return true;
}

// ShapeKDTree::rayIntersect(ray) shadow variant (skdtree.cpp:207-227)
inline bool Scene::occludedImpl(const Ray &ray) const {
    float mint, maxt;
    if (!bounds.rayIntersect(ray, mint, maxt)) return false;
    float rayMinT = ray.mint;
    if (rayMinT == kEpsilon) rayMinT *= std::max(std::max(std::fabs(ray.o.x), std::fabs(ray.o.y)), std::fabs(ray.o.z));
    if (rayMinT > mint) mint = rayMinT;
    if (ray.maxt < maxt) maxt = ray.maxt;
    if (!(maxt > mint)) return false;
    float t, u, v;
    uint32_t prim;
    return traverse(ray, mint, maxt, true, t, u, v, prim);
}

// ShapeKDTree::rayIntersect(ray, t, shape, n, uv) (skdtree.cpp:144-162): closest hit with the
// shadow-ray epsilon rule; the caller takes the unflipped face normal from `prim`
inline bool Scene::intersectRaw(const Ray &ray, float &tOut, uint32_t &prim) const {
    tOut = kInf;
    float mint, maxt;
    if (!bounds.rayIntersect(ray, mint, maxt)) return false;
    float rayMinT = ray.mint;
    if (rayMinT == kEpsilon) rayMinT *= std::max(std::max(std::fabs(ray.o.x), std::fabs(ray.o.y)), std::fabs(ray.o.z));
    if (rayMinT > mint) mint = rayMinT;
    if (ray.maxt < maxt) maxt = ray.maxt;
    if (!(maxt > mint)) return false;
    float t, u, v;
    if (!traverse(ray, mint, maxt, false, t, u, v, prim)) return false;
    tOut = t;
    return true;
}

// DiscreteDistribution::sampleReuse (pmf.h:124-169) over a normalized CDF
inline uint32_t sampleReuseCdf(const std::vector<float> &cdf, float &s) {
    auto it = std::lower_bound(cdf.begin(), cdf.end(), s);
    ptrdiff_t e = it - cdf.begin() - 1;
    size_t index = std::min(cdf.size() - 2, (size_t)std::max((ptrdiff_t)0, e));
    while (cdf[index + 1] - cdf[index] == 0 && index < cdf.size() - 2) ++index;
    s = (s - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return (uint32_t)index;
}

struct DirectRec {
    V3 ref, refN, p, n, d;
    float dist = 0, pdf = 0;
    int emitter = -1;
};

// Scene::sampleEmitterDirect without the visibility test (scene.cpp:871-895 up to the shadow ray):
// returns radiance / pdf with dr.pdf including the emitter-selection pdf; dr.pdf = 0 on failure
inline V3 sampleEmitterNoVis(const Scene &S, DirectRec &dr, float sx, float sy) {
    uint32_t ne = S.numEmitters();
    dr.pdf = 0;
    if (ne == 0) return V3(0.f);
    // uniform emitter pdf (every sampling weight is 1): sampleReuse on a uniform CDF
    float emPdf = 1.0f / (float)ne;
    uint32_t ei = std::min((uint32_t)(sx * (float)ne), ne - 1);
    sx = sx * (float)ne - (float)ei;
    if (S.env.valid && ei == ne - 1) {  // the environment emitter (no refN test: envmap.cpp:516-543)
        float pdf;
        V3 value = S.env.sampleDirect(dr.ref, sx, sy, dr.d, dr.dist, pdf);
        if (pdf == 0) return V3(0.f);
        dr.p = dr.ref + dr.d * dr.dist;
        dr.n = -dr.d;
        dr.emitter = (int)ei;
        dr.pdf = pdf * emPdf;
        return value / emPdf;
    }
    const pg_emitter &em = S.emitters[ei];
    const pg_shape &sh = S.shapes[em.shape];
    // TriMesh::samplePosition: triangle by area on sample.y (reuse), then Triangle::sample(sample)
    uint32_t ti = sampleReuseCdf(S.emCdf[ei], sy);
    uint32_t tri = sh.tri_begin + ti;
    uint32_t i0 = S.idx[3 * tri], i1 = S.idx[3 * tri + 1], i2 = S.idx[3 * tri + 2];
    V3 p0 = S.pos[i0], p1 = S.pos[i1], p2 = S.pos[i2];
    float a = safe_sqrt(1.0f - sx);
    float bx = 1 - a, by = a * sy;
    V3 sideA = p1 - p0, sideB = p2 - p0;
    V3 p = p0 + (sideA * bx) + (sideB * by);
    V3 n;
    if (!S.nrm.empty()) n = normalize(S.nrm[i0] * (1.0f - bx - by) + S.nrm[i1] * bx + S.nrm[i2] * by);
    else n = normalize(cross(sideA, sideB));
    dr.p = p;
    dr.n = n;
    dr.pdf = 1.0f / S.emArea[ei];
    // Shape::sampleDirect
    dr.d = p - dr.ref;
    float distSq = lengthSq(dr.d);
    dr.dist = std::sqrt(distSq);
    dr.d = dr.d / dr.dist;
    float dp = absDot(dr.d, dr.n);
    dr.pdf *= dp != 0 ? (distSq / dp) : 0.0f;
    // AreaLight::sampleDirect
    if (!(dot(dr.d, dr.refN) >= 0 && dot(dr.d, dr.n) < 0 && dr.pdf != 0)) {
        dr.pdf = 0;
        return V3(0.f);
    }
    V3 value = V3(em.radiance[0], em.radiance[1], em.radiance[2]) / dr.pdf;
    dr.emitter = (int)ei;
    dr.pdf *= emPdf;
    return value / emPdf;
}

// Scene::sampleEmitterDirect with visibility (scene.cpp:871-895)
inline V3 sampleEmitterDirect(const Scene &S, DirectRec &dr, float sx, float sy) {
    V3 value = sampleEmitterNoVis(S, dr, sx, sy);
    if (dr.pdf == 0) return V3(0.f);
    Ray sr{dr.ref, dr.d, kEpsilon, dr.dist * (1 - kShadowEpsilon)};
    if (S.occluded(sr)) return V3(0.f);
    return value;
}

// Scene::pdfEmitterDirect for a BSDF-sampled hit on emitter `ei` (records.inl:170-178 setQuery)
inline float pdfEmitterDirect(const Scene &S, int ei, V3 refN, V3 d, V3 n, float dist) {
    if (!(dot(d, refN) >= 0 && dot(d, n) < 0)) return 0.0f;
    float pdfPos = 1.0f / S.emArea[ei];
    return pdfPos * (dist * dist) / absDot(d, n) * (1.0f / (float)S.numEmitters());
}

// Scene::pdfEmitterDirect for a BSDF-sampled direction that escaped to the environment emitter
// (fillDirectSamplingRecord: solid-angle measure, envmap.cpp:358-374,545-556)
inline float pdfEnvDirect(const Scene &S, V3 d) { return S.env.pdf(d) * (1.0f / (float)S.numEmitters()); }

inline V3 emitterLe(const Scene &S, const Its &its, V3 w) {
    int e = S.shapes[its.shape].emitter;
    if (e < 0) return V3(0.f);
    if (dot(its.sh.n, w) <= 0) return V3(0.f);
    const pg_emitter &em = S.emitters[e];
    return V3(em.radiance[0], em.radiance[1], em.radiance[2]);
}

}  // namespace orc
