// Environment-emitter tables (EnvironmentMap::configure, src/emitters/envmap.cpp:260-329, and the
// MIP map's level 0, include/mitsuba/render/mipmap.h:225-240).  The arithmetic keeps the
// reference's types: the CDFs accumulate in Float (fp32) and are stored as float; the row weights,
// the normalisation and the pixel size are evaluated in double (M_PI is a double) and stored as fp32.
#include "pg_envmap.h"

#include <cmath>
#include <limits>

namespace pgh {

float roundToHalf(float f) {
    if (!std::isfinite(f) || f == 0.0f) return f;
    const float a = std::fabs(f);
    if (a >= 65520.0f) return std::copysign(std::numeric_limits<float>::infinity(), f);
    float q;
    if (a < 6.103515625e-05f) {
        q = 5.9604644775390625e-08f;  // 2^-24: the binary16 subnormal spacing
    } else {
        int e;
        std::frexp(a, &e);             // a = m 2^e, m in [0.5, 1): 11 significant bits -> spacing 2^(e - 11)
        q = std::ldexp(1.0f, e - 11);
    }
    return std::copysign(std::nearbyint(a / q) * q, f);  // ties to even (default rounding mode)
}

bool buildEnvTables(const pg_envmap &e, const float lo[3], const float hi[3], EnvTables &out, std::string &err) {
    const uint32_t W = e.width, H = e.height;
    if (!e.rgb || W < 1 || H < 1 || W > 0xFFFF || H > 0xFFFF) {  // envmap.cpp:161-163
        err = "envmap: empty image or a side >= 65536";
        return false;
    }
    for (int k = 0; k < 9; ++k)
        if (!std::isfinite(e.to_world[k])) {
            err = "envmap: non-finite to_world";
            return false;
        }
    if (!(e.scale >= 0) || !std::isfinite(e.scale)) {
        err = "envmap: scale must be finite and >= 0";
        return false;
    }
    out.width = W;
    out.height = H;
    out.scale = e.scale;
    for (int k = 0; k < 9; ++k) out.R[k] = e.to_world[k];
    out.texels.assign((size_t)W * H * 4, 0.0f);
    for (size_t i = 0; i < (size_t)W * H; ++i)
        for (int ch = 0; ch < 3; ++ch) {
            float v = e.rgb[3 * i + ch];
            if (!std::isfinite(v)) {
                err = "envmap: the image contains an invalid floating point value";
                return false;
            }
            out.texels[4 * i + ch] = roundToHalf(std::max(v, 0.0f));  // clampNegative, then half storage
        }
    // marginal & conditional CDFs over sin(theta)-weighted luminance (envmap.cpp:279-310)
    out.cdf_cols.assign((size_t)(W + 1) * H, 0.0f);
    out.cdf_rows.assign(H + 1, 0.0f);
    out.row_weights.assign(H, 0.0f);
    size_t colPos = 0, rowPos = 0;
    float rowSum = 0.0f;
    out.cdf_rows[rowPos++] = 0;
    for (uint32_t y = 0; y < H; ++y) {
        float colSum = 0;
        out.cdf_cols[colPos++] = 0;
        for (uint32_t x = 0; x < W; ++x) {
            const float *t = &out.texels[4 * ((size_t)y * W + x)];
            colSum += t[0] * 0.212671f + t[1] * 0.715160f + t[2] * 0.072169f;
            out.cdf_cols[colPos++] = colSum;
        }
        if (colSum > 0) {
            const float normalization = 1.0f / colSum;
            for (uint32_t x = 1; x < W; ++x) out.cdf_cols[colPos - x - 1] *= normalization;
        } else {
            // a black row never gets picked (zero marginal mass); the reference divides by 0 here,
            // a uniform row keeps its conditional CDF finite
            for (uint32_t x = 1; x < W; ++x) out.cdf_cols[colPos - x - 1] = (float)(W - x) / (float)W;
        }
        out.cdf_cols[colPos - 1] = 1.0f;
        const float weight = (float)std::sin((y + 0.5f) * M_PI / H);
        out.row_weights[y] = weight;
        rowSum += colSum * weight;
        out.cdf_rows[rowPos++] = rowSum;
    }
    if (!(rowSum > 0)) {
        err = "envmap: the environment map is completely black";
        return false;
    }
    if (!std::isfinite(rowSum)) {
        err = "envmap: the image contains an invalid floating point value";
        return false;
    }
    const float normalization = 1.0f / rowSum;
    for (uint32_t y = 1; y < H; ++y) out.cdf_rows[rowPos - y - 1] *= normalization;
    out.cdf_rows[rowPos - 1] = 1.0f;
    out.normalization = (float)(1.0f / (rowSum * (2 * M_PI / W) * (M_PI / H)));
    out.pixel_size[0] = (float)(2 * M_PI / W);
    out.pixel_size[1] = (float)(M_PI / H);
    // createShape (envmap.cpp:331-356): the scene AABB's bounding sphere, radius x 1.5
    float r2 = 0;
    for (int a = 0; a < 3; ++a) {
        out.center[a] = (lo[a] + hi[a]) * 0.5f;
        const float d = hi[a] - out.center[a];
        r2 += d * d;
    }
    out.radius = std::max(1e-4f, std::sqrt(r2) * 1.5f);
    return true;
}

}  // namespace pgh
