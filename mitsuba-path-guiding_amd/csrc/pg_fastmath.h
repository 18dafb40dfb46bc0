// math::fastlog / math::fastexp as the reference builds them on Linux x86_64
// (include/mitsuba/core/math.h:175-199): the double-precision libm call rounded to float.  The result
// is the correctly rounded float log / exp except for double rounding, so oracle (glibc) and kernels
// agree whenever both evaluate the double function to well under half a float ulp.  The device
// library's logf rounds differently from it on 39 % of the tracking loops' arguments
// (profiles/r05x_fastlog/log_rounding.json); its double log never does, but costs ~70 FP64
// instructions.  `fastlog` below evaluates the double log to ~2^-52 relative in ~20 FP64 operations
// for positive normal arguments and equals (float)log((double)x) on every tracking argument and on
// 22 M sampled positive floats (same file).
//
// The tracking loops (heterogeneous.cpp:568,634) use `trackLog`: the device library's logf by default.
// With fastlog there, C5 runs at 407 against 445 Mpaths/s (the FP64 temporaries push k_vflight from 0
// to 68 B/lane of scratch and k_vvertex's surface launch from 156 to 304, profiles/r05x_fastlog/), while
// the C5 image-level parity prints are the same with either (every smoke pixel within 1e-3 of the
// oracle's, the same-tree renders 0.999 / 1.000, identical record counts): a tracking step's distance
// differs by an ulp where the roundings differ, and paths almost never part ways over it.
// PG_TRACK_FASTLOG=1 builds the tracking loops with fastlog (unit tests then match the oracle bit for bit).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

// log(x) for float x, rounded to float exactly as (float)log((double)x) but for ties within ~2^-52
__device__ __forceinline__ float fastlog(float x) {
#if PG_FASTLOG_LIBM  // A/B: the device library's double log (tools/r05x_gpu.sh ab/dbl)
    return (float)log((double)x);
#endif
    // special arguments without the library call (whose inlined body would cost registers at every
    // call site): 0 -> -inf, negative / NaN -> NaN, +inf -> +inf; denormals are scaled by 2^23 (exact)
    if (!(x > 0.0f) || x == __int_as_float(0x7f800000)) return x == 0.0f ? -__int_as_float(0x7f800000) : x * (x > 0.0f ? 1.0f : __int_as_float(0x7fc00000));
    const bool den = x < 0x1p-126f;
    const uint32_t b = __float_as_uint(den ? x * 0x1p23f : x);
    int e = (int)(b >> 23) - (den ? 150 : 127);
    uint32_t mb = (b & 0x007FFFFFu) | 0x3F800000u;  // m in [1, 2)
    if (mb > 0x3FB504F3u) {                          // m in [sqrt(2)/2, sqrt(2)): |s| <= 0.1716
        mb -= 0x00800000u;
        e += 1;
    }
    const double f = (double)(__uint_as_float(mb) - 1.0f);  // exact (Sterbenz)
    const double d = 2.0 + f;                               // exact
    // s = f / d: a float reciprocal seed, then two residual steps in double (error ~2^-53)
    const double r = (double)__builtin_amdgcn_rcpf((float)d);
    double s = f * r;
    s = fma(fma(-s, d, f), r, s);
    s = fma(fma(-s, d, f), r, s);
    // log(m) = 2 atanh(s) = 2s + s z P(z), z = s^2 <= 0.02944; ten terms leave < 2^-55 relative
    const double z = s * s;
    double p = 2.0 / 21;
    p = fma(p, z, 2.0 / 19);
    p = fma(p, z, 2.0 / 17);
    p = fma(p, z, 2.0 / 15);
    p = fma(p, z, 2.0 / 13);
    p = fma(p, z, 2.0 / 11);
    p = fma(p, z, 2.0 / 9);
    p = fma(p, z, 2.0 / 7);
    p = fma(p, z, 2.0 / 5);
    p = fma(p, z, 2.0 / 3);
    const double lm = fma(s * z, p, 2.0 * s);
    return (float)fma((double)e, 0.69314718055994530942, lm);
}
__device__ __forceinline__ float fastexp(float x) { return (float)exp((double)x); }

#ifndef PG_TRACK_FASTLOG
#define PG_TRACK_FASTLOG 0
#endif
// the tracking loops' log(1 - u) (see above)
__device__ __forceinline__ float trackLog(float x) {
#if PG_TRACK_FASTLOG
    return fastlog(x);
#else
    return logf(x);
#endif
}
