// Rough dielectric transmittance tables for roughplastic (host, computed at scene upload).
//
// The reference ships them precomputed (data/microfacet/*.dat, written by src/utils/rdielprec.cpp
// and reduced to a 1D slice by src/bsdfs/rtrans.h setEta/setAlpha for constant-roughness
// materials, roughplastic.cpp:283-299).  Here the same quantities are integrated directly at the
// material's (eta, alpha):
//   table[j] = T(cos theta = t_j^4), t_j = j / (N - 1) (t_0 = 0.1 / (N - 1), rdielprec.cpp:87-90),
//   T(wi)    = hemispherical transmittance of the rough dielectric interface (transmission-only
//              sample weight of roughdielectric.cpp:431-518 in importance mode, integrated over the
//              sample square),
//   fdr_int  = 1 - clamp(int_0^1 2 x T_int(x) dx) with T_int the table at 1/eta
//              (rdielprec.cpp:54-58 + RoughTransmittance::evalDiffuse).
// tests/test_rtrans.py pins both against the reference's .dat slices.
#pragma once
#include <stdint.h>

namespace pgh {

constexpr int kRoughTransSamples = 100;  // RESOLUTION_THETA of rdielprec.cpp

// dist: PG_DIST_*; returns the external table (kRoughTransSamples floats) and the internal
// diffuse Fresnel reflectance Fdr used by roughplastic's diffuse normalisation.
void roughTransmittance(int dist, float alpha, float eta, float *table, float *fdrInt);

// Mitsuba's evalCubicInterp1D over [0, 1] (src/libcore/spline.cpp:23-60)
float cubicInterp1D(float x, const float *values, int size);

}  // namespace pgh
