// Host-side tables of the environment emitter (EnvironmentMap::configure, envmap.cpp:260-329), built
// once at scene upload and copied to the device (GEnv, pg_layout.h).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/pg_capi.h"

namespace pgh {

struct EnvTables {
    uint32_t width = 0, height = 0;
    std::vector<float> texels;       // width * height * 4: rgb at half precision, 0
    std::vector<float> cdf_rows;     // height + 1
    std::vector<float> cdf_cols;     // height * (width + 1)
    std::vector<float> row_weights;  // height
    float normalization = 0, pixel_size[2] = {0, 0};
    float center[3] = {0, 0, 0}, radius = 0;
    float R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    float scale = 1;
};

// IEEE binary16 round-to-nearest-even of a float, returned as float (the MIP map's SpectrumHalf storage)
float roundToHalf(float f);

// Validates `e` and fills `out`; lo/hi = the scene AABB (the bounding sphere's box).  false + err on
// bad input (empty, non-finite, all black: envmap.cpp:312-316 rejects the last two as well).
bool buildEnvTables(const pg_envmap &e, const float lo[3], const float hi[3], EnvTables &out, std::string &err);

}  // namespace pgh
