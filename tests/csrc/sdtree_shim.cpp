// Test-only shim: the library's host SD-tree refit (mitsuba-path-guiding_amd/csrc/pg_sdtree.cpp)
// driven from a serialized tree, so tests/test_sdtree_host_refit.py can compare it with the oracle's
// refit on the CPU (pg_refit itself needs a device context).
#include <cstring>

#include "../../mitsuba-path-guiding_amd/csrc/pg_sdtree.h"

extern "C" int shim_refit(const uint8_t *blob, size_t n, uint32_t iter, float sthr, float rho, int max_depth,
                          int learn, uint8_t *out, size_t cap, size_t *out_n) {
    pgh::SdTree t;
    if (!t.deserialize(blob, n)) return 1;
    t.refit(iter, sthr, rho, max_depth, learn != 0);
    std::vector<uint8_t> v = t.serialize();
    *out_n = v.size();
    if (out && cap >= v.size()) std::memcpy(out, v.data(), v.size());
    return 0;
}
