// wave_scan.hpp -- wave64 prefix sums in VALU (DPP), for gfx950.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mbrwt {

#if defined(__HIP_DEVICE_COMPILE__)
// Inclusive prefix sum over the 64 lanes of a wave (every lane active): a
// Hillis-Steele scan inside each row of 16 lanes (DPP row_shr 1, 2, 4, 8),
// then the rows joined by the gfx9 row broadcasts (lane 15 of each row into
// rows 1 and 3, lane 31 into rows 2 and 3).  Six DPP adds and no LDS: the
// shfl_up form compiles to six DEPENDENT ds_bpermute round trips, which under
// a persistent kernel's LDS traffic cost ~3.9k cycles per 64-row tile
// (k_traverse_rows phase stamps, profiles/r05).  A lane whose DPP source is
// outside its row (or whose row the mask excludes) adds the `old` operand, 0.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
#else
__device__ uint32_t wave_incl_sum(uint32_t x);  // (the host pass only parses the kernels)
#endif

}  // namespace mbrwt
