// come_wave.h -- wavefront-level helpers shared by the kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>

namespace come {

// One stage of the 64-lane sum.  Stage s adds the partner group that differs in lane bit s, so
// the tree is the xor butterfly over offsets 1, 2, 4, 8, 16, 32 (the oracle's WAVE64 order).
// After each stage every lane of a group holds the same value (a + b == b + a bit for bit), so
// any partner in the other group gives the same sum: DPP quad_perm for bits 0-1, row_half_mirror
// / row_mirror for bits 2-3, and gfx950's v_permlane16_swap / v_permlane32_swap for bits 4-5
// (all VALU: no LDS round trip, unlike ds_bpermute).
template <int S>
__device__ inline float reduce_stage(float p) {
    const int x = __float_as_int(p);
    if constexpr (S == 0) return p + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
    if constexpr (S == 1) return p + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
    if constexpr (S == 2) return p + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));
    if constexpr (S == 3) return p + __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));
    if constexpr (S == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return __int_as_float(r[0]) + __int_as_float(r[1]);  // lower row + upper row, every lane
    }
    if constexpr (S == 5) {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return __int_as_float(r[0]) + __int_as_float(r[1]);  // lower half + upper half
    }
    return p;
}

}  // namespace come
