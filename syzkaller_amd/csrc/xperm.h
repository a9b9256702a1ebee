// xperm.h — lane exchanges v(lane ^ M) for the masks a 64-lane bitonic
// network needs, in VALU form (no LDS): DPP patterns for masks inside a row
// of 16 lanes, v_permlane16_swap / v_permlane32_swap (gfx950) across rows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace syz {

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

enum : int {
    DPP_QP_XOR1 = 0xB1,        // quad_perm [1,0,3,2]
    DPP_QP_XOR2 = 0x4E,        // quad_perm [2,3,0,1]
    DPP_QP_XOR3 = 0x1B,        // quad_perm [3,2,1,0]
    DPP_ROW_MIRROR = 0x140,    // lane ^ 15 within a row
    DPP_ROW_HALF_MIRROR = 0x141,  // lane ^ 7 within 8 lanes
};

// lane ^ 16: odd rows of the first operand swap with even rows of the second
__device__ __forceinline__ uint32_t xor16(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (__lane_id() & 16) ? r[0] : r[1];
}

// lane ^ 32: upper half of the first operand swaps with lower half of the second
__device__ __forceinline__ uint32_t xor32(uint32_t v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (__lane_id() & 32) ? r[0] : r[1];
}

template <int M>
__device__ __forceinline__ uint32_t xperm(uint32_t v) {
    if constexpr (M == 1) return dpp<DPP_QP_XOR1>(v);
    else if constexpr (M == 2) return dpp<DPP_QP_XOR2>(v);
    else if constexpr (M == 3) return dpp<DPP_QP_XOR3>(v);
    else if constexpr (M == 4) return dpp<DPP_QP_XOR3>(dpp<DPP_ROW_HALF_MIRROR>(v));  // ^7 ^3
    else if constexpr (M == 7) return dpp<DPP_ROW_HALF_MIRROR>(v);
    else if constexpr (M == 8) return dpp<DPP_ROW_HALF_MIRROR>(dpp<DPP_ROW_MIRROR>(v));  // ^15 ^7
    else if constexpr (M == 15) return dpp<DPP_ROW_MIRROR>(v);
    else if constexpr (M == 16) return xor16(v);
    else if constexpr (M == 31) return xor16(dpp<DPP_ROW_MIRROR>(v));
    else if constexpr (M == 32) return xor32(v);
    else if constexpr (M == 63) return xor32(xor16(dpp<DPP_ROW_MIRROR>(v)));
    else return __shfl_xor(v, M, 64);  // not needed by the networks here
}

}  // namespace syz

namespace syz {
// Lane l receives v of lane l-1; lane 0 receives `first` (DPP wave_shr:1).
__device__ __forceinline__ uint32_t shift_up(uint32_t v, uint32_t first) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xF, 0xF, false);
}
// Lane l receives v of lane l-1, lane 0 that of lane 63 (DPP wave_ror:1).
__device__ __forceinline__ uint32_t rotate_up(uint32_t v) {
    // (mov_dpp with bound_ctrl: no `old` operand, which update_dpp copies
    // into the destination first although every lane has a source)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, true);
}
}  // namespace syz
