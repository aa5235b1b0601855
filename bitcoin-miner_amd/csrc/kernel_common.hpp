// kernel_common.hpp -- device helpers shared by the search kernels
// (search_kernels.hip) and the fast run kernel (fast_search.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.hpp"

namespace mh {
namespace dev {


__device__ __forceinline__ bool lex_less(uint64_t ha, uint64_t na, uint64_t hb, uint64_t nb) {
    return ha < hb || (ha == hb && na < nb);
}

// One exchange step of the wave reduction: the partner's (hash, nonce),
// fetched dword by dword by a DPP move (CTRL < 0x200: CTRL is the dpp_ctrl)
// or by a ds_swizzle (CTRL >= 0x200: the swizzle offset is CTRL - 0x200).
template <int CTRL>
__device__ __forceinline__ uint32_t xlane(uint32_t v) {
    if constexpr (CTRL < 0x200)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
    else
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, CTRL - 0x200);
}

template <int CTRL>
__device__ __forceinline__ void wave_step(uint64_t& h, uint64_t& n) {
    const uint64_t oh = ((uint64_t)xlane<CTRL>((uint32_t)(h >> 32)) << 32) | xlane<CTRL>((uint32_t)h);
    const uint64_t on = ((uint64_t)xlane<CTRL>((uint32_t)(n >> 32)) << 32) | xlane<CTRL>((uint32_t)n);
    if (lex_less(oh, on, h, n)) {
        h = oh;
        n = on;
    }
}

// Wave-wide minimum of a u32 (every lane active): DPP butterfly within each
// 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror),
// then the four rows' minima through readlane and scalar mins.  Wave-uniform.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return min(min(a, b), min(c, d));
}

// Workgroup lexicographic min; the result is valid in thread 0.
// Wave level: DPP quad_perm [1,0,3,2] and [2,3,0,1], row_half_mirror,
// row_mirror (each step joins two groups whose lanes already agree, so after
// it every lane of the doubled group holds its min), then ds_swizzle xor 16
// (bit mode, within 32 lanes), then lane 0 takes lane 32's value.  Then LDS
// across the workgroup's waves.
template <int NT = kBlockThreads>
__device__ __forceinline__ void block_min(uint64_t& h, uint64_t& n) {
    wave_step<0xB1>(h, n);              // quad_perm [1,0,3,2]: lane ^ 1
    wave_step<0x4E>(h, n);              // quad_perm [2,3,0,1]: lane ^ 2
    wave_step<0x141>(h, n);             // row_half_mirror: quads of 8 lanes
    wave_step<0x140>(h, n);             // row_mirror: halves of 16-lane rows
    wave_step<0x200 + 0x401F>(h, n);    // ds_swizzle and 0x1F, xor 0x10: rows 0<->1, 2<->3
    {
        const uint64_t oh = ((uint64_t)__builtin_amdgcn_readlane((int)(h >> 32), 32) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)h, 32);
        const uint64_t on = ((uint64_t)__builtin_amdgcn_readlane((int)(n >> 32), 32) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)n, 32);
        if (lex_less(oh, on, h, n)) {
            h = oh;
            n = on;
        }
    }
    __shared__ uint64_t sh[NT / 64], sn[NT / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) {
        sh[wv] = h;
        sn[wv] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 1; i < NT / 64; ++i)
            if (lex_less(sh[i], sn[i], h, n)) {
                h = sh[i];
                n = sn[i];
            }
    }
}

// w[wi] += v for a word index that is not a compile-time constant, without
// dynamic register indexing (which would go to scratch).
template <int NW>
__device__ __forceinline__ void add_word(uint32_t (&w)[NW], uint32_t wi, uint32_t v) {
#pragma unroll
    for (int x = 0; x < NW; ++x) w[x] += (wi == (uint32_t)x) ? v : 0u;
}

}  // namespace dev
}  // namespace mh
