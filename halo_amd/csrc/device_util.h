// device_util.h — wave-level building blocks shared by the gfx950 kernels (rx_parse.hip,
// tx_fixup.hip): one's-complement folds, group broadcast / reduction over DPP, and the
// global-address-space 16-byte frame load. gfx950 (CDNA4, wave64) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace halo {
namespace {

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }

// fold a 32-bit sum to 16 bits, as protocol/utils.go:26-28 (two steps suffice for 32 bits)
__device__ __forceinline__ uint32_t fold16(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    return (s & 0xFFFFu) + (s >> 16);
}
// fold a 64-bit sum to < 2^18 keeping its value mod 0xFFFF and its zero-ness
__device__ __forceinline__ uint32_t fold64(uint64_t s) {
    uint64_t t = (s & 0xFFFFFFFFull) + (s >> 32);
    return (uint32_t)((t & 0xFFFFull) + (t >> 16));
}
__device__ __forceinline__ uint32_t hsum(uint32_t w) { return (w & 0xFFFFu) + (w >> 16); }

// DPP controls (gfx9 encoding): quad_perm, row_half_mirror, row_mirror, row_newbcast
constexpr int kDppQuadBcast(int k) { return k | (k << 2) | (k << 4) | (k << 6); }
constexpr int kDppHalfMirror = 0x141, kDppMirror = 0x140, kDppRowNewBcast0 = 0x150;

// value of `x` in lane k of this lane's group of G lanes
template <int G, int K>
__device__ __forceinline__ uint32_t group_bcast(uint32_t x, uint32_t grp_base) {
    if constexpr (G == 4) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppQuadBcast(K), 0xF, 0xF, false);
    } else if constexpr (G == 16) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppRowNewBcast0 + K, 0xF, 0xF, false);
    } else if constexpr (G == 64) {
        return (uint32_t)__builtin_amdgcn_readlane((int)x, K);
    } else {
        return (uint32_t)__shfl((int)x, (int)(grp_base + K), 64);
    }
}

// sum of `x` over this lane's group of G lanes, in every lane of the group
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
    if constexpr (G >= 2) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    if constexpr (G >= 4) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    if constexpr (G >= 8) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppHalfMirror, 0xF, 0xF, false);
    if constexpr (G >= 16) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kDppMirror, 0xF, 0xF, false);
    if constexpr (G >= 32) x += (uint32_t)__shfl_xor((int)x, 16, 64);
    if constexpr (G >= 64) x += (uint32_t)__shfl_xor((int)x, 32, 64);
    return x;
}

// Load dwords [d0, d0+4) of a frame that has ndw readable dwords; zero beyond. Never touches a
// dword past the one holding the frame's last byte (halo_rx.h layout contract).
// Frame bytes are always in global memory: say so, so that a pointer that came through LDS or a
// register still compiles to global_load (a flat_load would also count against lgkmcnt and make
// every later LDS access wait for it).
typedef const __attribute__((address_space(1))) uint32_t gu32;

// load4 with a non-temporal hint on the 16-byte path (bytes read once: not kept in the L2 ahead
// of lines another group will read)
__device__ __forceinline__ void load4_nt(const uint8_t* frame, uint32_t d0, uint32_t ndw, uint32_t (&w)[4]) {
    gu32* p = (gu32*)(reinterpret_cast<const uint32_t*>(frame) + d0);
    if (d0 + 4 <= ndw) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
        const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)p);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (d0 + j < ndw) ? p[j] : 0u;
    }
}
__device__ __forceinline__ void load4(const uint8_t* frame, uint32_t d0, uint32_t ndw, uint32_t (&w)[4]) {
    gu32* p = (gu32*)(reinterpret_cast<const uint32_t*>(frame) + d0);
    if (d0 + 4 <= ndw) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));  // 4-byte aligned 16 B
#if HALO_RX_NT_LOADS
        const u32x4 v = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)p);
#else
        const u32x4 v = *(const __attribute__((address_space(1))) u32x4*)p;
#endif
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (d0 + j < ndw) ? p[j] : 0u;
    }
}

}  // namespace
}  // namespace halo
