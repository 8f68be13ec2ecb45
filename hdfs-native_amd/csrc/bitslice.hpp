// bitslice.hpp -- the 8x8 bit transpose behind the bit-sliced GF(2^8)
// multiply (xor_networks.hpp): 8 dwords d[0..7] hold 4 independent 8x8 bit
// matrices, one per byte lane y (row w = byte y of d[w], column b = bit b).
// transpose8 turns them into bit planes -- after it, d[b] byte y bit w = bit b
// of byte y of the original d[w] -- and, being a transpose, is its own
// inverse: run on the output planes it yields the output bytes in place.
// Three delta-swap stages (4x4, 2x2, 1x1 blocks), 4 VALU per swap (two
// shifts, two bit-field inserts), 48 per 8 dwords.
#pragma once

#include <cstdint>

namespace hec {
namespace bitslice {

// m ? a : b, bitwise (v_bfi_b32 / v_bitop3_b32 0xCA on the device)
__host__ __device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(m, a, b, 0xCA);
#else
    return (m & a) | (~m & b);
#endif
}

// rows (lo, hi = lo + step): exchange bits [s, 2s) of each 2s-bit field of
// lo with bits [0, s) of the same field of hi
template <int S>
__host__ __device__ __forceinline__ void delta_swap(uint32_t& lo, uint32_t& hi, uint32_t m) {
    const uint32_t x = lo >> S;  // lo's upper half-fields, moved down
    const uint32_t y = hi << S;  // hi's lower half-fields, moved up
    hi = bfi(m, x, hi);
    lo = bfi(m << S, y, lo);
}

__host__ __device__ __forceinline__ void transpose8(uint32_t (&d)[8]) {
#pragma unroll
    for (int w = 0; w < 4; w++) delta_swap<4>(d[w], d[w + 4], 0x0F0F0F0Fu);
#pragma unroll
    for (int w = 0; w < 8; w += 4) {
        delta_swap<2>(d[w], d[w + 2], 0x33333333u);
        delta_swap<2>(d[w + 1], d[w + 3], 0x33333333u);
    }
#pragma unroll
    for (int w = 0; w < 8; w += 2) delta_swap<1>(d[w], d[w + 1], 0x55555555u);
}

}  // namespace bitslice
}  // namespace hec
