// checksum_device.hpp -- per-lane chunk-checksum building blocks shared by
// the checksum kernels (checksum.hip) and the fused coding+checksum kernels
// (ec_kernels.hip).  A lane computes the linear part L of one 128-B QUARTER
// of a 512-B chunk from register state 0; callers place it in the chunk
// with the "append 384/256/128 zero bytes" tables and combine quarters by
// XOR (checksum_tables.hpp).  REFL = reflected (CRC32C) or MSB-first
// (CRC32 = CRC_32_CKSUM) register.
//   slicing-by-8 : 8 x 256-word tables, 1 random ds_read_b32 per byte
//   replicated   : one 256-entry table copied into all 32 banks of a
//                  ds_read_b32 half-wave (rep[e][b]); lane l reads column
//                  l%32, so lookups are bank-conflict free; the quarter runs
//                  as NCHAIN independent segment chains (latency) combined
//                  by the "append 16*(7-i) zero bytes" tables seg[i]
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "checksum_tables.hpp"

namespace hec {
namespace crcdev {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// 8 message bytes (lo = bytes 0..3, hi = 4..7 as little-endian words).  An
// MSB-first register meets the same index pattern byte-swapped.
template <bool REFL>
__device__ __forceinline__ uint32_t step8(const uint32_t (*t)[256], uint32_t crc, uint32_t lo, uint32_t hi) {
    lo ^= REFL ? crc : __builtin_bswap32(crc);
    return t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
           t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
}

// r -> the register state after appending the zero bytes the table encodes
__device__ __forceinline__ uint32_t apply_shift(const uint32_t (*t)[256], uint32_t r) {
    return t[0][r & 0xFF] ^ t[1][(r >> 8) & 0xFF] ^ t[2][(r >> 16) & 0xFF] ^ t[3][r >> 24];
}

template <bool REFL>
__device__ __forceinline__ uint32_t quarter_s8(const uint32_t (*tab)[256], const uint8_t* row) {
    uint32_t r = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const v4u w = *reinterpret_cast<const v4u*>(row + t * 16);
        r = step8<REFL>(tab, r, w.x, w.y);
        r = step8<REFL>(tab, r, w.z, w.w);
    }
    return r;
}

template <int NCHAIN, bool REFL>
__device__ __forceinline__ uint32_t quarter_rep(const uint32_t (*rep)[32], const uint32_t (*seg)[4][256],
                                                const uint8_t* row, int bank) {
    static_assert(NCHAIN == 4 || NCHAIN == 8, "4 or 8 chains");
    constexpr int SEGW = 32 / NCHAIN;  // dwords per segment
    constexpr int PH = SEGW / 4;       // 16-B row reads per segment = read phases
    uint32_t c[NCHAIN];
#pragma unroll
    for (int s = 0; s < NCHAIN; s++) c[s] = 0;
#pragma unroll
    for (int ph = 0; ph < PH; ph++) {
        // phase ph: the ph-th 16 B of every segment (keeps 16 B x NCHAIN live)
        v4u w[NCHAIN];
#pragma unroll
        for (int s = 0; s < NCHAIN; s++) w[s] = *reinterpret_cast<const v4u*>(row + s * SEGW * 4 + ph * 16);
#pragma unroll
        for (int d = 0; d < 4; d++) {
#pragma unroll
            for (int s = 0; s < NCHAIN; s++) c[s] ^= REFL ? w[s][d] : __builtin_bswap32(w[s][d]);
#pragma unroll
            for (int b = 0; b < 4; b++)
#pragma unroll
                for (int s = 0; s < NCHAIN; s++)
                    c[s] = REFL ? rep[c[s] & 0xFF][bank] ^ (c[s] >> 8) : rep[c[s] >> 24][bank] ^ (c[s] << 8);
        }
    }
    uint32_t q = c[NCHAIN - 1];
#pragma unroll
    for (int s = 0; s < NCHAIN - 1; s++) q ^= apply_shift(seg[7 - (NCHAIN - 1 - s) * (8 / NCHAIN)], c[s]);
    return q;
}

// One byte through the register (tails): t0 = the classic table, read at
// idx * STRIDE words (1 for slice tables, 32 for the replicated table).
template <bool REFL, int STRIDE>
__device__ __forceinline__ uint32_t byte_step(const uint32_t* t0, uint32_t r, uint32_t b) {
    return REFL ? t0[((r ^ b) & 0xFF) * STRIDE] ^ (r >> 8) : t0[(((r >> 24) ^ b) & 0xFF) * STRIDE] ^ (r << 8);
}

// slice[8][256] (scheme 1) | rep[256][32] (schemes 4, 8) ; shift[3][4][256] ;
// seg[7][4][256] (schemes 4, 8)
template <int SCHEME>
struct TableLayout {
    static constexpr int kMainWords = SCHEME <= 1 ? 8 * 256 : 256 * 32;
    static constexpr int kShiftOff = kMainWords;
    static constexpr int kSegOff = kShiftOff + 3 * 4 * 256;
    static constexpr int kWords = kSegOff + (SCHEME <= 1 ? 0 : 7 * 4 * 256);
};

// Fills a block's LDS table image (TableLayout<SCHEME>) from the constant
// tables; caller synchronises.
template <int SCHEME, int BS, typename T>
__device__ __forceinline__ void stage_tables(uint32_t* s, const T& tab) {
    if constexpr (SCHEME <= 1) {
        for (int t = threadIdx.x; t < 8 * 256; t += BS) s[t] = (&tab.slice[0][0])[t];
    } else {
        for (int t = threadIdx.x; t < 256 * 32; t += BS) s[t] = tab.slice[0][t / 32];
        for (int t = threadIdx.x; t < 7 * 4 * 256; t += BS) s[TableLayout<SCHEME>::kSegOff + t] = (&tab.seg[0][0][0])[t];
    }
    for (int t = threadIdx.x; t < 3 * 4 * 256; t += BS) s[TableLayout<SCHEME>::kShiftOff + t] = (&tab.shift[0][0][0])[t];
}

// Linear part of the quarter at `row` under the block's LDS tables.
template <int SCHEME, bool REFL>
__device__ __forceinline__ uint32_t quarter(const uint32_t* s, const uint8_t* row, int lane) {
    if constexpr (SCHEME <= 1)
        return quarter_s8<REFL>(reinterpret_cast<const uint32_t(*)[256]>(s), row);
    else
        return quarter_rep<SCHEME, REFL>(reinterpret_cast<const uint32_t(*)[32]>(s),
                                         reinterpret_cast<const uint32_t(*)[4][256]>(s + TableLayout<SCHEME>::kSegOff),
                                         row, lane & 31);
}

}  // namespace crcdev
}  // namespace hec
