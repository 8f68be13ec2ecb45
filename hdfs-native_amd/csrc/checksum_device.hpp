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

#ifndef __HIPCC_RTC__  // hiprtc (jit.cpp) provides the HIP runtime itself
#include <hip/hip_runtime.h>
#endif

#include <cstdint>

#include "checksum_tables.hpp"

namespace hec {
namespace crcdev {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// a ^ b ^ c as one v_bitop3_b32 (hipcc mostly emits two v_xor_b32)
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// 8 message bytes (lo = bytes 0..3, hi = 4..7 as little-endian words).  An
// MSB-first register meets the same index pattern byte-swapped.
template <bool REFL>
__device__ __forceinline__ uint32_t step8(const uint32_t (*t)[256], uint32_t crc, uint32_t lo, uint32_t hi) {
    lo ^= REFL ? crc : __builtin_bswap32(crc);
    // 8 lookups folded with 3-input XORs (4 VALU ops instead of 7)
    return x3(x3(x3(t[7][lo & 0xFF], t[6][(lo >> 8) & 0xFF], t[5][(lo >> 16) & 0xFF]), t[4][lo >> 24],
                 t[3][hi & 0xFF]),
              t[2][(hi >> 8) & 0xFF], t[1][(hi >> 16) & 0xFF]) ^
           t[0][hi >> 24];
}

// r -> the register state after appending the zero bytes the table encodes
__device__ __forceinline__ uint32_t apply_shift(const uint32_t (*t)[256], uint32_t r) {
    return x3(t[0][r & 0xFF], t[1][(r >> 8) & 0xFF], t[2][(r >> 16) & 0xFF]) ^ t[3][r >> 24];
}

// 8 message bytes through the 11-bit field tables (checksum_tables.hpp w11),
// packed in LDS at word offsets 0, 2048, 4096, 5120, 7168, 9216.  Each
// field's byte offset into its table is one VALU op on its word.
__device__ __forceinline__ uint32_t w11_off0(uint32_t w) { return w & 0x1FFCu; }
__device__ __forceinline__ uint32_t w11_off1(uint32_t w) { return (w >> 11) & 0x1FFCu; }
__device__ __forceinline__ uint32_t w11_off2(uint32_t w) { return __builtin_rotateright32(w, 22) & 0xFFCu; }

template <bool REFL>
__device__ __forceinline__ uint32_t step8_w11(const uint32_t* t, uint32_t crc, uint32_t lo, uint32_t hi) {
    lo ^= REFL ? crc : __builtin_bswap32(crc);
    const char* tb = reinterpret_cast<const char*>(t);
    auto at = [&](int word_off, uint32_t byte_off) {
        return *reinterpret_cast<const uint32_t*>(tb + word_off * 4 + byte_off);
    };
    return x3(x3(at(0, w11_off0(lo)), at(2048, w11_off1(lo)), at(4096, w11_off2(lo))), at(5120, w11_off0(hi)),
              at(7168, w11_off1(hi))) ^
           at(9216, w11_off2(hi));
}

template <bool REFL>
__device__ __forceinline__ uint32_t quarter_w11(const uint32_t* t, const uint8_t* row) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const v4u w = *reinterpret_cast<const v4u*>(row + i * 16);
        r = step8_w11<REFL>(t, r, w.x, w.y);
        r = step8_w11<REFL>(t, r, w.z, w.w);
    }
    return r;
}

// Scheme 12: fold, then 11-bit slicing over the last 32 B only.  CRC is the
// remainder mod P, and Q(x) = x^209 + x^144 + x^54 + x^39 + x^14 + 1 is a
// multiple of the CRC32C polynomial (found by a collision search over
// residues x^t mod P; CRC32C's Hamming distance 6 up to 5243 bits rules out
// sparser ones this short).  So a message bit at degree g >= 209 equals the
// five bits at degrees g - 209 + {0, 14, 39, 54, 144}: in a reflected
// register (bit b of little-endian dword j = message position 32j + b) it
// moves 209, 195, 170, 155 and 65 positions later.  Folding dwords 0..23 of
// the quarter forward that way (one v_alignbit per source pair and offset,
// 3-input XORs) leaves a 256-bit message with the same remainder: its
// linear CRC from state 0 is the quarter's.  4 steps = 24 lookups instead of
// 96, for ~120 more VALU.  Reflected (CRC32C) only; the MSB-first register
// keeps quarter_w11.  Checked bit for bit by tests/cpp/crc_tables_check.cpp.
struct Fold {
    static constexpr int kN = 5, kDwords = 24;                // offsets; folded dwords
    static constexpr int q[kN] = {6, 6, 5, 4, 2}, s[kN] = {17, 3, 10, 27, 1};  // offset = 32q + s
};

// FD = folded dwords (24: default, 256-bit tail; 16 / 20: measurement
// schemes 13 / 14, fewer v_alignbit, a 512- / 384-bit tail of lookups).  Any
// FD <= 25 is valid: a bit is folded only at degree >= 1024 - 32 FD >= 224 > 209.
// The quarter's 32 little-endian dwords, folded in place: dwords FD..31 then
// hold a message with the quarter's remainder.
template <int FD = Fold::kDwords>
__device__ __forceinline__ void fold_in_place(uint32_t (&w)[32]) {
    // target i takes (w[i-q] << s) | (w[i-q-1] >> (32-s)) from folded
    // sources only (indices < FD); sources are at i-2 or earlier, so every
    // source is final when a target reads it
#pragma unroll
    for (int i = 2; i < 32; i++) {
        uint32_t acc = w[i], pend = 0;
        bool has = false;
#pragma unroll
        for (int o = 0; o < Fold::kN; o++) {
            const int hi = i - Fold::q[o], lo = hi - 1;
            const bool h = hi >= 0 && hi < FD, l = lo >= 0 && lo < FD;
            if (!h && !l) continue;
            const uint32_t c = h && l ? __builtin_amdgcn_alignbit(w[hi], w[lo], 32 - Fold::s[o])
                               : h    ? w[hi] << Fold::s[o]
                                      : w[lo] >> (32 - Fold::s[o]);
            if (has) {
                acc = x3(acc, pend, c);
                has = false;
            } else {
                pend = c;
                has = true;
            }
        }
        w[i] = has ? acc ^ pend : acc;
    }
}

template <bool REFL, int FD = Fold::kDwords>
__device__ __forceinline__ uint32_t quarter_fold(const uint32_t* t, const uint8_t* row) {
    static_assert(FD % 2 == 0 && FD >= 2 && FD <= 24, "even fold depth, 256-bit tail at least");
    if constexpr (!REFL) {
        return quarter_w11<REFL>(t, row);
    } else {
        uint32_t w[32];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const v4u v = *reinterpret_cast<const v4u*>(row + i * 16);
            w[4 * i] = v.x, w[4 * i + 1] = v.y, w[4 * i + 2] = v.z, w[4 * i + 3] = v.w;
        }
        fold_in_place<FD>(w);
        uint32_t r = 0;
#pragma unroll
        for (int i = FD; i < 32; i += 2) r = step8_w11<REFL>(t, r, w[i], w[i + 1]);
        return r;
    }
}

// The fold of a quarter already in registers, its 32-B tail through the
// slicing-by-8 tables t[8][256] (8 KiB: the LDS-DMA CRC kernel, whose stages
// leave no room for the 40-KiB 11-bit tables at 3 stages per wave).  CRC32C.
__device__ __forceinline__ uint32_t quarter_fold_regs_s8(uint32_t (&w)[32], const uint32_t (*t)[256]) {
    fold_in_place(w);
    uint32_t r = 0;
#pragma unroll
    for (int i = Fold::kDwords; i < 32; i += 2) r = step8<true>(t, r, w[i], w[i + 1]);
    return r;
}

// Scheme 15 (CRC32C; measurement build): the same fold, then the 256-bit
// tail through slicing-by-32 tables (checksum_tables.hpp Slice32, 32 KiB):
// 32 lookups with no dependency between them, one LDS round trip, where the
// 11-bit tail chains four (each step's index depends on the previous
// register).  t = the 32 x 256 tables in LDS.
template <bool REFL>
__device__ __forceinline__ uint32_t quarter_fold32(const uint32_t* t, const uint8_t* row) {
    static_assert(REFL, "the fold is for the reflected register");
    uint32_t w[32];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const v4u v = *reinterpret_cast<const v4u*>(row + i * 16);
        w[4 * i] = v.x, w[4 * i + 1] = v.y, w[4 * i + 2] = v.z, w[4 * i + 3] = v.w;
    }
    fold_in_place(w);
    // tail byte i (0..31) of dwords 24..31 -> t[31 - i][byte]
    uint32_t v[32];
#pragma unroll
    for (int d = 0; d < 8; d++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int i = 4 * d + b;
            v[i] = t[(31 - i) * 256 + ((w[Fold::kDwords + d] >> (8 * b)) & 0xFFu)];
        }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 32; i += 2) r = x3(r, v[i], v[i + 1]);
    return r;
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

// Bank-replicated slicing-by-2 (scheme 22): rep[k][e][b] at k*8192 + e*32 +
// b, b = lane % 32, so a half-wave's lookups are conflict free; rep[0] =
// slice[1] (the step's first byte), rep[1] = slice[0].  Four chains over the
// quarter's 32-B segments (latency), combined by Horner with the "append
// 32 zero bytes" table seg32.  An MSB-first register runs byte-swapped
// (tables stored byte-swapped) so that both kinds share the reflected step
// c' = T1[c & 0xFF] ^ T0[(c >> 8) & 0xFF] ^ (c >> 16).
template <bool REFL>
__device__ __forceinline__ uint32_t quarter_rep2(const uint32_t* s, const uint32_t (*seg32)[256], const uint8_t* row,
                                                 int bank) {
    const uint32_t* t0 = s + bank;
    const uint32_t* t1 = s + 8192 + bank;
    uint32_t c[4] = {0, 0, 0, 0};
#pragma unroll
    for (int ph = 0; ph < 2; ph++) {
        v4u w[4];
#pragma unroll
        for (int g = 0; g < 4; g++) w[g] = *reinterpret_cast<const v4u*>(row + g * 32 + ph * 16);
#pragma unroll
        for (int d = 0; d < 4; d++) {
#pragma unroll
            for (int g = 0; g < 4; g++) c[g] ^= w[g][d];
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int g = 0; g < 4; g++)
                    c[g] = x3(t0[(c[g] & 0xFF) * 32], t1[((c[g] >> 8) & 0xFF) * 32], c[g] >> 16);
        }
    }
    if constexpr (!REFL) {
#pragma unroll
        for (int g = 0; g < 4; g++) c[g] = __builtin_bswap32(c[g]);
    }
    uint32_t q = c[0];
#pragma unroll
    for (int g = 1; g < 4; g++) q = apply_shift(seg32, q) ^ c[g];
    return q;
}

// One byte through the register (tails): t0 = the classic table, read at
// idx * STRIDE words (1 for slice tables, 32 for the replicated table).
template <bool REFL, int STRIDE, bool BSWAP = false>
__device__ __forceinline__ uint32_t byte_step(const uint32_t* t0, uint32_t r, uint32_t b) {
    if constexpr (REFL) return t0[((r ^ b) & 0xFF) * STRIDE] ^ (r >> 8);
    const uint32_t t = t0[(((r >> 24) ^ b) & 0xFF) * STRIDE];
    return (BSWAP ? __builtin_bswap32(t) : t) ^ (r << 8);
}

// r -> shifted state from nibble tables t[8][16] (8 lookups instead of 4)
__device__ __forceinline__ uint32_t apply_shift_nib(const uint32_t (*t)[16], uint32_t r) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) v ^= t[q][(r >> (4 * q)) & 15];
    return v;
}

// Schemes: 15 = the fold + a slicing-by-32 tail (CRC32C, measurement);
// 1 = slicing-by-8 (256-thread blocks); 11 = 11-bit slicing (6
// lookups per 8 bytes from 40 KiB of tables, nibble shift tables; 256-thread
// blocks, 2 per CU); 16 = slicing-by-8 in
// 1024-thread blocks (4 waves per SIMD) with nibble shift tables so the
// tables (9.5 KiB) and 16 wave images (144 KiB) fit one CU's LDS; 4 / 8 =
// bank-replicated slicing-by-1; 0 = memory side only.
// 11-bit field tables: 11-bit slicing, the fold (12) and its depth variants (13, 14)
constexpr bool w11(int scheme) { return scheme >= 11 && scheme <= 14; }
constexpr bool sliced(int scheme) { return scheme <= 1 || scheme == 15 || scheme == 16 || w11(scheme); }
constexpr bool nib_shift(int scheme) { return scheme == 15 || scheme == 16 || w11(scheme); }

// slice[8][256] (schemes 1, 16) | rep[256][32] (schemes 4, 8) ; shift[3][4][256]
// (shift_nib[3][8][16] for scheme 16) ; seg[7][4][256] (schemes 4, 8)
// scheme 22: rep[2][256][32] ; seg32[4][256] ; shift[3][4][256] (80 KiB)
template <int SCHEME>
struct TableLayout {
    static constexpr int kMainWords = SCHEME == 22   ? 2 * 256 * 32 + 4 * 256
                                      : SCHEME == 15 ? 32 * 256
                                      : w11(SCHEME) ? 4 * 2048 + 2 * 1024
                                      : sliced(SCHEME) ? 8 * 256
                                                       : 256 * 32;
    static constexpr int kShiftOff = kMainWords;
    static constexpr int kShiftWords = nib_shift(SCHEME) ? 3 * 8 * 16 : 3 * 4 * 256;
    static constexpr int kSegOff = kShiftOff + kShiftWords;
    static constexpr int kWords = kSegOff + ((sliced(SCHEME) || SCHEME == 22) ? 0 : 7 * 4 * 256);
};

// Where the classic byte table (slice[0]) sits in a scheme's LDS image, for
// byte-serial tails: slice[0][x] = t[off + x * stride].  Scheme 11 has no
// byte table, but its field 5 (hi bits 24..31 + 0..1) holds it: byte 7 of
// the step is field bits 0..7, so slice[0][x] = w11[5][x].
template <int SCHEME>
struct ByteTable {
    static constexpr int off = w11(SCHEME) ? 9216 : SCHEME == 22 ? 8192 : 0;
    static constexpr int stride = sliced(SCHEME) ? 1 : 32;
    static constexpr bool bswap = SCHEME == 22;  // MSB-first kind: stored byte-swapped
};

// Moves quarter qi's linear CRC (qi < 3) to its place in the 512-B chunk.
template <int SCHEME>
__device__ __forceinline__ uint32_t shift_quarter(const uint32_t* s, int qi, uint32_t r) {
    if constexpr (nib_shift(SCHEME))
        return apply_shift_nib(reinterpret_cast<const uint32_t(*)[8][16]>(s + TableLayout<SCHEME>::kShiftOff)[qi], r);
    else
        return apply_shift(reinterpret_cast<const uint32_t(*)[4][256]>(s + TableLayout<SCHEME>::kShiftOff)[qi], r);
}

// Fills a block's LDS table image (TableLayout<SCHEME>) from the constant
// tables; caller synchronises.
template <int SCHEME, int BS, int KIND>
__device__ __forceinline__ void stage_tables(uint32_t* s, const crc::Tables<KIND>& tab) {
    if constexpr (SCHEME == 22) {
        constexpr bool REFL = crc::Spec<KIND>::kReflected;
        for (int t = threadIdx.x; t < 2 * 256 * 32; t += BS) {
            const uint32_t v = tab.slice[1 - t / 8192][(t / 32) % 256];
            s[t] = REFL ? v : __builtin_bswap32(v);
        }
        for (int t = threadIdx.x; t < 4 * 256; t += BS) s[2 * 256 * 32 + t] = (&tab.seg[5][0][0])[t];
    } else if constexpr (SCHEME == 15) {
        // the slicing-by-32 tables come from their own constant (stage_slice32)
    } else if constexpr (w11(SCHEME)) {
        constexpr int off[6] = {0, 2048, 4096, 5120, 7168, 9216}, len[6] = {2048, 2048, 1024, 2048, 2048, 1024};
#pragma unroll
        for (int f = 0; f < 6; f++)
            for (int t = threadIdx.x; t < len[f]; t += BS) s[off[f] + t] = tab.w11[f][t];
    } else if constexpr (sliced(SCHEME)) {
        for (int t = threadIdx.x; t < 8 * 256; t += BS) s[t] = (&tab.slice[0][0])[t];
    } else {
        for (int t = threadIdx.x; t < 256 * 32; t += BS) s[t] = tab.slice[0][t / 32];
        for (int t = threadIdx.x; t < 7 * 4 * 256; t += BS) s[TableLayout<SCHEME>::kSegOff + t] = (&tab.seg[0][0][0])[t];
    }
    if constexpr (nib_shift(SCHEME))
        for (int t = threadIdx.x; t < 3 * 8 * 16; t += BS) s[TableLayout<SCHEME>::kShiftOff + t] = (&tab.shift_nib[0][0][0])[t];
    else
        for (int t = threadIdx.x; t < 3 * 4 * 256; t += BS) s[TableLayout<SCHEME>::kShiftOff + t] = (&tab.shift[0][0][0])[t];
}

// Linear part of the quarter at `row` under the block's LDS tables.
template <int SCHEME, bool REFL>
__device__ __forceinline__ uint32_t quarter(const uint32_t* s, const uint8_t* row, int lane) {
    if constexpr (SCHEME == 22)
        return quarter_rep2<REFL>(s, reinterpret_cast<const uint32_t(*)[256]>(s + 2 * 256 * 32), row, lane & 31);
    else if constexpr (SCHEME == 11)
        return quarter_w11<REFL>(s, row);
    else if constexpr (SCHEME == 12)
        return quarter_fold<REFL>(s, row);
    else if constexpr (SCHEME == 13)
        return quarter_fold<REFL, 16>(s, row);
    else if constexpr (SCHEME == 14)
        return quarter_fold<REFL, 20>(s, row);
    else if constexpr (SCHEME == 15)
        return quarter_fold32<REFL>(s, row);
    else if constexpr (sliced(SCHEME))
        return quarter_s8<REFL>(reinterpret_cast<const uint32_t(*)[256]>(s), row);
    else
        return quarter_rep<SCHEME, REFL>(reinterpret_cast<const uint32_t(*)[32]>(s),
                                         reinterpret_cast<const uint32_t(*)[4][256]>(s + TableLayout<SCHEME>::kSegOff),
                                         row, lane & 31);
}

}  // namespace crcdev
}  // namespace hec
