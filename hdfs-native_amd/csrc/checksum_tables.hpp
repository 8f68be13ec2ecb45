// checksum_tables.hpp -- compile-time tables for the two DataTransferProtocol
// chunk checksums the reference implements (rust/src/hdfs/connection.rs:37-38,
// crc 3.4.0 / crc-catalog 2.4.0, Cargo.lock:375-387):
//   CRC32C = CRC_32_ISCSI : reflected, poly 0x1EDC6F41 (0x82F63B78 reversed),
//                           init 0xFFFFFFFF, xorout 0xFFFFFFFF, check 0xE3069283
//   CRC32  = CRC_32_CKSUM : MSB-first, poly 0x04C11DB7, init 0,
//                           xorout 0xFFFFFFFF, check 0x765E7680
// (ChecksumTypeProto CHECKSUM_CRC32C = 2 / CHECKSUM_CRC32 = 1,
// rust/src/proto/hadoop.hdfs.rs:1363; ReadPacket::get_data maps them at
// connection.rs:483-487.)
//
// Both are affine over GF(2): crc(M) = L(M) ^ A_len with L linear in the
// message bits.  The kernels compute L of 128-B quarters from register state
// 0 and move each to its place in the chunk with "append n zero bytes"
// tables (L of the zero-extended quarter).  Per kind:
//   slice[8][256]      slicing-by-8 byte tables (slice[0] = the classic table)
//   shift[3][4][256]   append 384/256/128 zero bytes, as byte tables: the
//                      register transform r -> state after n zero bytes is
//                      linear, so shift_n(r) = XOR_b shift[..][b][byte b of r]
//   seg[7][4][256]     the same for 112/96/.../16 zero bytes (seg[i] appends
//                      16*(7-i) bytes): combines 16- or 32-B segments of a quarter
//   final512           A_512 = zero_bytes(init, 512) ^ xorout: the affine
//                      constant of a full 512-byte chunk
// MSB-first step on little-endian words: the same slicing-by-8 index pattern
// as the reflected one once the register is byte-swapped before the XOR
// (checksum_device.hpp).
#pragma once

#include <cstdint>

namespace hec {
namespace crc {

enum Kind : int { kCrc32c = 0, kCksum = 1 };

template <int KIND>
struct Spec;
template <>
struct Spec<kCrc32c> {
    static constexpr bool kReflected = true;
    static constexpr uint32_t kPoly = 0x82F63B78u;  // reversed 0x1EDC6F41
    static constexpr uint32_t kInit = 0xFFFFFFFFu;
    static constexpr uint32_t kXorout = 0xFFFFFFFFu;
};
template <>
struct Spec<kCksum> {
    static constexpr bool kReflected = false;
    static constexpr uint32_t kPoly = 0x04C11DB7u;
    static constexpr uint32_t kInit = 0u;
    static constexpr uint32_t kXorout = 0xFFFFFFFFu;
};

template <int KIND>
struct Tables {
    using S = Spec<KIND>;
    uint32_t slice[8][256]{};
    uint32_t shift[3][4][256]{};  // [0] = 384 B, [1] = 256 B, [2] = 128 B
    uint32_t seg[7][4][256]{};    // [i] = 16*(7-i) B: 112, 96, ..., 16
    uint32_t shift_nib[3][8][16]{};  // shift[] as nibble tables (1.5 KiB: the 1024-thread CRC kernel)
    // 11-bit slicing: the 8-byte step's 64 message bits (lo = bytes 0-3, hi =
    // 4-7, little-endian) in six fields, three per word w: w[2:13],
    // w[13:24] and w[24:32] + w[0:2] (10 bits).  The fields sit where one
    // VALU op turns a word into a table byte offset (index * 4): w & 0x1FFC,
    // (w >> 11) & 0x1FFC, rotr(w, 22) & 0xFFC.  w11[f][x] = XOR of the
    // single-bit columns of the byte tables, slice[7 - j/8][1 << j%8] for
    // message bit j.  6 lookups per 8 bytes instead of 8.
    uint32_t w11[6][2048]{};
    uint32_t final512 = 0;

    // one byte through the register
    static constexpr uint32_t byte_step(const uint32_t* t0, uint32_t r, uint32_t b) {
        return S::kReflected ? t0[(r ^ b) & 0xFF] ^ (r >> 8) : t0[((r >> 24) ^ b) & 0xFF] ^ (r << 8);
    }

    static constexpr uint32_t zero_bytes(const uint32_t* t0, uint32_t r, int n) {
        for (int i = 0; i < n; i++) r = byte_step(t0, r, 0);
        return r;
    }

    static constexpr void zero_shift_table(const uint32_t* t0, int n, uint32_t (*out)[256]) {
        uint32_t col[32]{};
        for (int j = 0; j < 32; j++) col[j] = zero_bytes(t0, 1u << j, n);
        for (int b = 0; b < 4; b++)
            for (int x = 0; x < 256; x++) {
                uint32_t v = 0;
                for (int j = 0; j < 8; j++)
                    if (x & (1 << j)) v ^= col[8 * b + j];
                out[b][x] = v;
            }
    }

    constexpr Tables() {
        for (int i = 0; i < 256; i++) {
            uint32_t c = 0;
            if (S::kReflected) {
                c = uint32_t(i);
                for (int b = 0; b < 8; b++) c = (c >> 1) ^ (S::kPoly & (0u - (c & 1u)));
            } else {
                c = uint32_t(i) << 24;
                for (int b = 0; b < 8; b++) c = (c << 1) ^ (S::kPoly & (0u - (c >> 31)));
            }
            slice[0][i] = c;
        }
        for (int s = 1; s < 8; s++)
            for (int i = 0; i < 256; i++) slice[s][i] = zero_bytes(slice[0], slice[s - 1][i], 1);
        for (int k = 0; k < 3; k++) zero_shift_table(slice[0], 128 * (3 - k), shift[k]);
        for (int k = 0; k < 3; k++)  // nibble q of r: XOR of the byte table's single-bit columns
            for (int q = 0; q < 8; q++)
                for (int x = 0; x < 16; x++) {
                    uint32_t v = 0;
                    for (int b = 0; b < 4; b++)
                        if (x & (1 << b)) v ^= shift[k][q / 2][1 << (4 * (q % 2) + b)];
                    shift_nib[k][q][x] = v;
                }
        for (int i = 0; i < 7; i++) zero_shift_table(slice[0], 16 * (7 - i), seg[i]);
        for (int f = 0; f < 6; f++) {
            const int word = f / 3, bits = (f % 3) == 2 ? 10 : 11;
            for (int x = 0; x < (1 << bits); x++) {
                uint32_t v = 0;
                for (int b = 0; b < bits; b++) {
                    const int j = 32 * word + (f % 3 == 0 ? 2 + b : f % 3 == 1 ? 13 + b : (24 + b) % 32);
                    if (x & (1 << b)) v ^= slice[7 - j / 8][1 << (j % 8)];
                }
                w11[f][x] = v;
            }
        }
        final512 = zero_bytes(slice[0], S::kInit, 512) ^ S::kXorout;
    }
};

// Slicing-by-32 byte tables: t[j][x] = the register after byte x then j zero
// bytes from state 0 (t[0] = the classic table, t[1..7] = Tables::slice), so
// 32 bytes from state 0 fold to XOR_i t[31 - i][m_i] with no dependency
// between the lookups (the fused kernels' scheme 15 tail; measurement build).
template <int KIND>
struct Slice32 {
    uint32_t t[32][256]{};
    constexpr Slice32() {
        const Tables<KIND> base;
        for (int x = 0; x < 256; x++) t[0][x] = base.slice[0][x];
        for (int j = 1; j < 32; j++)
            for (int x = 0; x < 256; x++) t[j][x] = Tables<KIND>::zero_bytes(t[0], t[j - 1][x], 1);
    }
};

}  // namespace crc
}  // namespace hec
