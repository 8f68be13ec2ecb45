// crc32c_tables.hpp -- compile-time CRC32C (Castagnoli, reflected
// 0x82F63B78) tables for the device kernels:
//   kSlice[8][256]   slicing-by-8 byte tables (kSlice[0] = the classic table)
//   kShift[3][4][256] "append 384/256/128 zero bytes" as byte tables: the
//                     register transform r -> state after n zero bytes is
//                     linear, so shift_n(r) = XOR_b kShift[..][b][byte b of r]
//   seg[7][4][256]    the same for 112/96/.../16 zero bytes (seg[i] appends
//                     16*(7-i) bytes): combines 16- or 32-B segments of a
//                     128-B quarter
//   kFinal512        shift_512(0xFFFFFFFF) ^ 0xFFFFFFFF: the init/xorout
//                     constant of a full 512-byte chunk
#pragma once

#include <array>
#include <cstdint>

namespace hec {
namespace crc {

constexpr uint32_t kPoly = 0x82F63B78u;

struct Tables {
    uint32_t slice[8][256]{};
    uint32_t shift[3][4][256]{};  // [0] = 384 B, [1] = 256 B, [2] = 128 B
    uint32_t seg[7][4][256]{};    // [i] = 16*(7-i) B: 112, 96, ..., 16
    uint32_t final512 = 0;

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

    static constexpr uint32_t zero_bytes(const uint32_t* t0, uint32_t r, int n) {
        for (int i = 0; i < n; i++) r = t0[r & 0xFF] ^ (r >> 8);
        return r;
    }

    constexpr Tables() {
        for (int i = 0; i < 256; i++) {
            uint32_t c = uint32_t(i);
            for (int b = 0; b < 8; b++) c = (c >> 1) ^ (kPoly & (0u - (c & 1u)));
            slice[0][i] = c;
        }
        for (int s = 1; s < 8; s++)
            for (int i = 0; i < 256; i++) slice[s][i] = (slice[s - 1][i] >> 8) ^ slice[0][slice[s - 1][i] & 0xFF];
        for (int k = 0; k < 3; k++) zero_shift_table(slice[0], 128 * (3 - k), shift[k]);
        for (int i = 0; i < 7; i++) zero_shift_table(slice[0], 16 * (7 - i), seg[i]);
        final512 = zero_bytes(slice[0], 0xFFFFFFFFu, 512) ^ 0xFFFFFFFFu;
    }
};

}  // namespace crc
}  // namespace hec
