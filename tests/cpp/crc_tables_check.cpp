// crc_tables_check.cpp -- host-side check of the compile-time CRC tables the
// GPU kernels use (hdfs-native_amd/csrc/checksum_tables.hpp): for CRC32C and
// CRC32 (CRC_32_CKSUM), the per-512-B-chunk checksum is recomputed on the CPU
// three ways with the kernels' own algebra --
//   s8  : 4 quarters by slicing-by-8 from state 0, placed with the
//         "append 384/256/128 zero bytes" byte tables, + final512;
//   w11 : the same quarters by 11-bit slicing, placed with the nibble tables;
//   fold: (CRC32C) each quarter's dwords 0..23 folded forward by the sparse
//         multiple x^209+x^144+x^54+x^39+x^14+1 of the polynomial, then
//         11-bit slicing over its last 32 B (checksum_device.hpp Fold);
//   byte: the classic byte-serial loop, from the table slot the 11-bit
//         scheme's tail reads (w11[5][x]);
//   fold32: (CRC32C) the same fold, then the last 32 B through the
//         slicing-by-32 tables (Slice32, measurement scheme 15);
// and printed as hex, one line per chunk, for tests/test_oracle.py to compare
// with the oracle.  Input: splitmix64 bytes (seed argv[1], chunks argv[2]).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../hdfs-native_amd/csrc/checksum_tables.hpp"

using namespace hec::crc;

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | (uint32_t(p[3]) << 24); }

template <int KIND>
struct Check {
    static constexpr bool REFL = Spec<KIND>::kReflected;
    const Tables<KIND>& t;
    explicit Check(const Tables<KIND>& tt) : t(tt) {}

    uint32_t pre(uint32_t crc) const { return REFL ? crc : __builtin_bswap32(crc); }
    uint32_t q_s8(const uint8_t* q) const {
        uint32_t r = 0;
        for (int i = 0; i < 128; i += 8) {
            const uint32_t lo = le32(q + i) ^ pre(r), hi = le32(q + i + 4);
            r = t.slice[7][lo & 0xFF] ^ t.slice[6][(lo >> 8) & 0xFF] ^ t.slice[5][(lo >> 16) & 0xFF] ^
                t.slice[4][lo >> 24] ^ t.slice[3][hi & 0xFF] ^ t.slice[2][(hi >> 8) & 0xFF] ^
                t.slice[1][(hi >> 16) & 0xFF] ^ t.slice[0][hi >> 24];
        }
        return r;
    }
    // the 11-bit fields of a word: w[2:13], w[13:24], w[24:32] + w[0:2]
    static uint32_t f0(uint32_t w) { return (w >> 2) & 0x7FF; }
    static uint32_t f1(uint32_t w) { return (w >> 13) & 0x7FF; }
    static uint32_t f2(uint32_t w) { return (w >> 24) | ((w & 3u) << 8); }
    uint32_t q_w11(const uint8_t* q) const {
        uint32_t r = 0;
        for (int i = 0; i < 128; i += 8) {
            const uint32_t lo = le32(q + i) ^ pre(r), hi = le32(q + i + 4);
            r = t.w11[0][f0(lo)] ^ t.w11[1][f1(lo)] ^ t.w11[2][f2(lo)] ^ t.w11[3][f0(hi)] ^ t.w11[4][f1(hi)] ^
                t.w11[5][f2(hi)];
        }
        return r;
    }
    uint32_t shift_byte(int k, uint32_t r) const {
        return t.shift[k][0][r & 0xFF] ^ t.shift[k][1][(r >> 8) & 0xFF] ^ t.shift[k][2][(r >> 16) & 0xFF] ^
               t.shift[k][3][r >> 24];
    }
    uint32_t shift_nib(int k, uint32_t r) const {
        uint32_t v = 0;
        for (int q = 0; q < 8; q++) v ^= t.shift_nib[k][q][(r >> (4 * q)) & 15];
        return v;
    }
    // scheme 12: the kernel's fold, the same offsets (32q + s) and order
    // (fd = folded dwords: 24 for scheme 12, 16 / 20 for the measurement schemes 13 / 14)
    // s32 = Slice32 tables: the tail's 32 bytes as independent lookups (scheme 15)
    uint32_t q_fold(const uint8_t* q, int fd = 24, const Slice32<KIND>* s32 = nullptr) const {
        static const int kq[5] = {6, 6, 5, 4, 2}, ks[5] = {17, 3, 10, 27, 1};
        uint32_t w[32];
        for (int i = 0; i < 32; i++) w[i] = le32(q + 4 * i);
        for (int i = 2; i < 32; i++)
            for (int o = 0; o < 5; o++) {
                const int hi = i - kq[o], lo = hi - 1;
                const uint32_t h = hi >= 0 && hi < fd ? w[hi] : 0, l = lo >= 0 && lo < fd ? w[lo] : 0;
                w[i] ^= (h << ks[o]) | (l >> (32 - ks[o]));
            }
        uint32_t r = 0;
        if (s32) {
            for (int i = 0; i < 32; i++) r ^= s32->t[31 - i][(w[24 + i / 4] >> (8 * (i % 4))) & 0xFF];
            return r;
        }
        for (int i = fd; i < 32; i += 2) {
            const uint32_t lo = w[i] ^ pre(r), hi = w[i + 1];
            r = t.w11[0][f0(lo)] ^ t.w11[1][f1(lo)] ^ t.w11[2][f2(lo)] ^ t.w11[3][f0(hi)] ^ t.w11[4][f1(hi)] ^
                t.w11[5][f2(hi)];
        }
        return r;
    }
    uint32_t chunk(const uint8_t* c, bool w11, bool fold = false, int fd = 24,
                   const Slice32<KIND>* s32 = nullptr) const {
        uint32_t v = 0;
        for (int qi = 0; qi < 4; qi++) {
            const uint32_t r = fold ? q_fold(c + 128 * qi, fd, s32) : w11 ? q_w11(c + 128 * qi) : q_s8(c + 128 * qi);
            v ^= qi < 3 ? (w11 ? shift_nib(qi, r) : shift_byte(qi, r)) : r;
        }
        return v ^ t.final512;
    }
    uint32_t chunk_bytes(const uint8_t* c) const {  // tail loop, 11-bit scheme's table slot
        uint32_t r = Spec<KIND>::kInit;
        for (int i = 0; i < 512; i++) {
            const uint32_t idx = REFL ? ((r ^ c[i]) & 0xFF) : (((r >> 24) ^ c[i]) & 0xFF);
            r = REFL ? (t.w11[5][idx] ^ (r >> 8)) : (t.w11[5][idx] ^ (r << 8));
        }
        return r ^ Spec<KIND>::kXorout;
    }
};

static const Tables<kCrc32c> kT32c;
static const Tables<kCksum> kTck;
static const Slice32<kCrc32c> kS32c;

int main(int argc, char** argv) {
    uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 1;
    const int chunks = argc > 2 ? std::atoi(argv[2]) : 8;
    std::vector<uint8_t> data(size_t(chunks) * 512);
    for (size_t i = 0; i < data.size(); i += 8) {
        const uint64_t v = splitmix(seed);
        for (int b = 0; b < 8; b++) data[i + b] = uint8_t(v >> (8 * b));
    }
    Check<kCrc32c> c32c(kT32c);
    Check<kCksum> cck(kTck);
    for (int k = 0; k < chunks; k++) {
        const uint8_t* c = data.data() + 512 * k;
        std::printf("%08x %08x %08x %08x %08x %08x %08x %08x %08x %08x\n", c32c.chunk(c, false), c32c.chunk(c, true),
                    c32c.chunk_bytes(c), cck.chunk(c, false), cck.chunk(c, true), cck.chunk_bytes(c),
                    c32c.chunk(c, true, true), c32c.chunk(c, true, true, 16), c32c.chunk(c, true, true, 20),
                    c32c.chunk(c, true, true, 24, &kS32c));
    }
    std::fflush(stdout);
    // the data itself, for the oracle side
    std::fwrite(data.data(), 1, data.size(), stderr);
    return 0;
}
