// gf256.hpp -- GF(2^8) arithmetic and RS coding-matrix construction for the
// host side of the MI355X EC engine (shared by the C ABI and the C++ mirror).
//
// Field: GF(2^8) modulo x^8+x^4+x^3+x^2+1 (0x11D), exactly the field declared
// by hdfs-native at rust/src/ec/gf256.rs:7 (g2p::g2p!(GF256, 8, modulus:
// 0b1_0001_1101)).  add = XOR, mul via exp/log over generator 2.
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (jit.cpp) compiles only the tables below
#include <array>
#include <cstddef>
#include <cstring>
#include <vector>
#endif
#include <cstdint>

namespace hec {

struct GfTables {
    uint8_t exp[512]{};
    uint8_t log[256]{};
    constexpr GfTables() {
        unsigned x = 1;
        for (int i = 0; i < 255; i++) {
            exp[i] = static_cast<uint8_t>(x);
            log[x] = static_cast<uint8_t>(i);
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; i++) exp[i] = exp[i - 255];
    }
};

inline constexpr GfTables kGf{};

constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : kGf.exp[kGf.log[a] + kGf.log[b]];
}
constexpr uint8_t gf_inv(uint8_t a) { return a == 0 ? 0 : kGf.exp[255 - kGf.log[a]]; }
constexpr uint8_t gf_div(uint8_t a, uint8_t b) { return gf_mul(a, gf_inv(b)); }

#ifndef __HIPCC_RTC__

// Coder::gen_rs_matrix (rust/src/ec/gf256.rs:40-57): (k+m) x k, row-major.
// Identity on top; parity row r, column c = 1 / (r XOR c) (Hadoop
// RSUtil.genCauchyMatrix).
inline std::vector<uint8_t> gen_rs_matrix(size_t k, size_t m) {
    std::vector<uint8_t> mat((k + m) * k, 0);
    for (size_t r = 0; r < k; r++) mat[r * k + r] = 1;
    for (size_t r = k; r < k + m; r++)
        for (size_t c = 0; c < k; c++) {
            uint8_t s = static_cast<uint8_t>(r) ^ static_cast<uint8_t>(c);
            mat[r * k + c] = s == 0 ? 0 : gf_div(1, s);
        }
    return mat;
}

// Hadoop's XOR-k-1 codec (XORRawEncoder): identity on top, one all-ones
// parity row (parity = XOR of the data units).  The reference names the
// codec (ec/mod.rs:9-11, policy 4 = XOR-2-1) but rejects it on read.
inline std::vector<uint8_t> gen_xor_matrix(size_t k) {
    std::vector<uint8_t> mat((k + 1) * k, 0);
    for (size_t r = 0; r < k; r++) mat[r * k + r] = 1;
    for (size_t c = 0; c < k; c++) mat[k * k + c] = 1;
    return mat;
}

// Hadoop's rs-legacy codec (policy 3, RS-LEGACY-6-3-1024k; the reference
// resolves the schema at ec/mod.rs:118-124 but has no coder for it).  Hadoop
// 3.x RSRawEncoderLegacy is a systematic cyclic RS code: generator polynomial
// g(x) = prod_{i<m} (x + 2^i) over this same field (RSUtil.getPrimitivePower,
// GaloisField.multiply), codeword = data unit i at degree m+i, parity unit j
// = coefficient j of (sum_i d_i x^(m+i)) mod g(x) (GaloisField.remainder).
// That is linear in the data, so it is a (k+m) x k matrix like the others:
// parity row k+j, column i = coefficient j of x^(m+i) mod g(x).  The code is
// MDS (m consecutive roots, k+m <= 255), so every k rows are invertible and
// the generic decode gives the unique codeword the legacy decoder finds.
inline std::vector<uint8_t> gen_rs_legacy_matrix(size_t k, size_t m) {
    std::vector<uint8_t> g(m + 1, 0);  // g[d] = coefficient of x^d, monic
    g[0] = 1;
    for (size_t i = 0; i < m; i++) {   // g *= (x + 2^i)
        const uint8_t root = kGf.exp[i % 255];
        for (size_t d = i + 1; d > 0; d--) g[d] = static_cast<uint8_t>(g[d - 1] ^ gf_mul(g[d], root));
        g[0] = gf_mul(g[0], root);
    }
    std::vector<uint8_t> mat((k + m) * k, 0);
    for (size_t r = 0; r < k; r++) mat[r * k + r] = 1;
    std::vector<uint8_t> rem(m, 0);  // x^m mod g, then x^(m+i) mod g by shifting
    for (size_t j = 0; j < m; j++) rem[j] = g[j];  // x^m = sum_{j<m} g_j x^j (char 2)
    for (size_t c = 0; c < k; c++) {
        for (size_t j = 0; j < m; j++) mat[(k + j) * k + c] = rem[j];
        const uint8_t top = rem[m - 1];  // rem * x mod g
        for (size_t j = m - 1; j > 0; j--) rem[j] = static_cast<uint8_t>(rem[j - 1] ^ gf_mul(top, g[j]));
        rem[0] = gf_mul(top, g[0]);
    }
    return mat;
}

// Matrix::invert (rust/src/ec/matrix.rs:101-162): Gauss-Jordan over GF(2^8)
// on [M | I].  The inverse is unique, so any pivoting gives the reference's
// result; we pick the first non-zero pivot below.  Returns false where the
// reference panics with "Matrix is singular" (matrix.rs:121-123).
inline bool invert(uint8_t* mat, size_t n) {
    const size_t w = 2 * n;
    std::vector<uint8_t> a(n * w, 0);
    for (size_t r = 0; r < n; r++) {
        std::memcpy(&a[r * w], mat + r * n, n);
        a[r * w + n + r] = 1;
    }
    for (size_t col = 0; col < n; col++) {
        size_t piv = col;
        while (piv < n && a[piv * w + col] == 0) piv++;
        if (piv == n) return false;
        if (piv != col)
            for (size_t c = 0; c < w; c++) std::swap(a[piv * w + c], a[col * w + c]);
        uint8_t s = gf_inv(a[col * w + col]);
        for (size_t c = 0; c < w; c++) a[col * w + c] = gf_mul(a[col * w + c], s);
        for (size_t r = 0; r < n; r++) {
            if (r == col) continue;
            uint8_t f = a[r * w + col];
            if (!f) continue;
            for (size_t c = 0; c < w; c++) a[r * w + c] ^= gf_mul(f, a[col * w + c]);
        }
    }
    for (size_t r = 0; r < n; r++) std::memcpy(mat + r * n, &a[r * w + n], n);
    return true;
}

// The 3-3-2 v_perm_b32 product tables for coefficient c (layout of
// hec::PermTable): words {t0lo, t0hi, t1lo, t1hi, t2, 0, 0, 0}.
inline std::array<uint32_t, 8> perm_table_words(uint8_t c) {
    auto pack = [](uint8_t a, uint8_t b, uint8_t d, uint8_t e) {
        return uint32_t(a) | (uint32_t(b) << 8) | (uint32_t(d) << 16) | (uint32_t(e) << 24);
    };
    uint8_t p0[8], p1[8], p2[4];
    for (int e = 0; e < 8; e++) {
        p0[e] = gf_mul(c, uint8_t(e));
        p1[e] = gf_mul(c, uint8_t(e << 3));
    }
    for (int e = 0; e < 4; e++) p2[e] = gf_mul(c, uint8_t(e << 6));
    return {pack(p0[0], p0[1], p0[2], p0[3]), pack(p0[4], p0[5], p0[6], p0[7]),
            pack(p1[0], p1[1], p1[2], p1[3]), pack(p1[4], p1[5], p1[6], p1[7]),
            pack(p2[0], p2[1], p2[2], p2[3]), 0u, 0u, 0u};
}

#endif  // __HIPCC_RTC__

}  // namespace hec
