// gf256.hpp -- GF(2^8) arithmetic and RS coding-matrix construction for the
// host side of the MI355X EC engine (shared by the C ABI and the C++ mirror).
//
// Field: GF(2^8) modulo x^8+x^4+x^3+x^2+1 (0x11D), exactly the field declared
// by hdfs-native at rust/src/ec/gf256.rs:7 (g2p::g2p!(GF256, 8, modulus:
// 0b1_0001_1101)).  add = XOR, mul via exp/log over generator 2.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

namespace hec {

struct GfTables {
    std::array<uint8_t, 512> exp{};
    std::array<uint8_t, 256> log{};
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

}  // namespace hec
