// host_gf.hpp -- the engine's host-side GF(2^8) stripe multiply, for rows
// too small to pay a PCIe round trip (the per-call drop-in's small-row path,
// hec_encode / hec_decode below the coder's host limit; hec_gf_matmul_host).
//
//   out[j][b] = XOR_i M[j][i] * in[i][b]    (GF(2^8), modulus 0x11D)
//
// Same map as the device kernels and the reference's hot loop
// (rust/src/ec/matrix.rs:204-231), restated for the CPU's byte-vector units:
//   * AVX-512BW + GFNI: multiplication by a constant c is GF(2)-linear on a
//     byte, so one vgf2p8affineqb applies c's 8x8 bit matrix to 64 bytes
//     (the instruction's own field is irrelevant: the matrix encodes 0x11D);
//     3-input XORs (vpternlogq) accumulate; masked loads/stores take any
//     length and alignment.
//   * AVX2: split-nibble product tables, two vpshufb per 32 bytes.
//   * scalar: log/antilog tables.
// The ISA is picked once at run time (CPUID).  No device, no allocation, no
// lock: thread-safe.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace hec {
namespace host {

enum Isa { kScalar = 0, kAvx2 = 1, kAvx512Gfni = 2 };

// The best ISA this CPU supports.
Isa best_isa();
const char* isa_name(Isa isa);

// The 8x8 GF(2) matrix of y = c * x as a vgf2p8affineqb qword (byte 7 - i =
// the input-bit mask of output bit i).
uint64_t affine_matrix(uint8_t c);

// affine_matrix of every entry of a rows x cols matrix (row-major), so that
// hot callers (a coder's encode matrix, a cached decode plan) build it once.
std::vector<uint64_t> affine_matrices(const uint8_t* mat, size_t n_entries);

// out[j] = sum_i mat[j*cols + i] * in[i] (n bytes each) with the given ISA
// (kAvx512Gfni / kAvx2 fall back to what the CPU supports).  rows, cols >= 1;
// aff = affine_matrices(mat) or null (then built per call).
void gf_matmul(Isa isa, const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols, const uint8_t* const* in,
               uint8_t* const* out, size_t n);

inline void gf_matmul(const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols, const uint8_t* const* in,
                      uint8_t* const* out, size_t n) {
    gf_matmul(best_isa(), mat, aff, rows, cols, in, out, n);
}

// The same with rows of at least split_min_bytes() (256 KiB) per shard cut
// into column ranges coded by a small process-wide worker pool plus the
// calling thread ($HEC_HOST_THREADS threads in all, default 4; 1 = never
// split).  A row that long is bound by one core's memory bandwidth, not its
// GFNI units; the pieces are 4 KiB aligned.  If another call holds the pool,
// the row is coded on the calling thread.  cols <= 64.
void gf_matmul_split(Isa isa, const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols,
                     const uint8_t* const* in, uint8_t* const* out, size_t n);
size_t split_min_bytes();

inline void gf_matmul_split(const uint8_t* mat, const uint64_t* aff, size_t rows, size_t cols,
                            const uint8_t* const* in, uint8_t* const* out, size_t n) {
    gf_matmul_split(best_isa(), mat, aff, rows, cols, in, out, n);
}

}  // namespace host
}  // namespace hec
