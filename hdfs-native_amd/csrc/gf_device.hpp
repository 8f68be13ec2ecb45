// gf_device.hpp -- device building blocks shared by the GF(2^8) coding
// kernels (ec_kernels.hip) and the fused coding + checksum kernels
// (ec_fused.hip): the LDS log/antilog prologue, the v_perm_b32 product
// tables (c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6]), the tile order and the
// 16-B non-temporal accesses.  See ec_kernels.hip for the design.
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (jit.cpp) provides the HIP runtime itself
#include <hip/hip_runtime.h>
#endif

#include <cstdint>

#include "ec_kernels.hpp"
#include "gf256.hpp"
#include "work_queue.hpp"

namespace hec {
namespace {  // per translation unit: each .hip file is its own code object

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__constant__ GfTables kDevGf = GfTables();

// PermTable (ec_kernels.hpp): 8 dwords (32 B) per coefficient so that a
// ds_read_b128 + ds_read_b32 pair fetches it (broadcast: all lanes read the
// same address, so no bank conflicts).

__device__ __forceinline__ uint8_t lds_gf_mul(const uint8_t* s_exp, const uint8_t* s_log, uint8_t a,
                                              uint8_t b) {
    return (a == 0 || b == 0) ? 0 : s_exp[s_log[a] + s_log[b]];
}

__device__ __forceinline__ uint32_t pack4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
    return uint32_t(a) | (uint32_t(b) << 8) | (uint32_t(c) << 16) | (uint32_t(d) << 24);
}

// Builds the v_perm_b32 product tables for coefficient c using the LDS
// log/antilog tables.
__device__ void build_perm_table(PermTable* t, uint8_t c, const uint8_t* s_exp, const uint8_t* s_log) {
    uint8_t p0[8], p1[8], p2[4];
#pragma unroll
    for (int e = 0; e < 8; e++) {
        p0[e] = lds_gf_mul(s_exp, s_log, c, uint8_t(e));
        p1[e] = lds_gf_mul(s_exp, s_log, c, uint8_t(e << 3));
    }
#pragma unroll
    for (int e = 0; e < 4; e++) p2[e] = lds_gf_mul(s_exp, s_log, c, uint8_t(e << 6));
    t->t0lo = pack4(p0[0], p0[1], p0[2], p0[3]);
    t->t0hi = pack4(p0[4], p0[5], p0[6], p0[7]);
    t->t1lo = pack4(p1[0], p1[1], p1[2], p1[3]);
    t->t1hi = pack4(p1[4], p1[5], p1[6], p1[7]);
    t->t2 = pack4(p2[0], p2[1], p2[2], p2[3]);
    t->pad0 = t->pad1 = t->pad2 = 0;
}

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96).  hipcc mostly
// emits two v_xor_b32 for it; spelled out, the GF math drops from 3 to 2
// XOR-type ops per (dword, coefficient).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// c * x for the four bytes of x.  v_perm_b32(S0=hi, S1=lo, sel): selector
// byte 0..3 picks a byte of lo, 4..7 a byte of hi.
__device__ __forceinline__ uint32_t gf_mul4(uint32_t t0lo, uint32_t t0hi, uint32_t t1lo, uint32_t t1hi,
                                            uint32_t t2, uint32_t s0, uint32_t s1, uint32_t s2) {
    uint32_t a = __builtin_amdgcn_perm(t0hi, t0lo, s0);
    uint32_t b = __builtin_amdgcn_perm(t1hi, t1lo, s1);
    uint32_t c = __builtin_amdgcn_perm(t2, t2, s2);
    return xor3(a, b, c);
}

struct Sel {
    uint32_t s0, s1, s2;
};

// Tile order: stripes are taken G at a time and, inside a group, tiles go
// column-major (tile-column c of all G stripes, then c+1), so the blocks in
// flight together touch G stripes x (grid/G) columns.  G = 1 is plain
// stripe-major order.  A stripe count that G does not divide leaves
// stripes % G remainder stripes after the last whole group
// (a.grouped_tiles = (stripes / G) * G * tiles_per_stripe); their tiles run
// stripe-major, so a prime batch keeps the grouped order for all but its last
// G - 1 stripes (it used to fall back to stripe-major throughout).
__device__ __forceinline__ void tile_coords(uint32_t tile, const MatmulArgs& a, uint32_t& stripe, uint32_t& tcol) {
    const uint32_t tps = a.tiles_per_stripe;
    const uint32_t G = a.group;
    if (G <= 1 || tile >= a.grouped_tiles) {
        // grouped_tiles is a whole number of stripes: tile / tps is the stripe
        stripe = tile / tps;
        tcol = tile - stripe * tps;
        return;
    }
    // G and tps are launch constants: their reciprocals are hoisted out of
    // the tile loop (a per-tile divisor made hipcc rebuild one with VALU
    // float ops in the loop, whose temporaries landed in in-flight store
    // registers and forced store drains)
    const uint32_t per_group = G * tps;
    const uint32_t g = tile / per_group;
    const uint32_t r = tile - g * per_group;
    tcol = r / G;
    stripe = g * G + (r - tcol * G);
}

// Tile-order group for a batch: `want` stripes per group (at most the
// stripe count), and the tiles those whole groups cover.
__host__ inline void tile_order(uint64_t stripes, uint32_t tiles_per_stripe, uint32_t want, uint32_t& group,
                                uint32_t& grouped_tiles) {
    group = uint32_t(want < 1 ? 1 : (stripes < want ? (stripes < 1 ? 1 : stripes) : want));
    grouped_tiles = uint32_t((stripes / group) * group * tiles_per_stripe);
}

__device__ __forceinline__ Sel make_sel(uint32_t x) {
    Sel s;
    s.s0 = x & 0x07070707u;
    s.s1 = (x >> 3) & 0x07070707u;
    s.s2 = (x >> 6) & 0x03030303u;
    return s;
}

template <bool NT>
__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
    if constexpr (NT)
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else
        return *reinterpret_cast<const u32x4*>(p);
}

template <bool NT>
__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else
        *reinterpret_cast<u32x4*>(p) = v;
}

// Stage log/antilog + coefficient rows in LDS, build the perm tables.
// KC = columns of the caller's s_tab (kMaxK, or K where LDS is tight).
template <int R, int BS, int KC = kMaxK>
__device__ __forceinline__ void prologue(const MatmulArgs& a, int k, PermTable (*s_tab)[KC], uint8_t* s_exp,
                                         uint8_t* s_log, uint8_t* s_coef) {
    static_assert(BS >= 256 && BS % 256 == 0, "prologue assumes >= 256 threads");
    const int tid = threadIdx.x;
    if (tid < 256) {
        s_exp[tid] = kDevGf.exp[tid];
        s_exp[tid + 256] = kDevGf.exp[tid + 256];
        s_log[tid] = kDevGf.log[tid];
    }
    if (tid < R * kMaxK) s_coef[tid] = a.coef[tid];
    __syncthreads();
    for (int t = tid; t < R * k; t += BS) {
        int j = t / k, i = t - j * k;
        build_perm_table(&s_tab[j][i], s_coef[j * kMaxK + i], s_exp, s_log);
    }
    __syncthreads();
}

}  // namespace
}  // namespace hec
