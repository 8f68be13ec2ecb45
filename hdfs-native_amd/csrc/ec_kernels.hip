// ec_kernels.hip -- hand-written gfx950 kernels for the GF(2^8) coding-matrix
// multiply over stripe cells: the MI355X replacement for the reference's hot
// loop, Mul<&[&[u8]]> for Matrix<GF256> (rust/src/ec/matrix.rs:204-231),
// driven by Coder::encode (gf256.rs:61-80) and Coder::decode (gf256.rs:84-137).
//
//   out[j][b] = XOR_i  M[j][i] * in[i][b]       (GF(2^8), modulus 0x11D)
//
// Design (see DESIGN.md "Kernels"):
//  * HBM-bound byte work, no MFMA.  Each lane owns one 16-byte column chunk
//    of every shard of a stripe (global_load_dwordx4 / 1 KiB per wave per
//    shard, fully coalesced), computes all R outputs from registers, writes
//    R x 16 B with dwordx4 stores.  Every input byte is read from HBM once
//    and every output byte written once: the algorithmic minimum (k+r)*cell.
//  * Per block, the coding-matrix rows and the log/antilog tables are staged
//    in LDS; from them the block builds, per coefficient c, three v_perm_b32
//    product tables: c*x = T0[x&7] ^ T1[(x>>3)&7] ^ T2[x>>6] (the 3-3-2 split
//    of the byte lets a 2-dword, 8-entry byte pool answer each lookup with
//    one v_perm_b32 on four bytes at once).  Per input dword: 5 selector ops;
//    per (input dword, coefficient): 3 v_perm_b32 + 2 XOR (v_bitop3).
//  * Grid-stride over (stripe, column-tile) tiles so the table prologue is
//    paid once per block.
//  * Layouts off the 16-B grid take a dword-realigning kernel (8 B per lane,
//    aligned dword loads + v_alignbyte, 0.79-0.84 of the aligned rate);
//    tails (cell_len % 16, or % 8 there) a byte-granular kernel with LDS
//    log/antilog lookups -- same results everywhere.
// Variants measured and rejected by more than 3 % (register double
// buffering, output bursts, store cache policies) were removed in round 6
// (git history: csrc/ec_experimental.hip); the HEC_EXPERIMENTAL library keeps
// the knob-selected shapes.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "bitslice.hpp"
#include "ec_kernels.hpp"
#include "gf_device.hpp"
#include "work_queue.hpp"
#include "xor_networks.hpp"

namespace hec {

namespace {
// A wave-uniform 64-bit value held in a VGPR (e.g. from a broadcast LDS
// read) moved into an SGPR pair (readfirstlane is int -> int: both halves
// go through uint32_t, no sign extension).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v))));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(v >> 32))));
    return uint64_t(lo) | (uint64_t(hi) << 32);
}

// Global-address-space byte pointers for bases that arrive as integers
// (the mixed kernel's LDS shard table): a generic pointer made from an
// integer compiles to flat_load / flat_store, which count in lgkmcnt as well
// as vmcnt, so every LDS wait of the tile (plan, tables) also waited for the
// cells in flight.  Global pointers keep them global_load / global_store.
typedef __attribute__((address_space(1))) uint8_t gbyte;
typedef __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ const gbyte* gptr(uint64_t a) { return reinterpret_cast<const gbyte*>(a); }
__device__ __forceinline__ gbyte* gptr_w(uint64_t a) { return reinterpret_cast<gbyte*>(a); }

__device__ __forceinline__ u32x4 gload16(const gbyte* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const gu32x4*>(p));
}
__device__ __forceinline__ void gstore16(gbyte* p, u32x4 v) {
    __builtin_nontemporal_store(v, reinterpret_cast<gu32x4*>(p));
}
}  // namespace

// ---------------------------------------------------------------------------
// Vector kernel: 16 B per lane per shard, U column chunks per lane (chunk u
// of a tile is a contiguous BS-lane slab: a wave's U pieces are BS*16 B
// apart).  K = compile-time input count (0 = runtime a.k), R = outputs (1..4).
// ---------------------------------------------------------------------------
// WQ > 0 (compile-time K; the default since round 5): the
// tiles are wave-tiles (64 lanes x U chunks) dealt round-robin to
// kMixedQueues launch counters (a.queue; block b takes from counter b %
// kMixedQueues, i.e. one per XCD), WQ rounds per atomic, the next batch
// fetched while the current one is coded.  Fast CUs take more tiles than slow
// ones, and the waves still walk the tile order together.  The counters are
// zero when the launch starts: the stream's previous launch zeroed this set
// (a.queue) and this one zeroes the other (a.queue_zero) for the next launch
// (work_queue.hpp queue_zero_next, ec_kernels.hip queue_lease).
template <int K, int R, int U, bool NT, int BS, int WQ = 0>
__global__ __launch_bounds__(BS) void gf_matmul_v16(MatmulArgs a) {
    static_assert(WQ == 0 || K > 0, "the work queue needs compile-time k");
    __shared__ PermTable s_tab[R][kMaxK];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    const int k = K ? K : a.k;
    prologue<R, BS>(a, k, s_tab, s_exp, s_log, s_coef);

    const uint32_t chunks = a.chunks;  // 16-B chunks per cell
    const uint32_t total = a.total_tiles;
    constexpr uint32_t TILE = WQ ? 64 * U : BS * U;  // chunks per tile (WQ: a wave-tile)
    constexpr uint32_t USTEP = WQ ? 64 : BS;          // chunks between a lane's U runs
    const uint32_t lcol = WQ ? (threadIdx.x & 63u) : threadIdx.x;

    // Previous tile's store data (compile-time K).  Held live until the next
    // tile's loads are issued, and every accumulator is materialised before
    // the first store: the compiler then never overwrites a VGPR that an
    // in-flight store still reads, so its waitcnt pass has no reason to drain
    // the stores (s_waitcnt vmcnt(0)) before the next loads or between the
    // chunks' stores -- it used to do both, twice per tile (same-box A/B:
    // RS(3,2) +8 %, RS(6,3) +2 %, RS(10,4) +3 %; profiles/r02_ab_drain/).
    u32x4 acc[U][R];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
    // WQ: this wave's counter, its next batch (lane 0, in flight) and the
    // rounds left of the current one; tile = round * wq_n + counter
    // counters in use: one per block up to kMixedQueues (a grid smaller than
    // that, tune key 7, must still reach every tile).  The counters are zero
    // at the launch's start (queue_zero_next, work_queue.hpp): this launch
    // zeroes the set of the stream's next launch and never resets its own.
    const uint32_t wq_n = gridDim.x < kMixedQueues ? gridDim.x : kMixedQueues;
    const uint32_t wq_q = blockIdx.x % wq_n;
    uint32_t* const wq_ctr = WQ ? a.queue + wq_q * (kMixedQueueStride / 4) : nullptr;
    if constexpr (WQ > 0) queue_zero_next(a.queue_zero);
    uint32_t wq_next, wq_round = 0, wq_left = 0;
    // defined in every lane (only lane 0's is read): the atomic's result is
    // not merged with an undefined value (as gf_decode_mixed's v_next)
    asm volatile("" : "=v"(wq_next));
    auto next_tile = [&]() -> uint32_t {
        for (;;) {
            if (wq_left == 0) {
                const uint32_t v = uint32_t(__builtin_amdgcn_readfirstlane(int(wq_next)));
                wq_round = v * uint32_t(WQ);
                wq_left = WQ;
                if (uint64_t(wq_round) * wq_n + wq_q >= total) return total;  // the wave is done
                if ((threadIdx.x & 63u) == 0) wq_next = atomicAdd(wq_ctr, 1u);
            } else {
                wq_round++;
            }
            wq_left--;
            const uint64_t t = uint64_t(wq_round) * wq_n + wq_q;
            if (t < total) return uint32_t(t);
            wq_left = 0;  // past the end inside a batch: read the fetch behind it
        }
    };
    if constexpr (WQ > 0)
        if ((threadIdx.x & 63u) == 0) wq_next = atomicAdd(wq_ctr, 1u);
    for (uint32_t tile = WQ ? next_tile() : blockIdx.x; tile < total; tile = WQ ? next_tile() : tile + gridDim.x) {
        uint32_t stripe, tcol;
        tile_coords(tile, a, stripe, tcol);
        // Keep the per-coefficient table reads inside the loop (LDS broadcast
        // reads) instead of letting LICM pin R*K*5 VGPRs for the whole kernel.
        asm volatile("" ::: "memory");
        if constexpr (K > 0) {
            // Compile-time K: every shard's loads for all U chunks are issued
            // before any arithmetic (K*U x 1 KiB in flight per wave).
            // 32-bit lane offsets from wave-uniform stripe bases: the loads
            // and stores take the saddr form, with no per-access 64-bit VALU
            // address add (the launcher keeps cells below 4 GiB here)
            u32x4 x[U][K];
            bool live[U];
            uint32_t offs[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t col = tcol * TILE + u * USTEP + lcol;
                live[u] = col < chunks;
                offs[u] = (live[u] ? col : 0u) * 16u;
            }
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int i = 0; i < K; i++)
                    x[u][i] = load16<NT>((a.in[i] + uint64_t(stripe) * a.in_stride[i]) + offs[u]);
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < R; j++) asm volatile("" ::"v"(acc[u][j]));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < K; i++) {
                // Opaque per-input table offset: input i's coefficient-table
                // reads cannot be hoisted above this point (otherwise the
                // compiler front-loads all R*K tables = R*K*5 VGPRs).
                uint32_t toff = uint32_t(i) * uint32_t(sizeof(PermTable));
                asm volatile("" : "+v"(toff));
                if (i > 0) {
#pragma unroll
                    for (int u = 0; u < U; u++)
#pragma unroll
                        for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
                }
                Sel s[U][4];
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int d = 0; d < 4; d++) s[u][d] = make_sel(x[u][i][d]);
#pragma unroll
                for (int j = 0; j < R; j++) {
                    const PermTable& t =
                        *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
                    const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
                    for (int u = 0; u < U; u++)
#pragma unroll
                        for (int d = 0; d < 4; d++) {
                            const uint32_t p = gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, s[u][d].s0, s[u][d].s1, s[u][d].s2);
                            acc[u][j][d] = i == 0 ? p : (acc[u][j][d] ^ p);
                        }
                }
                // one input at a time: stops the scheduler from hoisting every
                // coefficient's table read (R*K*5 VGPRs) to the top
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]));
            if ((tcol + 1) * TILE <= chunks) {  // block-uniform: the whole tile lies inside the cell
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int j = 0; j < R; j++)
                        store16<NT>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
            } else {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (!live[u]) continue;
#pragma unroll
                    for (int j = 0; j < R; j++)
                        store16<NT>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
                }
            }
            // drain policy (tune key 6): the tile's stores complete before the
            // next tile's loads are issued -- writes and reads then reach DRAM
            // in per-wave bursts rather than interleaved
            if (a.drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            // Runtime K: one shard at a time, U chunks per lane.
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t col = tcol * TILE + u * BS + threadIdx.x;
                if (col >= chunks) continue;
                const uint64_t off = uint64_t(col) * 16u;
                u32x4 racc[R];
#pragma unroll
                for (int j = 0; j < R; j++) racc[j] = u32x4{0, 0, 0, 0};
                for (int i = 0; i < k; i++) {
                    u32x4 x = load16<NT>(a.in[i] + uint64_t(stripe) * a.in_stride[i] + off);
                    Sel s[4];
#pragma unroll
                    for (int d = 0; d < 4; d++) s[d] = make_sel(x[d]);
#pragma unroll
                    for (int j = 0; j < R; j++) {
                        const PermTable& t = s_tab[j][i];
                        const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
                        for (int d = 0; d < 4; d++)
                            racc[j][d] ^= gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, s[d].s0, s[d].s1, s[d].s2);
                    }
                }
#pragma unroll
                for (int j = 0; j < R; j++) store16<NT>(a.out[j] + uint64_t(stripe) * a.out_stride[j] + off, racc[j]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Bit-sliced encode: gf_matmul_v16's skeleton (all K x U loads issued first,
// the previous tile's store data held live across them, store drain per
// tile) with the RS parity rows applied as generated XOR networks
// (xor_networks.hpp) instead of the v_perm product tables.  Each lane's U
// chunks of an input pair up into U/2 groups of 8 dwords; a group is
// transposed into 8 bit planes (bitslice.hpp) and folded into its R x 8
// accumulator planes by input i's network; at the end every parity row's
// planes are transposed back into bytes.  RS(6,3): 650 VALU per 8 dwords of
// every input instead of 960 (no selector ops, no table reads, no LDS
// prologue).  Only for the RS coding matrix of (K, R) (gen_rs_matrix,
// gf256.rs:40-57): the networks are that matrix's.
// ---------------------------------------------------------------------------
template <int K, int R, int U, int BS>
__global__ __launch_bounds__(BS) void gf_encode_bsl(MatmulArgs a) {
    static_assert(bitslice::rs_net_available<K, R>() && U % 2 == 0, "bit-sliced RS encode");
    constexpr int G = U / 2;
    const uint32_t chunks = a.chunks;
    const uint32_t total = a.total_tiles;
    constexpr uint32_t TILE = BS * U;
    u32x4 acc[U][R];  // previous tile's store data (see gf_matmul_v16)
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        uint32_t stripe, tcol;
        tile_coords(tile, a, stripe, tcol);
        u32x4 x[U][K];
        bool live[U];
        uint32_t offs[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t col = tcol * TILE + u * BS + threadIdx.x;
            live[u] = col < chunks;
            offs[u] = (live[u] ? col : 0u) * 16u;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int i = 0; i < K; i++) x[u][i] = load16<true>((a.in[i] + uint64_t(stripe) * a.in_stride[i]) + offs[u]);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" ::"v"(acc[u][j]));
        __builtin_amdgcn_sched_barrier(0);
        uint32_t accp[G][R * 8];
#pragma unroll
        for (int i = 0; i < K; i++) {
#pragma unroll
            for (int g = 0; g < G; g++) {
                uint32_t pl[8] = {x[2 * g][i][0],     x[2 * g][i][1],     x[2 * g][i][2],     x[2 * g][i][3],
                                  x[2 * g + 1][i][0], x[2 * g + 1][i][1], x[2 * g + 1][i][2], x[2 * g + 1][i][3]};
                if (i > 0) {
                    // opaque per input: the accumulators' XOR chains are not
                    // reassociated across inputs (that spills)
#pragma unroll
                    for (int t = 0; t < R * 8; t++) asm volatile("" : "+v"(accp[g][t]));
                }
                bitslice::transpose8(pl);
                bitslice::rs_absorb_at<K, R>(i, pl, accp[g]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < R; j++) {
                uint32_t q[8];
#pragma unroll
                for (int t = 0; t < 8; t++) q[t] = accp[g][8 * j + t];
                bitslice::transpose8(q);
                acc[2 * g][j] = u32x4{q[0], q[1], q[2], q[3]};
                acc[2 * g + 1][j] = u32x4{q[4], q[5], q[6], q[7]};
            }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]));
        if ((tcol + 1) * TILE <= chunks) {  // block-uniform
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < R; j++)
                    store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (!live[u]) continue;
#pragma unroll
                for (int j = 0; j < R; j++)
                    store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
            }
        }
        if (a.drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// ---------------------------------------------------------------------------
// LDS-DMA pipelined vector kernel (compile-time K only).  Each wave streams
// its part of tile t+1 straight into LDS with global_load_lds_dwordx4 while
// it computes tile t from registers, so at one wave per SIMD the HBM queue
// never drains during the GF math.  LDS image per wave: [K][U] pieces of
// 1 KiB (one wave-instruction each, lane-linear), read back by the SAME wave
// (ds_read_b128 at lane*16) -- no cross-wave hand-off, no barrier.
// ---------------------------------------------------------------------------
// BSL: the RS parity rows as bit-sliced XOR networks (see gf_encode_bsl).
template <int K, int R, int U, int BS, bool BSL = false>
__global__ __launch_bounds__(BS) void gf_matmul_dma(MatmulArgs a) {
    static_assert(K > 0, "DMA kernel needs a compile-time input count");
    static_assert(!BSL || (bitslice::rs_net_available<K, R>() && U % 2 == 0), "bit-sliced RS encode");
    constexpr int WAVES = BS / 64;
    constexpr int PIECE = 1024;  // one wave-instruction: 64 lanes x 16 B
    // One LDS array for everything (a second __shared__ object next to the
    // DMA image can make hipcc add vmcnt(0) waits; cdna guide §5 item 4a).
    constexpr int STAGE = WAVES * K * U * PIECE;
    constexpr int TAB = R * kMaxK * int(sizeof(PermTable));
    __shared__ __attribute__((aligned(16))) uint8_t s_mem[STAGE + TAB + 512 + 256 + R * kMaxK];
    PermTable(*s_tab)[kMaxK] = reinterpret_cast<PermTable(*)[kMaxK]>(s_mem + STAGE);
    uint8_t* s_exp = s_mem + STAGE + TAB;
    uint8_t* s_log = s_exp + 512;
    uint8_t* s_coef = s_log + 256;
    prologue<R, BS>(a, K, s_tab, s_exp, s_log, s_coef);

    const uint32_t chunks = a.chunks;
    const uint32_t total = a.total_tiles;
    constexpr uint32_t TILE = BS * U;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    const int lane = threadIdx.x & 63;
    uint8_t* stage = s_mem + wave * (K * U * PIECE);

    auto issue = [&](uint32_t tile) {
        uint32_t stripe, tcol;
        tile_coords(tile, a, stripe, tcol);
#pragma unroll
        for (int u = 0; u < U; u++) {
            uint32_t col = tcol * TILE + u * BS + wave * 64 + lane;
            col = col < chunks ? col : chunks - 1;  // dead lanes fetch a valid chunk, never stored
            const uint32_t off = col * 16u;           // cells < 4 GiB (launcher): saddr + 32-bit offset
#pragma unroll
            for (int i = 0; i < K; i++) {
                const uint8_t* src = (a.in[i] + uint64_t(stripe) * a.in_stride[i]) + off;
                __builtin_amdgcn_global_load_lds(
                    reinterpret_cast<const void*>(src),
                    (__attribute__((address_space(3))) void*)(stage + (i * U + u) * PIECE), 16, 0,
                    2 /* nt */);
            }
        }
    };

    uint32_t tile = blockIdx.x;
    if (tile < total) issue(tile);
    bool prev_full = false;  // previous iteration issued exactly R*U stores
    for (; tile < total; tile += gridDim.x) {
        // This tile's K*U pieces are the oldest vector-memory ops of the
        // wave.  After a full tile exactly R*U stores are younger and may
        // stay in flight; otherwise (first tile, or a partial tile whose
        // dead-lane stores were skipped) drain everything.
        if (prev_full)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * U) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 x[U][K];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int i = 0; i < K; i++)
                x[u][i] = *reinterpret_cast<const u32x4*>(stage + (i * U + u) * PIECE + lane * 16);
        // every read of the image has landed in VGPRs before it is refilled
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t next = tile + gridDim.x;
        if (next < total) issue(next);
        __builtin_amdgcn_sched_barrier(0);

        uint32_t stripe, tcol;
        tile_coords(tile, a, stripe, tcol);
        u32x4 acc[U][R];
        if constexpr (BSL) {
            constexpr int G = U / 2;
            uint32_t accp[G][R * 8];
#pragma unroll
            for (int i = 0; i < K; i++) {
#pragma unroll
                for (int g = 0; g < G; g++) {
                    uint32_t pl[8] = {x[2 * g][i][0],     x[2 * g][i][1],     x[2 * g][i][2],     x[2 * g][i][3],
                                      x[2 * g + 1][i][0], x[2 * g + 1][i][1], x[2 * g + 1][i][2], x[2 * g + 1][i][3]};
                    if (i > 0) {
#pragma unroll
                        for (int t = 0; t < R * 8; t++) asm volatile("" : "+v"(accp[g][t]));
                    }
                    bitslice::transpose8(pl);
                    bitslice::rs_absorb_at<K, R>(i, pl, accp[g]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int g = 0; g < G; g++)
#pragma unroll
                for (int j = 0; j < R; j++) {
                    uint32_t q[8];
#pragma unroll
                    for (int t = 0; t < 8; t++) q[t] = accp[g][8 * j + t];
                    bitslice::transpose8(q);
                    acc[2 * g][j] = u32x4{q[0], q[1], q[2], q[3]};
                    acc[2 * g + 1][j] = u32x4{q[4], q[5], q[6], q[7]};
                }
        } else {
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < K; i++) {
            uint32_t toff = uint32_t(i) * uint32_t(sizeof(PermTable));
            asm volatile("" : "+v"(toff));
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
            Sel sl[U][4];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int d = 0; d < 4; d++) sl[u][d] = make_sel(x[u][i][d]);
#pragma unroll
            for (int j = 0; j < R; j++) {
                const PermTable& t =
                    *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
                const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int d = 0; d < 4; d++)
                        acc[u][j][d] ^= gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, sl[u][d].s0, sl[u][d].s1, sl[u][d].s2);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        }  // !BSL
        // wave-uniform: every lane of every chunk of this wave is live
        const bool full = __builtin_amdgcn_readfirstlane(
                              int(tcol * TILE + (U - 1) * BS + wave * 64 + 63 < chunks)) != 0;
        if (full) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t off = (tcol * TILE + u * BS + threadIdx.x) * 16u;
#pragma unroll
                for (int j = 0; j < R; j++)
                    store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + off, acc[u][j]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t col = tcol * TILE + u * BS + threadIdx.x;
                if (col >= chunks) continue;
                const uint32_t off = col * 16u;
#pragma unroll
                for (int j = 0; j < R; j++)
                    store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + off, acc[u][j]);
            }
        }
        prev_full = full;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// Mixed-pattern decode: every stripe carries its own erasure pattern, as a
// striped read over many block groups does (ec/mod.rs:71 decodes row by
// row).  Same register math as gf_matmul_v16; per tile the block finds the
// stripe's plan (header: survivor and missing shard indices; e x K
// coefficient tables) and gathers the survivors by shard index through the
// block's LDS copy of the shard base / stride table.
//  RESIDENT: the per-stripe plan offsets and every plan sit in LDS for the
//    whole launch, so a tile's metadata costs a few broadcast LDS reads and
//    no memory round trip (a per-tile global read of the plan index used to
//    wait behind the previous tile's stores: vmcnt is in order).
//  otherwise: blocks walk contiguous runs of whole stripes and restage the
//    plan into LDS once per stripe.
// ---------------------------------------------------------------------------
//  WQ > 0 (measurement build, tune key 26; RESIDENT only): a work queue of
//    wave-tiles (64 lanes x U chunks of one stripe) instead of block tiles in
//    a fixed order.  The tile order is dealt round-robin to kMixedQueues
//    launch counters (a.queue, zeroed by the workspace upload; block b takes
//    from counter b % kMixedQueues, i.e. one per XCD), each atomic hands a
//    wave WQ rounds of its counter's tiles, and a wave fetches its next batch
//    while it codes the current one.  So the unequal stripes (k reads + e
//    writes each) even out at wave-tile grain, a grid of one block per CU
//    stages the plans once per CU, and the waves still walk the tile order
//    together (the DRAM window stays a few stripes wide).
// ---------------------------------------------------------------------------
template <int K, int R, int U, int BS, bool RESIDENT, bool MIXED_SKIP = true, int WQ = 0>
__global__ __launch_bounds__(BS) void gf_decode_mixed(MixedArgs a) {
    static_assert(WQ == 0 || RESIDENT, "the work queue needs resident plans");
    static_assert(K > 0, "compile-time k");
    __shared__ PermTable s_tab[RESIDENT ? 1 : R][K];  // non-resident: the current plan's rows
    __shared__ DevPlanHeader s_hdr;
    __shared__ uint64_t s_base[kMaxShards], s_stride[kMaxShards], s_obase[kMaxK], s_ostride[kMaxK];
    // RESIDENT: [stripe plan offsets: u32 x stripes, 16-B padded][plan blob]
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    const int tid = threadIdx.x;
    if (tid < kMaxShards) {
        s_base[tid] = reinterpret_cast<uint64_t>(a.base[tid]);
        s_stride[tid] = a.stride[tid];
    }
    if (tid < kMaxK) {
        s_obase[tid] = reinterpret_cast<uint64_t>(a.out[tid]);
        s_ostride[tid] = a.out_stride[tid];
    }
    const uint32_t off_bytes = (uint32_t(a.stripes) * 4u + 15u) & ~15u;
    if constexpr (RESIDENT) {
        const uint32_t off_words = uint32_t(a.stripes);
        for (uint32_t t = tid; t < off_words; t += BS) reinterpret_cast<uint32_t*>(s_dyn)[t] = a.stripe_off[t];
        const uint32_t words = a.blob_bytes / 4;
        for (uint32_t t = tid; t < words; t += BS)
            reinterpret_cast<uint32_t*>(s_dyn + off_bytes)[t] = reinterpret_cast<const uint32_t*>(a.plans)[t];
    }
    __syncthreads();
    const uint32_t chunks = a.chunks;
    const uint32_t total = a.total_tiles;
    constexpr uint32_t TILE = WQ ? 64 * U : BS * U;  // chunks per tile (WQ: a wave-tile)
    constexpr uint32_t USTEP = WQ ? 64 : BS;          // chunks between a lane's U runs
    const uint32_t lcol = WQ ? (threadIdx.x & 63u) : threadIdx.x;
    MatmulArgs order;  // tile_coords reads tiles_per_stripe / group only
    order.tiles_per_stripe = a.tiles_per_stripe;
    order.group = a.group;
    order.grouped_tiles = a.grouped_tiles;
    order.stripes = a.stripes;

    // RESIDENT: grouped interleaved order (best DRAM locality).  Otherwise
    // each block walks a contiguous range of whole stripes, so its plan
    // changes (and LDS restaging with two barriers) once per stripe.
    uint32_t t_begin = blockIdx.x, t_end = total, t_step = gridDim.x;
    if constexpr (!RESIDENT) {
        const uint32_t per = (total + gridDim.x - 1) / gridDim.x;
        t_begin = blockIdx.x * per;
        t_end = min(total, t_begin + per);
        t_step = 1;
        order.group = 1;
    }
    uint32_t cur_stripe = 0xFFFFFFFFu;
    bool cur_none = true;
    u32x4 acc[U][R];  // previous tile's store data, held through the next loads (see gf_matmul_v16)
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
    auto run_tile = [&](uint32_t tile) {
        uint32_t stripe, tcol;
        tile_coords(tile, order, stripe, tcol);
        const DevPlanHeader* hdr = &s_hdr;
        const PermTable* tabs = &s_tab[0][0];  // row r, input i at tabs[r * K + i]
        if constexpr (RESIDENT) {
            const uint32_t off = __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t*>(s_dyn)[stripe]);
            if (off == kNoPlan) return;
            hdr = reinterpret_cast<const DevPlanHeader*>(s_dyn + off_bytes + off);
            tabs = reinterpret_cast<const PermTable*>(s_dyn + off_bytes + off + sizeof(DevPlanHeader)) + a.row0 * K;
        } else {
            if (stripe != cur_stripe) {  // block-uniform
                __syncthreads();         // every wave is done with the previous plan
                const uint32_t off = a.stripe_off[stripe];
                cur_none = off == kNoPlan;
                if (!cur_none) {
                    const uint8_t* blob = a.plans + off;
                    if (tid < 16) reinterpret_cast<uint32_t*>(&s_hdr)[tid] = reinterpret_cast<const uint32_t*>(blob)[tid];
                    const uint32_t e_all = reinterpret_cast<const DevPlanHeader*>(blob)->e;
                    const PermTable* src = reinterpret_cast<const PermTable*>(blob + sizeof(DevPlanHeader));
                    for (int t = tid; t < R * K * 8; t += BS) {
                        const int j = t / (K * 8), rem = t - j * (K * 8), i = rem / 8, w = rem - i * 8;
                        const int row = a.row0 + j;
                        reinterpret_cast<uint32_t*>(&s_tab[j][i])[w] =
                            row < int(e_all) ? reinterpret_cast<const uint32_t*>(&src[row * K + i])[w] : 0u;
                    }
                }
                __syncthreads();
                cur_stripe = stripe;
            }
            if (cur_none) return;
        }
        // The tile's metadata in three dependent LDS round trips, whatever K:
        // the header words (e, survivor and missing shard bytes), then every
        // survivor's and output's base / stride (VGPR-addressed broadcast
        // reads, all in flight at once), then one wait and the readfirstlanes.
        // Reading them survivor by survivor (LDS read, wait, readfirstlane,
        // next) cost K + R serial round trips before the tile's loads.
        const uint32_t* hw = reinterpret_cast<const uint32_t*>(hdr);
        constexpr int SW = (K + 3) / 4;  // words of survivor bytes (surv[] at byte 4)
        uint32_t w_surv[SW];
        const uint32_t w_e = hw[0];
        const uint32_t w_miss = hw[9 + a.row0 / 4];  // miss[] at byte 36; row0 is a multiple of kMaxR = 4
#pragma unroll
        for (int t = 0; t < SW; t++) w_surv[t] = hw[1 + t];
        uint64_t v_base[K], v_stride[K], v_obase[R], v_ostride[R];
#pragma unroll
        for (int i = 0; i < K; i++) {
            const uint32_t sh = (w_surv[i / 4] >> (8 * (i % 4))) & 0xFFu;
            v_base[i] = s_base[sh];
            v_stride[i] = s_stride[sh];
        }
#pragma unroll
        for (int j = 0; j < R; j++) {
            const uint32_t mi = (w_miss >> (8 * j)) & (kMaxK - 1);  // rows past e read a valid slot, never stored
            v_obase[j] = s_obase[mi];
            v_ostride[j] = s_ostride[mi];
        }
        // all of it read before the row-count branch below (otherwise hipcc
        // sinks the reads past it: one more round trip)
        uint32_t w_e2 = w_e;
#pragma unroll
        for (int i = 0; i < K; i++) asm volatile("" : "+v"(v_base[i]), "+v"(v_stride[i]), "+v"(w_e2));
        const int nrows = int(__builtin_amdgcn_readfirstlane(w_e2)) - a.row0;  // rows of this launch in the plan
        if (nrows <= 0) return;
        asm volatile("" ::: "memory");

        bool live[U];
        uint32_t offs[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t col = tcol * TILE + u * USTEP + lcol;
            live[u] = col < chunks;
            offs[u] = (live[u] ? col : 0u) * 16u;
        }
        u32x4 x[U][K];
#pragma unroll
        for (int i = 0; i < K; i++) {
            const gbyte* ib = gptr(uniform64(v_base[i]) + uint64_t(stripe) * uniform64(v_stride[i]));
#pragma unroll
            for (int u = 0; u < U; u++) x[u][i] = gload16(ib + offs[u]);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" ::"v"(acc[u][j]));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < K; i++) {
            uint32_t toff = uint32_t(i) * uint32_t(sizeof(PermTable));
            asm volatile("" : "+v"(toff));
            if (i > 0) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
            }
            Sel sl[U][4];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int d = 0; d < 4; d++) sl[u][d] = make_sel(x[u][i][d]);
#pragma unroll
            for (int j = 0; j < R; j++) {
                // rows past the plan's e are skipped (nrows is wave-uniform: a
                // scalar branch); their accumulators are never stored
                if (MIXED_SKIP && j > 0 && j >= nrows) break;
                const PermTable& t =
                    *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(tabs + j * K) + toff);
                const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int d = 0; d < 4; d++) {
                        const uint32_t p = gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, sl[u][d].s0, sl[u][d].s1, sl[u][d].s2);
                        acc[u][j][d] = i == 0 ? p : (acc[u][j][d] ^ p);
                    }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]));
        const bool full = (tcol + 1) * TILE <= chunks;  // block-uniform (WQ: wave-uniform)
#pragma unroll
        for (int j = 0; j < R; j++) {
            if (j >= nrows) break;  // block-uniform
            gbyte* ob = gptr_w(uniform64(v_obase[j]) + uint64_t(stripe) * uniform64(v_ostride[j]));
#pragma unroll
            for (int u = 0; u < U; u++)
                if (full || live[u]) gstore16(ob + offs[u], acc[u][j]);
        }
        if (a.drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // as gf_matmul_v16
    };
    if constexpr (WQ > 0) {
        // lane 0 holds the next batch index; the other lanes' copies are
        // never read (readfirstlane), so the atomic's result needs no merge
        // and is first waited for at the next batch, behind the tile drains
        const uint32_t nq = gridDim.x < kMixedQueues ? gridDim.x : kMixedQueues;  // every tile has a block
        const uint32_t q = blockIdx.x % nq;
        uint32_t* ctr = a.queue + q * (kMixedQueueStride / 4);
        uint32_t v_next;
        asm volatile("" : "=v"(v_next));  // defined, unread outside lane 0: no merge with the atomic's result
        if ((threadIdx.x & 63u) == 0) v_next = atomicAdd(ctr, 1u);
        for (;;) {
            const uint32_t r0 = uint32_t(__builtin_amdgcn_readfirstlane(int(v_next))) * uint32_t(WQ);
            if (uint64_t(r0) * nq + q >= total) break;  // 64-bit: no wrap past 2^32 tiles
            if ((threadIdx.x & 63u) == 0) v_next = atomicAdd(ctr, 1u);
            for (uint32_t r = r0; r < r0 + uint32_t(WQ); r++) {
                if (uint64_t(r) * nq + q >= total) break;
                run_tile(r * nq + q);
            }
        }
    } else {
        for (uint32_t tile = t_begin; tile < t_end; tile += t_step) run_tile(tile);
    }
}

// ---------------------------------------------------------------------------
// Wave-pair kernel for wide codes (round 6, RS(10,4)):
// the register kernel's memory schedule at RS(6,3) -- U = 4 chunks of 1 KiB
// per lane and input stream, one wave-tile per queue fetch -- for K = 10,
// whose K x U = 40 loads do not fit one wave beside its accumulators.  A
// 128-thread block is one wave PAIR working one wave-tile together: wave w
// loads and multiplies inputs [w K/2, (w+1) K/2) into partial sums of all R
// rows, hands the other wave the partials of ITS rows through LDS (double-
// buffered, one barrier per tile), XORs in the partials it receives and
// stores its own rows (wave 0 rows [0, R0), wave 1 [R0, R), R0 = ceil(R/2)).
// Each wave streams 5 inputs x 4 KiB (RS(6,3)'s wave streams 6), so the
// DRAM sees the same 4-KiB runs per stream, and the GF math per wave halves
// against one wave doing all 10 inputs.  The pair fetches its tiles from the
// work queue (wave 0, lane 0; the next tile travels through LDS with the
// partials), so its loop bound is block-uniform and both waves meet every
// barrier.
// ---------------------------------------------------------------------------
template <int K, int R, int U>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2, 2))) void gf_matmul_pair(MatmulArgs a) {
    static_assert(K % 2 == 0 && K <= 2 * 8, "the pair splits an even K");
    constexpr int KH = K / 2, R0 = (R + 1) / 2, R1 = R - R0, BS = 128;
    __shared__ PermTable s_tab[R][K];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    // partials for the other wave: [buffer][row slot][u][lane]; rows [0, R0)
    // are wave 0's (written by wave 1), rows [R0, R) wave 1's
    __shared__ u32x4 s_part[2][R][U][64];
    __shared__ uint32_t s_tile[2];
    const int tid = threadIdx.x;
    for (int t = tid; t < 256; t += BS) {
        s_exp[t] = kDevGf.exp[t];
        s_exp[t + 256] = kDevGf.exp[t + 256];
        s_log[t] = kDevGf.log[t];
    }
    for (int t = tid; t < R * kMaxK; t += BS) s_coef[t] = a.coef[t];
    queue_zero_next(a.queue_zero);
    const uint32_t n = gridDim.x < kMixedQueues ? gridDim.x : kMixedQueues;
    const uint32_t q = blockIdx.x % n;
    uint32_t* const ctr = a.queue + q * (kMixedQueueStride / 4);
    const uint32_t total = a.total_tiles;
    auto tile_of = [&](uint32_t v) -> uint32_t {
        const uint64_t t = uint64_t(v) * n + q;
        return t < total ? uint32_t(t) : total;
    };
    if (tid == 0) s_tile[0] = tile_of(atomicAdd(ctr, 1u));
    __syncthreads();
    for (int t = tid; t < R * K; t += BS) {
        const int j = t / K, i = t - j * K;
        build_perm_table(&s_tab[j][i], s_coef[j * kMaxK + i], s_exp, s_log);
    }
    __syncthreads();

    const int w = __builtin_amdgcn_readfirstlane(tid / 64);  // wave in the pair
    const uint32_t lane = tid & 63u;
    const uint32_t chunks = a.chunks;
    constexpr uint32_t TILE = 64 * U;
    uint32_t tile = uint32_t(__builtin_amdgcn_readfirstlane(int(s_tile[0])));
    for (int buf = 0; tile < total; buf ^= 1) {
        uint32_t stripe, tcol;
        tile_coords(tile, a, stripe, tcol);
        asm volatile("" ::: "memory");
        bool live[U];
        uint32_t offs[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t col = tcol * TILE + u * 64 + lane;
            live[u] = col < chunks;
            offs[u] = (live[u] ? col : 0u) * 16u;
        }
        u32x4 x[U][KH];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int i = 0; i < KH; i++) {
                const int ii = w * KH + i;
                x[u][i] = load16<true>((a.in[ii] + uint64_t(stripe) * a.in_stride[ii]) + offs[u]);
            }
        uint32_t fetch;
        asm volatile("" : "=v"(fetch));  // defined in every lane; lane 0's is the one used
        if (tid == 0) fetch = atomicAdd(ctr, 1u);  // the pair's next tile, in flight while this one is coded
        __builtin_amdgcn_sched_barrier(0);
        u32x4 acc[U][R];
#pragma unroll
        for (int i = 0; i < KH; i++) {
            uint32_t toff = uint32_t(w * KH + i) * uint32_t(sizeof(PermTable));
            asm volatile("" : "+v"(toff));
            if (i > 0) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
            }
            Sel sl[U][4];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int d = 0; d < 4; d++) sl[u][d] = make_sel(x[u][i][d]);
#pragma unroll
            for (int j = 0; j < R; j++) {
                const PermTable& t =
                    *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
                const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int d = 0; d < 4; d++) {
                        const uint32_t pr = gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, sl[u][d].s0, sl[u][d].s1, sl[u][d].s2);
                        acc[u][j][d] = i == 0 ? pr : (acc[u][j][d] ^ pr);
                    }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // hand over the other wave's rows, take the next tile, meet
#pragma unroll
        for (int j = 0; j < R; j++) {
            if ((j < R0) == (w == 0)) continue;  // my own row
#pragma unroll
            for (int u = 0; u < U; u++) s_part[buf][j][u][lane] = acc[u][j];
        }
        if (tid == 0) s_tile[buf ^ 1] = tile_of(fetch);
        __syncthreads();
        // every partial of my rows read before the first store (one wait)
#pragma unroll
        for (int j = 0; j < R; j++) {
            if ((j < R0) != (w == 0)) continue;  // the other wave's row
#pragma unroll
            for (int u = 0; u < U; u++) acc[u][j] ^= s_part[buf][j][u][lane];
        }
        if ((tcol + 1) * TILE <= chunks) {  // block-uniform: the whole tile lies inside the cell
#pragma unroll
            for (int j = 0; j < R; j++) {
                if ((j < R0) != (w == 0)) continue;
#pragma unroll
                for (int u = 0; u < U; u++)
                    store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < R; j++) {
                if ((j < R0) != (w == 0)) continue;
#pragma unroll
                for (int u = 0; u < U; u++)
                    if (live[u]) store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
            }
        }
        if (a.drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tile = uint32_t(__builtin_amdgcn_readfirstlane(int(s_tile[buf ^ 1])));
    }
    (void)R1;
}

// ---------------------------------------------------------------------------
// Unaligned layouts: 8 bytes per lane from naturally aligned dword loads.
// A batch whose base pointers or strides are off the 16-B grid cannot take
// the dwordx4 kernels.  Here lane g of stripe s owns bytes [8g, 8g+8) of the
// cell: per input it loads the 2 or 3 aligned dwords that cover them (every
// such dword holds at least one byte of the cell, so it never leaves the
// cell's pages) and shifts them into place with v_alignbyte; the GF math is
// the v_perm product tables of gf_matmul_v16; each output is stored as two
// dwords, four shorts or eight bytes by its own alignment.  Bytes
// [8 * (cell_len / 8), cell_len) are left to the byte kernel.
// ---------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(256) void gf_matmul_dw(MatmulArgs a) {
    __shared__ PermTable s_tab[R][kMaxK];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    const int k = a.k;
    prologue<R, 256>(a, k, s_tab, s_exp, s_log, s_coef);
    const uint64_t groups = a.cell_len / 8;
    const uint64_t total = groups * a.stripes;
    for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < total; t += uint64_t(gridDim.x) * 256) {
        const uint64_t stripe = t / groups;
        const uint64_t off = (t - stripe * groups) * 8;
        uint32_t acc[R][2];
#pragma unroll
        for (int j = 0; j < R; j++) acc[j][0] = acc[j][1] = 0;
        for (int i = 0; i < k; i++) {
            const uintptr_t p = reinterpret_cast<uintptr_t>(a.in[i] + stripe * a.in_stride[i] + off);
            // global pointer: an integer-made generic one compiles to flat loads (see gbyte)
            const __attribute__((address_space(1))) uint32_t* w =
                reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(p & ~uintptr_t(3));
            const uint32_t sh = uint32_t(p & 3);
            const uint32_t w0 = w[0], w1 = w[1];
            const uint32_t w2 = sh ? w[2] : 0u;  // holds bytes 8g+8-sh.. of this group only when sh != 0
            const uint32_t x[2] = {__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh)};
#pragma unroll
            for (int d = 0; d < 2; d++) {
                const Sel sl = make_sel(x[d]);
#pragma unroll
                for (int j = 0; j < R; j++) {
                    const PermTable& tb = s_tab[j][i];
                    acc[j][d] ^= gf_mul4(tb.t0lo, tb.t0hi, tb.t1lo, tb.t1hi, tb.t2, sl.s0, sl.s1, sl.s2);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < R; j++) {
            uint8_t* q = a.out[j] + stripe * a.out_stride[j] + off;
            const uintptr_t qa = reinterpret_cast<uintptr_t>(q);
            if ((qa & 3) == 0) {
                reinterpret_cast<uint32_t*>(q)[0] = acc[j][0];
                reinterpret_cast<uint32_t*>(q)[1] = acc[j][1];
            } else if ((qa & 1) == 0) {
                uint16_t* h = reinterpret_cast<uint16_t*>(q);
                h[0] = uint16_t(acc[j][0]);
                h[1] = uint16_t(acc[j][0] >> 16);
                h[2] = uint16_t(acc[j][1]);
                h[3] = uint16_t(acc[j][1] >> 16);
            } else {
#pragma unroll
                for (int b = 0; b < 8; b++) q[b] = uint8_t(acc[j][b / 4] >> (8 * (b % 4)));
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Byte kernel: tails (and, on tune key 18 = 1, whole unaligned batches).  One
// thread per (stripe, byte) in [a.byte_begin, a.cell_len); LDS log/antilog
// lookups.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void gf_matmul_bytes(MatmulArgs a) {
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_lc[kMaxR * kMaxK];  // log of each coefficient
    __shared__ uint8_t s_nz[kMaxR * kMaxK];
    const int tid = threadIdx.x;
    s_exp[tid] = kDevGf.exp[tid];
    s_exp[tid + 256] = kDevGf.exp[tid + 256];
    s_log[tid] = kDevGf.log[tid];
    if (tid < kMaxR * kMaxK) {
        const int t = tid;
        uint8_t c = a.coef[t];
        s_lc[t] = kDevGf.log[c];
        s_nz[t] = c != 0;
    }
    __syncthreads();
    const uint64_t width = a.cell_len - a.byte_begin;
    const uint64_t total = width * a.stripes;
    for (uint64_t g = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; g < total;
         g += uint64_t(gridDim.x) * blockDim.x) {
        const uint64_t stripe = g / width;
        const uint64_t b = a.byte_begin + (g - stripe * width);
        uint32_t acc[kMaxR] = {0, 0, 0, 0};
        for (int i = 0; i < a.k; i++) {
            const uint8_t x = a.in[i][stripe * a.in_stride[i] + b];
            if (!x) continue;
            const uint32_t lx = s_log[x];
            for (int j = 0; j < a.r; j++)
                if (s_nz[j * kMaxK + i]) acc[j] ^= s_exp[lx + s_lc[j * kMaxK + i]];
        }
        for (int j = 0; j < a.r; j++) a.out[j][stripe * a.out_stride[j] + b] = uint8_t(acc[j]);
    }
}

// ---------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------
namespace {

template <int K, int R, int U, bool NT, int BS>
const void* vec_fn() {
    return reinterpret_cast<const void*>(&gf_matmul_v16<K, R, U, NT, BS>);
}

template <int R, int U, bool NT, int BS>
const void* pick_k(int k) {
    switch (k) {
        case 2: return vec_fn<2, R, U, NT, BS>();
        case 3: return vec_fn<3, R, U, NT, BS>();
        case 6: return vec_fn<6, R, U, NT, BS>();
        case 10: return vec_fn<10, R, U, NT, BS>();
        default: return vec_fn<0, R, U, NT, BS>();
    }
}

template <int U, bool NT, int BS>
const void* pick_r(int k, int r) {
    switch (r) {
        case 1: return pick_k<1, U, NT, BS>(k);
        case 2: return pick_k<2, U, NT, BS>(k);
        case 3: return pick_k<3, U, NT, BS>(k);
        default: return pick_k<4, U, NT, BS>(k);
    }
}

#ifdef HEC_EXPERIMENTAL
// Measurement build: every shape a knob can ask for, (chunks per lane U,
// block size BS) in {(1,256),(2,256),(4,256),(1,512),(2,512)} plus (8,256)
// for k <= 3, each with and without non-temporal access.
template <bool NT>
const void* pick_shape(int k, int r, int unroll, int bs) {
    if (bs == 512) return unroll >= 2 ? pick_r<2, NT, 512>(k, r) : pick_r<1, NT, 512>(k, r);
    if (unroll == 8 && (k == 2 || k == 3)) {
        switch (r) {
            case 1: return k == 2 ? vec_fn<2, 1, 8, NT, 256>() : vec_fn<3, 1, 8, NT, 256>();
            case 2: return k == 2 ? vec_fn<2, 2, 8, NT, 256>() : vec_fn<3, 2, 8, NT, 256>();
            case 3: return k == 2 ? vec_fn<2, 3, 8, NT, 256>() : vec_fn<3, 3, 8, NT, 256>();
            default: return k == 2 ? vec_fn<2, 4, 8, NT, 256>() : vec_fn<3, 4, 8, NT, 256>();
        }
    }
    if (unroll >= 4) return pick_r<4, NT, 256>(k, r);
    if (unroll == 2) return pick_r<2, NT, 256>(k, r);
    return pick_r<1, NT, 256>(k, r);
}
#endif

// The register kernel for a launch shape.  The product library compiles only
// the default shapes (default_shape below): (4, 256) for k <= 6 and (2, 512)
// above, non-temporal.
template <typename Sh>
const void* pick_vec(int k, int r, const Sh& sh) {
#ifdef HEC_EXPERIMENTAL
    return sh.nt ? pick_shape<true>(k, r, sh.unroll, sh.block) : pick_shape<false>(k, r, sh.unroll, sh.block);
#else
    return sh.block == 512 ? pick_r<2, true, 512>(k, r) : pick_r<4, true, 256>(k, r);
#endif
}

template <int R, int U, int BS>
const void* dma_pick_k(int k) {
    switch (k) {
        case 2: return reinterpret_cast<const void*>(&gf_matmul_dma<2, R, U, BS>);
        case 3: return reinterpret_cast<const void*>(&gf_matmul_dma<3, R, U, BS>);
        case 6: return reinterpret_cast<const void*>(&gf_matmul_dma<6, R, U, BS>);
        default: return nullptr;
    }
}

template <int U, int BS>
const void* dma_pick(int k, int r) {
    switch (r) {
        case 1: return dma_pick_k<1, U, BS>(k);
        case 2: return dma_pick_k<2, U, BS>(k);
        case 3: return dma_pick_k<3, U, BS>(k);
        default: return dma_pick_k<4, U, BS>(k);
    }
}

// LDS-DMA pipelined kernel: the product default is (4, 256) for k in {2, 3,
// 6}; the measurement build adds (2,256), (2,512) and k = 10 at (2,256)
// (10 x 2 x 4 waves x 1 KiB = 80 KiB of LDS).
const void* pick_dma(int k, int r, int unroll, int bs) {
#ifndef HEC_EXPERIMENTAL
    // the product runs the register kernel on the work queue at every cell
    // size (default_shape); the LDS-DMA kernel is measurement-only
    (void)k;
    (void)r;
    (void)unroll;
    (void)bs;
    return nullptr;
#else
    if (k == 10) {
        switch (r) {
            case 1: return reinterpret_cast<const void*>(&gf_matmul_dma<10, 1, 2, 256>);
            case 2: return reinterpret_cast<const void*>(&gf_matmul_dma<10, 2, 2, 256>);
            case 3: return reinterpret_cast<const void*>(&gf_matmul_dma<10, 3, 2, 256>);
            default: return reinterpret_cast<const void*>(&gf_matmul_dma<10, 4, 2, 256>);
        }
    }
    if (bs == 512) return dma_pick<2, 512>(k, r);
    if (unroll == 4) return dma_pick<4, 256>(k, r);
    return dma_pick<2, 256>(k, r);
#endif
}

// register kernel with the work queue, default shapes only
template <int WQ, int R>
const void* wq_vec_k(int k) {
    switch (k) {
        case 2: return reinterpret_cast<const void*>(&gf_matmul_v16<2, R, 4, true, 256, WQ>);
        case 3: return reinterpret_cast<const void*>(&gf_matmul_v16<3, R, 4, true, 256, WQ>);
        case 6: return reinterpret_cast<const void*>(&gf_matmul_v16<6, R, 4, true, 256, WQ>);
        case 10: return reinterpret_cast<const void*>(&gf_matmul_v16<10, R, 2, true, 512, WQ>);
        default: return nullptr;
    }
}
template <int WQ>
const void* wq_vec(int k, int r) {
    switch (r) {
        case 1: return wq_vec_k<WQ, 1>(k);
        case 2: return wq_vec_k<WQ, 2>(k);
        case 3: return wq_vec_k<WQ, 3>(k);
        default: return wq_vec_k<WQ, 4>(k);
    }
}
#ifdef HEC_EXPERIMENTAL
// measurement: k = 10 in 256-thread blocks (key 4 = 256, key 1 = 2 or 4) on the queue
template <int WQ, int U>
const void* wq_vec_k10_256(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_matmul_v16<10, 1, U, true, 256, WQ>);
        case 2: return reinterpret_cast<const void*>(&gf_matmul_v16<10, 2, U, true, 256, WQ>);
        case 3: return reinterpret_cast<const void*>(&gf_matmul_v16<10, 3, U, true, 256, WQ>);
        default: return reinterpret_cast<const void*>(&gf_matmul_v16<10, 4, U, true, 256, WQ>);
    }
}
#endif

const void* pick_wq(int k, int r, int wq, int block = 0, int unroll = 0) {
#ifdef HEC_EXPERIMENTAL
    if (k == 10 && block == 256 && unroll == 4) return wq_vec_k10_256<1, 4>(r);
    if (k == 10 && block == 256) return wq == 2 ? wq_vec_k10_256<2, 2>(r) : wq_vec_k10_256<1, 2>(r);
    return wq == 2 ? wq_vec<2>(k, r) : wq_vec<1>(k, r);
#else
    (void)block;
    // the product compiles the default batch per k (default_wq)
    if (k == 2 || k == 3) return wq == 2 ? wq_vec<2>(k, r) : nullptr;
    return wq == 1 ? wq_vec<1>(k, r) : nullptr;
#endif
}

// The wave-pair kernel for k = 10 (tune key 32 = 1, measurement build).
const void* pick_pair(int k, int r) {
#ifdef HEC_EXPERIMENTAL
    if (k == 10) {
        switch (r) {
            case 1: return reinterpret_cast<const void*>(&gf_matmul_pair<10, 1, 4>);
            case 2: return reinterpret_cast<const void*>(&gf_matmul_pair<10, 2, 4>);
            case 3: return reinterpret_cast<const void*>(&gf_matmul_pair<10, 3, 4>);
            default: return reinterpret_cast<const void*>(&gf_matmul_pair<10, 4, 4>);
        }
    }
#endif
    (void)k;
    (void)r;
    return nullptr;
}

// Rounds of wave-tiles per atomic: same process, same buffers, 2 sets x 5
// alternated rounds of the bench step (encode + decode of data 0..m-1;
// scripts/probe_matmul_wq.py, profiles/r05t): RS(6,3) x 1024 0.795-0.798 of
// HBM peak at 1 vs 0.739-0.747 for the fixed order (0.780-0.782 at 2),
// RS(3,2) x 1024 0.775-0.776 at 2 (0.752-0.753 at 1) vs 0.711-0.713,
// RS(10,4) x 256 0.740 at 1 vs 0.729-0.732.
int default_wq(int k) { return k == 2 || k == 3 ? 2 : (k == 6 || k == 10) ? 1 : 0; }

#ifdef HEC_EXPERIMENTAL
// Bit-sliced encode for the (K, R) pairs with a generated network (K > 2:
// RS(2,1)'s network is no shorter than its tables); nullptr otherwise.
template <int K, int R>
const void* bsl_fn(int block) {
    if constexpr (bitslice::rs_net_available<K, R>() && K > 2) {
        if (block == 512) return reinterpret_cast<const void*>(&gf_encode_bsl<K, R, 2, 512>);
        return reinterpret_cast<const void*>(&gf_encode_bsl<K, R, 4, 256>);
    }
    (void)block;
    return nullptr;
}

template <typename Sh>
const void* pick_bsl(int k, int r, const Sh& sh) {
    if (sh.unroll != (sh.block == 512 ? 2 : 4)) return nullptr;  // the compiled shapes only
    switch (k) {
        case 3: return r == 2 ? bsl_fn<3, 2>(sh.block) : nullptr;
        case 6: return r == 3 ? bsl_fn<6, 3>(sh.block) : nullptr;
        case 10: return r == 4 ? bsl_fn<10, 4>(sh.block) : nullptr;
        default: return nullptr;
    }
}

// LDS-DMA kernel with the bit-sliced RS parity (the product's (4, 256) shape)
const void* pick_dma_bsl(int k, int r, int unroll, int bs) {
    if (unroll != 4 || bs != 256) return nullptr;
    if (k == 3 && r == 2) return reinterpret_cast<const void*>(&gf_matmul_dma<3, 2, 4, 256, true>);
    if (k == 6 && r == 3) return reinterpret_cast<const void*>(&gf_matmul_dma<6, 3, 4, 256, true>);
    return nullptr;
}
#endif  // HEC_EXPERIMENTAL

// Launch shape chosen from the MI355X sweeps in DESIGN.md ("Tuning"): long
// per-wave runs (4 x 1 KiB per stream) at one 256-thread block per CU keep
// the fewest DRAM rows open for a given bytes-in-flight.
struct Shape {
    int unroll, block, blocks_per_cu;
    bool nt;
    bool dma;
};

Shape default_shape(int k, uint64_t cell_len) {
    // RS(10,4): 20 x 1 KiB loads in flight per wave already.  One 512-thread
    // block is resident per CU; a grid of 8 per CU (8 rounds) beats 2 by 3 %
    // at 256-512 stripes and ties at 2048 (profiles/r01f_probe_bpc_k10_*.log)
    if (k > 6) return {2, 512, 8, true, false};
    // RS(3,2), RS(6,3): one wave per SIMD, 4 x 1 KiB per stream per wave.
    // Every cell size takes the register kernel on the work queue since round
    // 5.  Before, cells <= 256 KiB took the LDS-DMA kernel (2-3 % over the
    // register kernel in the fixed order, profiles/r01_probe_dma_pipeline.log);
    // the queue's wave-tiles (4 KiB per cell) beat it at every small size:
    // same process and buffers, encode + decode of data 0..2, RS(6,3)
    // (scripts/probe_matmul_wq.py PROBE_C64K=1, profiles/r05ac, r05ad): 64 KiB
    // x 65536 0.785-0.788 of HBM peak vs 0.766-0.774 for the LDS-DMA kernel;
    // 4 / 8 / 16 / 128 / 256 KiB 0.758 / 0.775 / 0.803 / 0.787 / 0.778 vs
    // 0.256 / 0.500 / 0.748 / 0.691 / 0.710 (the fixed order's 16-KiB block
    // tiles left most lanes of a small cell idle).  Measurement build: tune
    // key 5 = 2 for the LDS-DMA kernel.
    (void)k;
    (void)cell_len;
    return {4, 256, 1, true, false};
}

}  // namespace

// ---------------------------------------------------------------------------
// Work-queue counter sets (DESIGN.md §3.1 "Counter sets", round 6).  A set is
// kMixedQueues counters kMixedQueueStride bytes apart (2 KiB).
//  * Direct launches: every stream has two sets and alternates between them.
//    Launch i counts on set i % 2 and zeroes set (i + 1) % 2 from its block 0
//    (queue_zero_next) -- the set launch i-1 used, which has completed since
//    a stream runs its launches in order.  So a launch starts on zeroed
//    counters whatever the previous launch left behind: a miscount, an early
//    exit or a fault can no longer leak tiles into the next launch.  Both sets
//    are zeroed on the stream when the stream is first seen.
//  * Streams are keyed by hipStreamGetId where the HIP runtime in the
//    process has it (ROCm >= 7.1; looked up at run time, so the library
//    still loads next to an older runtime such as the one a torch wheel
//    bundles): ids are unique for the process's life, handles are not.
//    Otherwise by handle: a handle comes back only after hipStreamDestroy,
//    which waits for the stream's work (scripts/probe_stream_id.py), so the
//    new stream inherits sets whose last launch has completed -- the same
//    state a stream's next launch sees.  hipStreamPerThread is a different
//    stream in every thread under one handle: its sets are thread_local
//    (only the owning thread launches on them).
//  * Stream capture: a launch into a capturing stream takes a set of its own
//    from the device's graph pool (allocated outside any capture by
//    queue_reserve) and a memset node zeroing it is captured right before the
//    kernel, so every replay starts from zero and no replay shares counters
//    with direct launches on the capture stream or another graph.  Graph sets
//    are never returned (the graph may be replayed at any time).
//  * Bounds: kMaxStreamSets streams and kGraphSets graph launches per device.
//    Past them (or when HIP refuses an allocation / a query) the lease is
//    empty and the caller launches the fixed-order kernel: slower, never
//    wrong.  Stream sets are never freed (a destroyed stream's id never comes
//    back, but its last launch may still be in flight when it is destroyed).
// ---------------------------------------------------------------------------
namespace {

constexpr size_t kSetBytes = size_t(kMixedQueues) * kMixedQueueStride;
constexpr size_t kMaxStreamSets = 4096;  // 2 sets x 2 KiB each: 16 MiB per device at most
constexpr size_t kGraphSets = 256;       // 512 KiB per device

struct StreamSets {
    std::mutex mu;
    uint32_t* set[2] = {nullptr, nullptr};
    unsigned cur = 0;     // the set the stream's next launch counts on
    bool zeroed = false;  // both sets zeroed on the stream (its first lease)
};

struct DeviceQueues {
    std::mutex mu;
    std::map<unsigned long long, std::unique_ptr<StreamSets>> streams;  // by stream id (or handle)
    std::vector<std::unique_ptr<StreamSets>> thread_sets;                // hipStreamPerThread, one per thread
    uint32_t* graph_pool = nullptr;
    size_t graph_next = 0;
    bool reserved = false;
};

DeviceQueues& device_queues(int device) {
    static std::mutex mu;
    static std::map<int, std::unique_ptr<DeviceQueues>> all;
    std::lock_guard<std::mutex> lk(mu);
    auto& d = all[device];
    if (!d) d.reset(new DeviceQueues);
    return *d;
}

}  // namespace

QueueLease::QueueLease(QueueLease&& o) noexcept : use(o.use), zero(o.zero), st_(o.st_) {
    o.use = o.zero = nullptr;
    o.st_ = nullptr;
}

QueueLease& QueueLease::operator=(QueueLease&& o) noexcept {
    if (this != &o) {
        if (st_) static_cast<StreamSets*>(st_)->mu.unlock();
        use = o.use;
        zero = o.zero;
        st_ = o.st_;
        o.use = o.zero = nullptr;
        o.st_ = nullptr;
    }
    return *this;
}

QueueLease::~QueueLease() {
    if (st_) static_cast<StreamSets*>(st_)->mu.unlock();
}

void QueueLease::launched() {
    if (st_) static_cast<StreamSets*>(st_)->cur ^= 1u;
}

void queue_reserve(int device) {
    DeviceQueues& d = device_queues(device);
    std::lock_guard<std::mutex> lk(d.mu);
    if (d.reserved) return;
    d.reserved = true;
    void* p = nullptr;
    if (hipMalloc(&p, kGraphSets * kSetBytes) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    d.graph_pool = static_cast<uint32_t*>(p);
}

void queue_stats(int device, uint64_t* streams, uint64_t* graph_sets) {
    DeviceQueues& d = device_queues(device);
    std::lock_guard<std::mutex> lk(d.mu);
    if (streams) *streams = d.streams.size() + d.thread_sets.size();
    if (graph_sets) *graph_sets = d.graph_next;
}

namespace {

typedef hipError_t (*StreamGetIdFn)(hipStream_t, unsigned long long*);

// hipStreamGetId of the HIP runtime this library is bound to, or nullptr
StreamGetIdFn stream_get_id() {
    static const StreamGetIdFn fn = []() -> StreamGetIdFn {
        Dl_info info;
        if (!dladdr(reinterpret_cast<void*>(&hipMemsetAsync), &info) || !info.dli_fname) return nullptr;
        void* h = dlopen(info.dli_fname, RTLD_LAZY | RTLD_NOLOAD);
        if (!h) return nullptr;
        void* f = dlsym(h, "hipStreamGetId");
        dlclose(h);  // NOLOAD: only drops the reference just taken
        return reinterpret_cast<StreamGetIdFn>(f);
    }();
    return fn;
}

// new sets for a stream: both zeroed on the stream itself (ordered before
// the stream's first queue kernel); nullptr when HIP refuses
std::unique_ptr<StreamSets> make_sets() {
    std::unique_ptr<StreamSets> n(new StreamSets);
    void* p = nullptr;
    if (hipMalloc(&p, 2 * kSetBytes) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    n->set[0] = static_cast<uint32_t*>(p);
    n->set[1] = n->set[0] + kSetBytes / 4;
    return n;
}

}  // namespace

int queue_keyed_by_id() { return stream_get_id() ? 1 : 0; }

QueueLease queue_lease(int device, hipStream_t stream) {
    QueueLease l;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cap) != hipSuccess) {
        (void)hipGetLastError();
        return l;  // e.g. the legacy stream while another stream captures
    }
    DeviceQueues& d = device_queues(device);
    if (cap != hipStreamCaptureStatusNone) {
        if (cap != hipStreamCaptureStatusActive) return l;  // invalidated capture: nothing to add to
        uint32_t* set = nullptr;
        {
            std::lock_guard<std::mutex> lk(d.mu);
            if (d.graph_pool && d.graph_next < kGraphSets) set = d.graph_pool + d.graph_next++ * (kSetBytes / 4);
        }
        if (!set) return l;
        if (hipMemsetAsync(set, 0, kSetBytes, stream) != hipSuccess) {  // captured: a memset node
            (void)hipGetLastError();
            return l;
        }
        l.use = set;
        return l;
    }
    StreamSets* st = nullptr;
    if (stream == hipStreamPerThread) {
        // this thread's own stream: sets of its own, per device (kept for
        // the thread's life and after: its last launches may be in flight)
        thread_local std::map<int, StreamSets*> mine;
        StreamSets*& t = mine[device];
        if (!t) {
            std::lock_guard<std::mutex> lk(d.mu);
            if (d.streams.size() + d.thread_sets.size() >= kMaxStreamSets) return l;
            std::unique_ptr<StreamSets> n = make_sets();
            if (!n) return l;
            t = n.get();
            d.thread_sets.push_back(std::move(n));
        }
        st = t;
    } else {
        unsigned long long key = reinterpret_cast<uintptr_t>(stream);
        if (StreamGetIdFn get_id = stream_get_id()) {
            if (get_id(stream, &key) != hipSuccess) {
                (void)hipGetLastError();
                return l;
            }
        }
        std::lock_guard<std::mutex> lk(d.mu);
        auto it = d.streams.find(key);
        if (it != d.streams.end()) {
            st = it->second.get();
        } else if (d.streams.size() + d.thread_sets.size() < kMaxStreamSets) {
            std::unique_ptr<StreamSets> n = make_sets();
            if (!n) return l;
            st = n.get();
            d.streams.emplace(key, std::move(n));
        }
    }
    if (!st) return l;
    st->mu.lock();
    if (!st->zeroed) {
        // first launch on this stream: both sets zeroed on the stream itself
        if (hipMemsetAsync(st->set[0], 0, 2 * kSetBytes, stream) != hipSuccess) {
            (void)hipGetLastError();
            st->mu.unlock();
            return l;  // the stream's next lease tries again
        }
        st->zeroed = true;
    }
    l.st_ = st;
    l.use = st->set[st->cur];
    l.zero = st->set[st->cur ^ 1u];
    return l;
}

bool rs_parity_matrix(const MatmulArgs& a) {
    if (a.k < 1 || a.k > kMaxK || a.r < 1 || a.r > kMaxR) return false;
    for (int j = 0; j < a.r; j++)
        for (int i = 0; i < a.k; i++) {
            const uint8_t s = uint8_t(a.k + j) ^ uint8_t(i);
            if (a.coef[j * kMaxK + i] != (s == 0 ? 0 : gf_div(1, s))) return false;
        }
    return true;
}

int launch_gf_matmul(const MatmulArgs& in, int device, hipStream_t stream) {
    MatmulArgs a = in;
    const Tune tn = tune_snapshot();
    bool aligned = true;
    for (int i = 0; i < a.k; i++)
        aligned &= ((reinterpret_cast<uintptr_t>(a.in[i]) | a.in_stride[i]) & 15u) == 0;
    for (int j = 0; j < a.r; j++)
        aligned &= ((reinterpret_cast<uintptr_t>(a.out[j]) | a.out_stride[j]) & 15u) == 0;
    // vector kernels address a cell with 32-bit lane offsets: cells of 4 GiB
    // or more (HDFS cell sizes are int32) take the byte kernel
    const uint64_t chunks = (aligned && a.cell_len < (uint64_t(1) << 32)) ? a.cell_len / 16 : 0;
    const int cus = num_cus(device);

    if (chunks > 0) {
        Shape sh = default_shape(a.k, a.cell_len);
        if (tn.unroll) sh.unroll = tn.unroll == 3 ? 2 : tn.unroll;
        if (tn.block) sh.block = tn.block;
        if (tn.nt >= 0) sh.nt = tn.nt != 0;
        if (tn.blocks_per_cu) sh.blocks_per_cu = tn.blocks_per_cu;
        if (tn.pipeline == 1 || tn.pipeline == 2) sh.dma = tn.pipeline == 2;
        if (sh.block == 512 && sh.unroll > 2) sh.unroll = 2;
        const bool dma_ok = (a.k == 2 || a.k == 3 || a.k == 6 || a.k == 10);
        if (sh.dma && !dma_ok) sh.dma = false;
        if (sh.dma) {
            if (a.k == 10) {
                sh.unroll = 2;
                sh.block = 256;
            } else if (sh.block == 512) {
                sh.unroll = 2;
            } else if (sh.unroll < 2) {
                sh.unroll = 2;
            }
        }
        const void* fn = nullptr;
        QueueLease lease;   // work-queue counters (held until the launch is enqueued)
        const int tile_mult = 1;  // column tiles per scheduling unit
#ifdef HEC_EXPERIMENTAL
        // bit-sliced RS parity in the register / LDS-DMA kernels (tune key 23
        // = 1).  Measured and not kept: same box, RS(6,3) 1
        // MiB encode 3438-3451 vs 3671-3701 GiB/s with the v_perm tables;
        // RS(3,2) and 64 KiB cells within noise
        if (!fn && tn.matmul_bsl == 1 && sh.unroll % 2 == 0 && rs_parity_matrix(a))
            fn = sh.dma ? pick_dma_bsl(a.k, a.r, sh.unroll, sh.block) : pick_bsl(a.k, a.r, sh);
#endif
        // the register kernel's default shapes take the work queue (tune key
        // 27, measurement build: 1 / 2 rounds per atomic, 3 = the fixed order)
        int wq = 0;
        bool pair = false;  // the wave-pair kernel (k = 10; tune key 32)
        if (!fn && tn.matmul_pair == 1 && sh.nt) {
            const void* f = pick_pair(a.k, a.r);
            if (f) lease = queue_lease(device, stream);
            if (f && lease) {
                fn = f;
                pair = true;
                wq = 1;
                a.queue = lease.use;
                a.queue_zero = lease.zero;
                sh.unroll = 4;
                sh.block = 128;
                if (!tn.blocks_per_cu) sh.blocks_per_cu = 4;  // two waves per SIMD
            }
        }
        const bool k10_256 = kExperimental && a.k == 10 && sh.block == 256 && (sh.unroll == 2 || sh.unroll == 4);  // measurement
        if (!fn && !pair && !sh.dma && sh.nt &&
            ((sh.unroll == (sh.block == 512 ? 2 : 4) && (sh.block == 512) == (a.k == 10)) || k10_256)) {
            wq = default_wq(a.k);
            if (kExperimental && tn.matmul_wq) wq = tn.matmul_wq == 3 ? 0 : tn.matmul_wq;
            const void* f = wq ? pick_wq(a.k, a.r, wq, sh.block, sh.unroll) : nullptr;
            if (f) lease = queue_lease(device, stream);
            a.queue = lease.use;
            a.queue_zero = lease.zero;
            if (a.queue) {
                fn = f;
                if (!tn.blocks_per_cu) sh.blocks_per_cu = 1;  // resident blocks only: each one drains the queue
            } else {
                wq = 0;
            }
        }
        if (!fn) fn = sh.dma ? pick_dma(a.k, a.r, sh.unroll, sh.block) : pick_vec(a.k, a.r, sh);
        if (!fn) return -1;
        const uint64_t tile = uint64_t(wq ? 64 : sh.block) * sh.unroll * tile_mult;
        const uint64_t tps = (chunks + tile - 1) / tile;
        const uint64_t total = tps * a.stripes;
        if (chunks > 0xFFFFFFFFull || total > 0xFFF00000ull) return -1;  // tile indices (+ a prefetch stride) in 32 bits
        a.chunks = uint32_t(chunks);
        a.tiles_per_stripe = uint32_t(tps);
        a.total_tiles = uint32_t(total);
        // 4 stripes column-interleaved: +1-4 % over stripe-major at 1 MiB
        // cells (profiles/r01_probe_tile_order.log)
        tile_order(a.stripes, a.tiles_per_stripe, tn.group > 0 ? uint32_t(tn.group) : 4u, a.group, a.grouped_tiles);
        // stores drained before the next tile's loads unless key 6 = 1: same-box
        // bench A/B (profiles/r02_drain_ab.txt): RS(6,3) 1 MiB 3702 vs 3514
        // GiB/s, RS(10,4) 3926 vs 3906, RS(3,2) 3089 vs 3075 -- DRAM prefers a
        // wave's writes and its next reads in separate bursts
        a.drain = tn.drain == 1 ? 0u : 1u;
        uint64_t grid = tn.grid ? uint64_t(tn.grid) : uint64_t(cus) * sh.blocks_per_cu;
        if (grid > total) grid = total;
        void* args[] = {&a};
        const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(sh.block), args, 0, stream);
        if (e != hipSuccess) return int(e);
        lease.launched();
    }
    uint64_t begin = chunks * 16;
    if (begin == 0 && !aligned && a.cell_len >= 8 && a.r >= 1 && a.r <= kMaxR && tn.unaligned != 1) {
        // unaligned layout: the dword kernel up to the last whole 8 bytes,
        // the byte kernel after (tune key 18 = 1: the byte kernel alone)
        const uint64_t total = (a.cell_len / 8) * a.stripes;
        uint64_t grid = (total + 255) / 256;
        const uint64_t cap = uint64_t(cus) * 8;
        if (grid > cap) grid = cap;
        const void* fn = a.r == 1   ? reinterpret_cast<const void*>(&gf_matmul_dw<1>)
                         : a.r == 2 ? reinterpret_cast<const void*>(&gf_matmul_dw<2>)
                         : a.r == 3 ? reinterpret_cast<const void*>(&gf_matmul_dw<3>)
                                    : reinterpret_cast<const void*>(&gf_matmul_dw<4>);
        void* args[] = {&a};
        const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(256), args, 0, stream);
        if (e != hipSuccess) return int(e);
        begin = (a.cell_len / 8) * 8;
    }
    if (begin < a.cell_len) {
        a.byte_begin = begin;
        const uint64_t total = (a.cell_len - begin) * a.stripes;
        uint64_t grid = (total + kBlock - 1) / kBlock;
        const uint64_t cap = uint64_t(cus) * 8;
        if (grid > cap) grid = cap;
        void* args[] = {&a};
        const hipError_t e = hipLaunchKernel(reinterpret_cast<const void*>(&gf_matmul_bytes), dim3(uint32_t(grid)),
                                             dim3(kBlock), args, 0, stream);
        if (e != hipSuccess) return int(e);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : int(e);
}

namespace {

template <int K, int R, bool RES, bool SKIP, int WQ = 0>
const void* mixed_fn() {
    if constexpr (K > 6)
        return reinterpret_cast<const void*>(&gf_decode_mixed<K, R, 2, 512, RES, SKIP, WQ>);
    else
        return reinterpret_cast<const void*>(&gf_decode_mixed<K, R, 4, 256, RES, SKIP, WQ>);
}

// The product library compiles the default row policy only (rows past a
// stripe's e skipped); the measurement build both (tune key 20).
template <int K, int R>
const void* mixed_sel(bool res, bool skip, int wq) {
    if (res && skip && wq == 1) return mixed_fn<K, R, true, true, 1>();
    if (res && skip && wq == 4) return mixed_fn<K, R, true, true, 4>();
#ifdef HEC_EXPERIMENTAL
    if (res && skip && wq == 2) return mixed_fn<K, R, true, true, 2>();
    return res ? (skip ? mixed_fn<K, R, true, true>() : mixed_fn<K, R, true, false>())
               : (skip ? mixed_fn<K, R, false, true>() : mixed_fn<K, R, false, false>());
#else
    (void)skip;
    return res ? mixed_fn<K, R, true, true>() : mixed_fn<K, R, false, true>();
#endif
}

template <int K>
const void* mixed_pick_r(int r, bool res, bool skip, int wq) {
    switch (r) {
        case 1: return mixed_sel<K, 1>(res, skip, wq);
        case 2: return mixed_sel<K, 2>(res, skip, wq);
        case 3: return mixed_sel<K, 3>(res, skip, wq);
        default: return mixed_sel<K, 4>(res, skip, wq);
    }
}

// LDS budget for a resident launch: the stripes' plan offsets plus every
// plan.  gfx950 has 160 KiB of LDS per CU and the mixed kernel's static LDS
// is under 2 KiB; dynamic LDS past 64 KiB needs the function attribute
// (hipFuncAttributeMaxDynamicSharedMemorySize), set at launch.  At 64 KiB,
// RS(10,4) x 256 stripes with random 1..4 data losses (144 plans, 149 KB)
// ran non-resident: per-stripe restaging and stripe-major tiles.
constexpr uint64_t kResidentMax = 156u << 10;
constexpr uint64_t kDynNoAttr = 64u << 10;

}  // namespace

int launch_decode_mixed(const MixedArgs& in, int rows, int device, hipStream_t stream) {
    MixedArgs a = in;
    const Tune tn = tune_snapshot();
    if (a.cell_len % 16 != 0 || a.cell_len / 16 > 0xFFFFFFFFull) return -1;
    const uint64_t dyn = ((a.stripes * 4 + 15) & ~uint64_t(15)) + a.blob_bytes;
    bool res = dyn <= kResidentMax && a.blob_bytes % 4 == 0;
    // rows past a stripe's e skipped behind a scalar branch: RS(6,3) mixed
    // +1.7 % (profiles/r02_ab_mixed_skip.txt); RS(10,4) x 256 decode +9.5 %
    // since the tile metadata moved to three LDS round trips and global loads
    // (same box, profiles/r03g/mx10: 4049-4074 vs 3683-3726 GiB/s; in round 2,
    // with the serial metadata and flat loads, skipping lost 3.5-4 % there).
    // Tune key 20: 1 = compute every row (measurement), 0 / 2 = skip.
    const bool skip = tn.mixed_skip != 1;
    // Work queue of wave-tiles over kMixedQueues counters (round 5), one
    // round per atomic for k >= 6, four below (more atomics per byte there).
    // Same process and buffers, 2 sets x 5 alternated rounds
    // (scripts/probe_mixed_wq.py, profiles/r05r): RS(10,4) x 256 0.658-0.662
    // vs 0.639-0.642 for the fixed order, RS(6,3) x 1024 0.744-0.755 vs
    // 0.683-0.699, RS(3,2) x 1024 (4 per atomic) 0.708-0.712 vs 0.674-0.715.
    // One counter measured 2-4x slower at one round per atomic (device-scope
    // atomics on one address top out near 85 M/s) and 16 or 64 per atomic
    // widened the DRAM window (slower again).  Tune key 26 (measurement
    // build): 1 / 2 / 4 rounds per atomic, 3 = the fixed order.  Needs the
    // launch counters (a.queue) and resident plans.
    int wq = (a.queue && skip) ? (a.k >= 6 ? 1 : 4) : 0;
    if (kExperimental && tn.mixed_wq) wq = tn.mixed_wq == 3 ? 0 : tn.mixed_wq;
    auto pick = [&](bool resident) -> const void* {
        const int w = resident ? wq : 0;
        switch (a.k) {
            case 2: return mixed_pick_r<2>(rows, resident, skip, w);
            case 3: return mixed_pick_r<3>(rows, resident, skip, w);
            case 6: return mixed_pick_r<6>(rows, resident, skip, w);
            case 10: return mixed_pick_r<10>(rows, resident, skip, w);
            default: return nullptr;
        }
    };
    const void* fn = pick(res);
    if (!fn) return -1;
    // The attribute is set to the resident ceiling, never to this launch's
    // size: a coder may be shared by threads, and one thread lowering the
    // limit between another's set and launch would fail that launch.
    if (res && dyn > kDynNoAttr &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(kResidentMax)) != hipSuccess) {
        (void)hipGetLastError();
        res = false;  // the runtime refused the LDS: restage per stripe instead
        fn = pick(false);
    }
    if (!res) wq = 0;
    const int U = a.k > 6 ? 2 : 4, BS = a.k > 6 ? 512 : 256;
    // K > 6: a grid of 8 per CU (one resident): RS(10,4) mixed decode 3216-3234
    // -> 3524-3621 GiB/s against 2 per CU
    const int bpc = tn.blocks_per_cu ? tn.blocks_per_cu : (a.k > 6 ? 8 : 1);
    const uint64_t chunks = a.cell_len / 16;
    const uint64_t tile = uint64_t(wq ? 64 : BS) * U;  // WQ: wave-tiles
    const uint64_t tps = (chunks + tile - 1) / tile;
    const uint64_t total = tps * a.stripes;
    if (total > 0xFFFFFFFFull) return -1;
    if (total == 0) return 0;
    a.chunks = uint32_t(chunks);
    a.tiles_per_stripe = uint32_t(tps);
    a.total_tiles = uint32_t(total);
    tile_order(a.stripes, a.tiles_per_stripe, tn.group > 0 ? uint32_t(tn.group) : 4u, a.group, a.grouped_tiles);
    a.drain = tn.drain == 1 ? 0u : 1u;
    // WQ: one block per CU unless key 3 says otherwise (resident plans are
    // staged once per block)
    uint64_t grid = uint64_t(num_cus(device)) * (wq && !tn.blocks_per_cu ? 1 : bpc);
    if (grid > total) grid = total;
    void* args[] = {&a};
    const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(BS), args, res ? uint32_t(dyn) : 0u, stream);
    return e == hipSuccess ? 0 : int(e);
}

}  // namespace hec
