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
//  * Grid = resident blocks only, grid-stride over (stripe, column-tile)
//    tiles so the table prologue is paid once per block.
//  * Tails (cell_len % 16) and unaligned layouts use a byte-granular kernel
//    with LDS log/antilog lookups -- same results, correctness path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "ec_kernels.hpp"
#include "gf_device.hpp"

namespace hec {

// ---------------------------------------------------------------------------
// Vector kernel: 16 B per lane per shard, U column chunks per lane.
// K = compile-time input count (0 = runtime a.k), R = outputs (1..4).
// ---------------------------------------------------------------------------
// Column of chunk u of this lane within a tile.  MAP 0: chunk u of the
// block is a contiguous BS-lane slab (a wave's U pieces are BS*16 B apart);
// MAP 1: each wave owns U*64 contiguous chunks (one 4 KiB run per stream at
// U=4) and issues a stream's pieces back to back.
template <int U, int BS, int MAP>
__device__ __forceinline__ uint32_t chunk_col(uint32_t tile_base, int u, uint32_t tid) {
    if constexpr (MAP == 0)
        return tile_base + u * BS + tid;
    else
        return tile_base + (tid / 64) * (U * 64) + u * 64 + (tid & 63);
}

template <int K, int R, int U, bool NT, int BS, int MAP = 0>
__global__ __launch_bounds__(BS) void gf_matmul_v16(MatmulArgs a) {
    __shared__ PermTable s_tab[R][kMaxK];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    const int k = K ? K : a.k;
    prologue<R, BS>(a, k, s_tab, s_exp, s_log, s_coef);

    const uint32_t chunks = a.chunks;  // 16-B chunks per cell
    const uint32_t total = a.total_tiles;
    constexpr uint32_t TILE = BS * U;

    // Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8);
    // xcd_remap gives XCD x's blocks the contiguous logical range
    // [x * grid/8, (x+1) * grid/8) (launcher: grid % 8 == 0)
    const uint32_t first = a.xcd_remap ? (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u : blockIdx.x;
    for (uint32_t tile = first; tile < total; tile += gridDim.x) {
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
                const uint32_t col = chunk_col<U, BS, MAP>(tcol * TILE, u, threadIdx.x);
                live[u] = col < chunks;
                offs[u] = (live[u] ? col : 0u) * 16u;
            }
            if constexpr (MAP == 0) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int i = 0; i < K; i++)
                        x[u][i] = load16<NT>((a.in[i] + uint64_t(stripe) * a.in_stride[i]) + offs[u]);
            } else {
#pragma unroll
                for (int i = 0; i < K; i++)
#pragma unroll
                    for (int u = 0; u < U; u++)
                        x[u][i] = load16<NT>((a.in[i] + uint64_t(stripe) * a.in_stride[i]) + offs[u]);
            }
            __builtin_amdgcn_sched_barrier(0);
            u32x4 acc[U][R];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < K; i++) {
                // Opaque per-input table offset: input i's coefficient-table
                // reads cannot be hoisted above this point (otherwise the
                // compiler front-loads all R*K tables = R*K*5 VGPRs).
                uint32_t toff = uint32_t(i) * uint32_t(sizeof(PermTable));
                asm volatile("" : "+v"(toff));
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
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
                        for (int d = 0; d < 4; d++)
                            acc[u][j][d] ^= gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, s[u][d].s0, s[u][d].s1, s[u][d].s2);
                }
                // one input at a time: stops the scheduler from hoisting every
                // coefficient's table read (R*K*5 VGPRs) to the top
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (MAP == 0) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (!live[u]) continue;
#pragma unroll
                    for (int j = 0; j < R; j++)
                        store16<NT>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        if (!live[u]) continue;
                        store16<NT>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + offs[u], acc[u][j]);
                    }
            }
        } else {
            // Runtime K: one shard at a time, U chunks per lane.
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t col = chunk_col<U, BS, MAP>(tcol * TILE, u, threadIdx.x);
                if (col >= chunks) continue;
                const uint64_t off = uint64_t(col) * 16u;
                u32x4 acc[R];
#pragma unroll
                for (int j = 0; j < R; j++) acc[j] = u32x4{0, 0, 0, 0};
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
                            acc[j][d] ^= gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, s[d].s0, s[d].s1, s[d].s2);
                    }
                }
#pragma unroll
                for (int j = 0; j < R; j++) store16<NT>(a.out[j] + uint64_t(stripe) * a.out_stride[j] + off, acc[j]);
            }
        }
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
template <int K, int R, int U, int BS>
__global__ __launch_bounds__(BS) void gf_matmul_dma(MatmulArgs a) {
    static_assert(K > 0, "DMA kernel needs a compile-time input count");
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
// Output-burst kernel (measurement variant, tune key 5 = 4): a block takes T
// adjacent column tiles of one stripe, parks each tile's R x U accumulators
// in LDS (every lane its own 16-B pieces: no barrier), and only after the T
// tiles issues all the stores, stream by stream -- T x 16 KiB contiguous per
// output stream per block instead of 16 KiB, and T tiles of pure reads
// between write bursts.  tiles_per_stripe / total_tiles count super-tiles.
// ---------------------------------------------------------------------------
template <int K, int R, int T>
__global__ __launch_bounds__(256) void gf_matmul_burst(MatmulArgs a) {
    constexpr int U = 4, BS = 256;
    constexpr uint32_t TILE = BS * U;
    __shared__ PermTable s_tab[R][kMaxK];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    __shared__ u32x4 s_out[T][R][U][BS];
    prologue<R, BS>(a, K, s_tab, s_exp, s_log, s_coef);
    const uint32_t chunks = a.chunks;
    const uint32_t tid = threadIdx.x;
    for (uint32_t st = blockIdx.x; st < a.total_tiles; st += gridDim.x) {
        uint32_t stripe, scol;
        tile_coords(st, a, stripe, scol);
        int nt = 0;
#pragma unroll
        for (int t = 0; t < T; t++) {
            const uint32_t base = (scol * T + t) * TILE;
            if (base >= chunks) break;  // block-uniform
            nt = t + 1;
            asm volatile("" ::: "memory");
            u32x4 x[U][K];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t col = base + u * BS + tid;
                const uint64_t off = uint64_t(col < chunks ? col : 0) * 16u;
#pragma unroll
                for (int i = 0; i < K; i++) x[u][i] = load16<true>(a.in[i] + uint64_t(stripe) * a.in_stride[i] + off);
            }
            __builtin_amdgcn_sched_barrier(0);
            u32x4 acc[U][R];
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
                    const PermTable& tb =
                        *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
                    const uint32_t t0lo = tb.t0lo, t0hi = tb.t0hi, t1lo = tb.t1lo, t1hi = tb.t1hi, t2 = tb.t2;
#pragma unroll
                    for (int u = 0; u < U; u++)
#pragma unroll
                        for (int d = 0; d < 4; d++)
                            acc[u][j][d] ^= gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, sl[u][d].s0, sl[u][d].s1, sl[u][d].s2);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < R; j++) s_out[t][j][u][tid] = acc[u][j];
        }
        // the burst: every parked tile, one output stream after the other
#pragma unroll
        for (int j = 0; j < R; j++) {
            uint8_t* ob = a.out[j] + uint64_t(stripe) * a.out_stride[j];
#pragma unroll
            for (int t = 0; t < T; t++) {
                if (t >= nt) break;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const uint32_t col = (scol * T + t) * TILE + u * BS + tid;
                    if (col < chunks) store16<true>(ob + uint64_t(col) * 16u, s_out[t][j][u][tid]);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Register double-buffered kernel (compile-time K only).  Two register sets
// of K x U chunks: the loads of tile t+1 are issued before tile t is
// computed, so a wave always has one tile of loads in flight during its GF
// math (the LDS-DMA kernel's overlap without the LDS round trip).
//  * Loads and stores address as (uniform stripe base) + 32-bit lane offset
//    (global_* saddr form), and the next tile's coordinates are computed
//    while the accumulators are still live, before the stores: no VGPR
//    temporary is written after a store is issued, so the waitcnt pass never
//    has to drain the in-flight loads to protect store data registers.
//  * Per input, the U chunks are walked u-outer with all R coefficient
//    tables live, so only one chunk's selectors are live at a time.
// ---------------------------------------------------------------------------
template <int U>
struct PipeCoords {
    uint32_t stripe;
    uint32_t off[U];  // byte offset of chunk u (clamped into the cell)
    bool live[U];
};

template <int U, int BS>
__device__ __forceinline__ PipeCoords<U> pipe_coords(const MatmulArgs& a, uint32_t tile) {
    PipeCoords<U> c;
    uint32_t tcol;
    tile_coords(tile < a.total_tiles ? tile : a.total_tiles - 1, a, c.stripe, tcol);
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t col = tcol * (BS * U) + u * BS + threadIdx.x;
        c.live[u] = tile < a.total_tiles && col < a.chunks;
        c.off[u] = (col < a.chunks ? col : a.chunks - 1) * 16u;  // dead lanes fetch a valid chunk
    }
    return c;
}

template <int K, int U>
__device__ __forceinline__ void pipe_load(const MatmulArgs& a, const PipeCoords<U>& c, u32x4 (&x)[U][K]) {
#pragma unroll
    for (int i = 0; i < K; i++) {
        const uint8_t* base = a.in[i] + uint64_t(c.stripe) * a.in_stride[i];
#pragma unroll
        for (int u = 0; u < U; u++) x[u][i] = load16<true>(base + c.off[u]);
    }
}

template <int K, int R, int U>
__device__ __forceinline__ void pipe_compute(const u32x4 (&x)[U][K], const PermTable (*s_tab)[kMaxK],
                                             u32x4 (&acc)[U][R]) {
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
        uint32_t tb[R][5];
#pragma unroll
        for (int j = 0; j < R; j++) {
            const PermTable& t =
                *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
            tb[j][0] = t.t0lo;
            tb[j][1] = t.t0hi;
            tb[j][2] = t.t1lo;
            tb[j][3] = t.t1hi;
            tb[j][4] = t.t2;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int d = 0; d < 4; d++) {
                const Sel s = make_sel(x[u][i][d]);
#pragma unroll
                for (int j = 0; j < R; j++)
                    acc[u][j][d] ^= gf_mul4(tb[j][0], tb[j][1], tb[j][2], tb[j][3], tb[j][4], s.s0, s.s1, s.s2);
            }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R, int U, int POL>
__device__ __forceinline__ void pipe_store(const MatmulArgs& a, const PipeCoords<U>& c, const u32x4 (&acc)[U][R]) {
#pragma unroll
    for (int j = 0; j < R; j++) {
        uint8_t* base = a.out[j] + uint64_t(c.stripe) * a.out_stride[j];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (c.live[u]) store16p<POL>(base + c.off[u], acc[u][j]);
    }
}

template <int K, int R, int U, int BS, int POL = 0>
__global__ __launch_bounds__(BS) void gf_matmul_pipe(MatmulArgs a) {
    static_assert(K > 0, "pipelined kernel needs a compile-time input count");
    __shared__ PermTable s_tab[R][kMaxK];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    prologue<R, BS>(a, K, s_tab, s_exp, s_log, s_coef);
    const uint32_t total = a.total_tiles;
    const uint32_t step = gridDim.x;
    u32x4 xa[U][K], xb[U][K], acc[U][R];
    // Tiles past the end load a clamped (valid) tile and store nothing.
    uint32_t tile = blockIdx.x;
    PipeCoords<U> ca = pipe_coords<U, BS>(a, tile);
    PipeCoords<U> cb = pipe_coords<U, BS>(a, tile + step);
    pipe_load<K, U>(a, ca, xa);
    for (; tile < total; tile += 2 * step) {
        pipe_load<K, U>(a, cb, xb);  // tile + step
        __builtin_amdgcn_sched_barrier(0);
        pipe_compute<K, R, U>(xa, s_tab, acc);
        PipeCoords<U> cur = ca;
        ca = pipe_coords<U, BS>(a, tile + 2 * step);
        __builtin_amdgcn_sched_barrier(0);
        pipe_store<R, U, POL>(a, cur, acc);
        __builtin_amdgcn_sched_barrier(0);
        if (tile + step >= total) break;  // wave-uniform
        pipe_load<K, U>(a, ca, xa);  // tile + 2 step
        __builtin_amdgcn_sched_barrier(0);
        pipe_compute<K, R, U>(xb, s_tab, acc);
        cur = cb;
        cb = pipe_coords<U, BS>(a, tile + 3 * step);
        __builtin_amdgcn_sched_barrier(0);
        pipe_store<R, U, POL>(a, cur, acc);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ---------------------------------------------------------------------------
// Mixed-pattern decode: every stripe carries its own erasure pattern (plan
// index), as a striped read over many block groups does.  Same register
// kernel shape as gf_matmul_v16; per tile the block looks up the stripe's
// plan, re-stages its header + coefficient tables into LDS when the plan
// changes (block-uniform), and gathers the survivors by shard index.
// ---------------------------------------------------------------------------
template <int K, int R, int U, int BS, bool RESIDENT>
__global__ __launch_bounds__(BS) void gf_decode_mixed(MixedArgs a) {
    static_assert(K > 0, "compile-time k");
    __shared__ PermTable s_tab[R][K];
    __shared__ DevPlanHeader s_hdr;
    // RESIDENT: the whole plan blob (a.blob_bytes) is copied to dynamic LDS
    // once per block, so per-tile plan switches need no barrier.
    extern __shared__ __attribute__((aligned(16))) uint8_t s_blob[];
    if constexpr (RESIDENT) {
        const uint32_t words = a.blob_bytes / 4;
        for (uint32_t t = threadIdx.x; t < words; t += BS)
            reinterpret_cast<uint32_t*>(s_blob)[t] = reinterpret_cast<const uint32_t*>(a.plans)[t];
        __syncthreads();
    }
    const uint32_t chunks = a.chunks;
    const uint32_t total = a.total_tiles;
    constexpr uint32_t TILE = BS * U;
    uint32_t cur_plan = 0xFFFFFFFFu;
    MatmulArgs dummy;  // tile_coords only reads tiles_per_stripe/group/stripes
    dummy.tiles_per_stripe = a.tiles_per_stripe;
    dummy.group = a.group;
    dummy.stripes = a.stripes;

    // RESIDENT: grouped interleaved order (best DRAM locality).  Otherwise
    // each block walks a contiguous range of whole stripes, so its plan
    // changes (and LDS restaging with two barriers) once per stripe, not once
    // per tile.
    uint32_t t_begin = blockIdx.x, t_end = total, t_step = gridDim.x;
    if constexpr (!RESIDENT) {
        const uint32_t per = (total + gridDim.x - 1) / gridDim.x;
        t_begin = blockIdx.x * per;
        t_end = min(total, t_begin + per);
        t_step = 1;
        dummy.group = 1;
    }
    for (uint32_t tile = t_begin; tile < t_end; tile += t_step) {
        uint32_t stripe, tcol;
        tile_coords(tile, dummy, stripe, tcol);
        const uint32_t p = a.stripe_plan[stripe];
        if (p == 0xFFFFu) continue;
        const DevPlanHeader* hdr = &s_hdr;
        const PermTable* tab_base = &s_tab[0][0];
        int tab_row0 = 0;  // row of tab_base[0]
        if constexpr (RESIDENT) {
            hdr = reinterpret_cast<const DevPlanHeader*>(s_blob + a.plan_off[p]);
            tab_base = reinterpret_cast<const PermTable*>(s_blob + a.plan_off[p] + sizeof(DevPlanHeader));
            tab_row0 = a.row0;
        } else if (p != cur_plan) {  // block-uniform: every thread sees the same tile
            __syncthreads();
            const uint8_t* blob = a.plans + a.plan_off[p];
            const int tid = threadIdx.x;
            if (tid < 16) reinterpret_cast<uint32_t*>(&s_hdr)[tid] = reinterpret_cast<const uint32_t*>(blob)[tid];
            const uint32_t e_all = reinterpret_cast<const DevPlanHeader*>(blob)->e;
            const PermTable* tabs = reinterpret_cast<const PermTable*>(blob + sizeof(DevPlanHeader));
            for (int t = tid; t < R * K * 8; t += BS) {
                const int j = t / (K * 8), rem = t - j * (K * 8), i = rem / 8, w = rem - i * 8;
                const int row = a.row0 + j;
                reinterpret_cast<uint32_t*>(&s_tab[j][i])[w] =
                    row < int(e_all) ? reinterpret_cast<const uint32_t*>(&tabs[row * K + i])[w] : 0u;
            }
            __syncthreads();
            cur_plan = p;
        }
        const int e_all = int(hdr->e);
        const int nrows = e_all - a.row0;  // rows of this launch that exist for this plan
        if (nrows <= 0) continue;
        asm volatile("" ::: "memory");

        u32x4 x[U][K];
        bool live[U];
        uint64_t offs[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t col = tcol * TILE + u * BS + threadIdx.x;
            live[u] = col < chunks;
            offs[u] = uint64_t(live[u] ? col : 0) * 16u;
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int i = 0; i < K; i++) {
                const int sh = hdr->surv[i];
                x[u][i] = load16<true>(a.base[sh] + uint64_t(stripe) * a.stride[sh] + offs[u]);
            }
        __builtin_amdgcn_sched_barrier(0);
        u32x4 acc[U][R];
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
                if (j >= nrows) break;  // block-uniform
                const PermTable& t = *reinterpret_cast<const PermTable*>(
                    reinterpret_cast<const char*>(tab_base + (tab_row0 + j) * K) + toff);
                const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int d = 0; d < 4; d++)
                        acc[u][j][d] ^= gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, sl[u][d].s0, sl[u][d].s1, sl[u][d].s2);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < R; j++) {
            if (j >= nrows) break;
            const int mi = hdr->miss[a.row0 + j];
            uint8_t* ob = a.out[mi] + uint64_t(stripe) * a.out_stride[mi];
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (!live[u]) continue;
                store16<true>(ob + offs[u], acc[u][j]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Byte kernel: tails and unaligned layouts.  One thread per (stripe, byte) in
// [a.byte_begin, a.cell_len); LDS log/antilog lookups.
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

struct KernelInfo {
    const void* fn = nullptr;
    int blocks_per_cu = 0;
};

template <int K, int R, int U, bool NT, int BS, int MAP>
const void* vec_fn() {
    return reinterpret_cast<const void*>(&gf_matmul_v16<K, R, U, NT, BS, MAP>);
}

template <int R, int U, bool NT, int BS, int MAP>
const void* pick_k(int k) {
    switch (k) {
        case 2: return vec_fn<2, R, U, NT, BS, MAP>();
        case 3: return vec_fn<3, R, U, NT, BS, MAP>();
        case 6: return vec_fn<6, R, U, NT, BS, MAP>();
        case 10: return vec_fn<10, R, U, NT, BS, MAP>();
        default: return vec_fn<0, R, U, NT, BS, MAP>();
    }
}

template <int U, bool NT, int BS, int MAP = 0>
const void* pick_r(int k, int r) {
    switch (r) {
        case 1: return pick_k<1, U, NT, BS, MAP>(k);
        case 2: return pick_k<2, U, NT, BS, MAP>(k);
        case 3: return pick_k<3, U, NT, BS, MAP>(k);
        default: return pick_k<4, U, NT, BS, MAP>(k);
    }
}

// Shapes compiled: (chunks per lane U, block size BS) in
// {(1,256),(2,256),(4,256),(1,512),(2,512)}, each with and without
// non-temporal access.
template <bool NT>
const void* pick_shape(int k, int r, int unroll, int bs, int map) {
    if (bs == 512) return unroll >= 2 ? pick_r<2, NT, 512>(k, r) : pick_r<1, NT, 512>(k, r);
    if (unroll == 4) return map ? pick_r<4, NT, 256, 1>(k, r) : pick_r<4, NT, 256>(k, r);
    if (unroll == 2) return pick_r<2, NT, 256>(k, r);
    return pick_r<1, NT, 256>(k, r);
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

// LDS-DMA pipelined kernel: (U, BS) in {(4,256), (2,256), (2,512)} for k <= 6;
// k = 10 only at (2,256) (10 x 2 x 4 waves x 1 KiB = 80 KiB of LDS).
const void* pick_dma(int k, int r, int unroll, int bs) {
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
}

// Register double-buffered kernel: K in {2,3,6} at U in {1,2,3} (256
// threads) and K = 10 at U in {1,2}.
template <int K, int U>
const void* pipe_pick_r(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, 1, U, 256>);
        case 2: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, 2, U, 256>);
        case 3: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, 3, U, 256>);
        default: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, 4, U, 256>);
    }
}

template <int U>
const void* pipe_pick_k(int k, int r) {
    switch (k) {
        case 2: return pipe_pick_r<2, U>(r);
        case 3: return pipe_pick_r<3, U>(r);
        case 6: return pipe_pick_r<6, U>(r);
        default: return nullptr;
    }
}

template <int K, int R, int U>
const void* pipe_pol(int pol) {
    switch (pol) {
        case 1: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, R, U, 256, 1>);
        case 2: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, R, U, 256, 2>);
        case 3: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, R, U, 256, 3>);
        default: return reinterpret_cast<const void*>(&gf_matmul_pipe<K, R, U, 256, 4>);
    }
}

// Output-burst kernel: K in {2,3,6}, R * T <= 9 (T x R x 16 KiB of LDS).
template <int T>
const void* burst_pick(int k, int r) {
    auto f = [](auto kk, auto rr) { return reinterpret_cast<const void*>(&gf_matmul_burst<kk.value, rr.value, T>); };
    using std::integral_constant;
    if (r > 9 / T) return nullptr;
    switch (k) {
        case 2: return r == 1 ? f(integral_constant<int, 2>{}, integral_constant<int, 1>{})
                     : r == 2 ? f(integral_constant<int, 2>{}, integral_constant<int, 2>{})
                              : f(integral_constant<int, 2>{}, integral_constant<int, (9 / T >= 3 ? 3 : 2)>{});
        case 3: return r == 1 ? f(integral_constant<int, 3>{}, integral_constant<int, 1>{})
                     : r == 2 ? f(integral_constant<int, 3>{}, integral_constant<int, 2>{})
                              : f(integral_constant<int, 3>{}, integral_constant<int, (9 / T >= 3 ? 3 : 2)>{});
        case 6: return r == 1 ? f(integral_constant<int, 6>{}, integral_constant<int, 1>{})
                     : r == 2 ? f(integral_constant<int, 6>{}, integral_constant<int, 2>{})
                              : f(integral_constant<int, 6>{}, integral_constant<int, (9 / T >= 3 ? 3 : 2)>{});
        default: return nullptr;
    }
}

const void* pick_pipe(int k, int r, int unroll) {
    // store-policy variants only at the bench shapes (RS(6,3), RS(10,4))
    if (g_tune_store_pol > 0 && unroll <= 2 && ((k == 6 && r == 3) || (k == 10 && r == 4))) {
        if (k == 6) return unroll == 2 ? pipe_pol<6, 3, 2>(g_tune_store_pol) : pipe_pol<6, 3, 1>(g_tune_store_pol);
        return unroll == 2 ? pipe_pol<10, 4, 2>(g_tune_store_pol) : pipe_pol<10, 4, 1>(g_tune_store_pol);
    }
    if (k == 10) return unroll >= 2 ? pipe_pick_r<10, 2>(r) : pipe_pick_r<10, 1>(r);
    if (unroll >= 3) return pipe_pick_k<3>(k, r);
    if (unroll == 2) return pipe_pick_k<2>(k, r);
    return pipe_pick_k<1>(k, r);
}

int g_num_cus[64] = {0};

int num_cus(int dev) {
    if (dev < 0 || dev >= 64) return 256;
    if (!g_num_cus[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        g_num_cus[dev] = v;
    }
    return g_num_cus[dev];
}

}  // namespace

int g_tune_unroll = 0;         // 0 = per-shape default
int g_tune_nt = -1;            // -1 = default (non-temporal on)
int g_tune_blocks_per_cu = 0;  // 0 = per-shape default
int g_tune_block = 0;          // 0 = per-shape default
int g_tune_pipeline = 0;       // 0 = per-shape default, 1 = register kernel, 2 = LDS-DMA kernel
int g_tune_map = 0;            // 0 = default, 1 = MAP 0, 2 = MAP 1
int g_tune_grid = 0;           // 0 = blocks_per_cu * CUs, else absolute block count
int g_tune_group = 0;          // 0 = default (1), else stripes per tile-order group
int g_tune_crc_unfused = 0;    // 1 = hec_encode_crc_device as two passes
int g_tune_crc_variant = 0;    // 0 = default, 1 = slice-by-8 CRC, 2/3 = bank-replicated slice-by-1, 4/8 chains
int g_tune_xcd_remap = 0;           // 1 = XCD-contiguous block -> tile mapping
int g_tune_burst_tiles = 0;         // output-burst kernel: column tiles per burst (2 or 3)
int g_tune_host_copy_threads = 0;  // 0 = default (4)
int g_tune_store_pol = 0;      // 0 = nt stores, else store16p policy (register double-buffered kernel)
int g_tune_crc_prefetch = 0;   // 0 = default (2), else tasks of register prefetch per wave (1 or 2)
int g_tune_fused_slabs = 0;    // 0 = default, 4 / 8 = slabs per wave of the fused encode+CRC

namespace {

// Launch shape chosen from the MI355X sweeps in DESIGN.md ("Tuning"): long
// per-wave runs (4 x 1 KiB per stream) at one 256-thread block per CU keep
// the fewest DRAM rows open for a given bytes-in-flight.
struct Shape {
    int unroll, block, blocks_per_cu;
    bool nt;
    bool dma;
    int map;  // chunk_col mapping (U=4, 256 threads only)
    bool rpipe = false;  // register double-buffered kernel
};

Shape default_shape(int k, uint64_t cell_len) {
    // RS(10,4): 20 x 1 KiB loads in flight per wave already.  One 512-thread
    // block is resident per CU; a grid of 8 per CU (8 rounds) beats 2 by 3 %
    // at 256-512 stripes and ties at 2048 (profiles/r01f_probe_bpc_k10_*.log)
    if (k > 6) return {2, 512, 8, true, false, 0};
    // RS(3,2), RS(6,3): one wave per SIMD, 4 x 1 KiB per stream per wave.
    // Small cells (many short stripes) gain 2-3 % from the LDS-DMA prefetch;
    // 1 MiB cells lose ~5 % with it (profiles/r01_probe_dma_pipeline.log).
    // The LDS-DMA kernel (one block resident per CU) runs a grid of 2 per CU:
    // +3.3 % at 64 KiB x 16384 stripes, +1 % at x 65536, against 1 per CU
    // (profiles/r01f_probe_grid_64k_*.log); the register kernel keeps exactly
    // the resident blocks (2 per CU: -9 % at 1 MiB).
    const bool small = cell_len <= (256u << 10);
    const bool dma = small && (k == 2 || k == 3 || k == 6);
    return {4, 256, dma ? 2 : 1, true, dma, 0};
}

}  // namespace

int launch_gf_matmul(const MatmulArgs& in, int device, hipStream_t stream) {
    MatmulArgs a = in;
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
        if (g_tune_unroll) sh.unroll = g_tune_unroll;
        if (g_tune_block) sh.block = g_tune_block;
        if (g_tune_nt >= 0) sh.nt = g_tune_nt != 0;
        if (g_tune_blocks_per_cu) sh.blocks_per_cu = g_tune_blocks_per_cu;
        if (g_tune_pipeline) {
            sh.dma = g_tune_pipeline == 2;
            sh.rpipe = g_tune_pipeline == 3;
        }
        if (g_tune_map) sh.map = g_tune_map - 1;
        if (g_tune_grid) sh.blocks_per_cu = 0;
        if (sh.block == 512 && sh.unroll > 2) sh.unroll = 2;
        const bool dma_ok = (a.k == 2 || a.k == 3 || a.k == 6 || a.k == 10);
        if (sh.dma && !dma_ok) sh.dma = false;
        if (sh.rpipe && !dma_ok) sh.rpipe = false;
        // output-burst kernel (tune key 5 = 4, key 15 = T in {2, 3}): U = 4, 256 threads
        const int burst_t = g_tune_pipeline == 4 ? (g_tune_burst_tiles == 3 ? 3 : 2) : 0;
        const void* burst_fn = burst_t == 3 ? burst_pick<3>(a.k, a.r) : burst_t == 2 ? burst_pick<2>(a.k, a.r) : nullptr;
        if (burst_fn) {
            sh.dma = sh.rpipe = false;
            sh.unroll = 4;
            sh.block = 256;
        }
        if (sh.rpipe) {
            sh.dma = false;
            sh.block = 256;
            sh.unroll = std::min(sh.unroll, a.k == 10 ? 2 : 3);
        }
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
        const uint64_t tile = uint64_t(sh.block) * sh.unroll * (burst_fn ? burst_t : 1);  // burst: super-tiles
        const uint64_t tps = (chunks + tile - 1) / tile;
        const uint64_t total = tps * a.stripes;
        if (chunks > 0xFFFFFFFFull || total > 0xFFFFFFFFull) return -1;
        if (sh.rpipe && total > 0xFFF00000ull) return -1;  // tile + 3 * grid stays in 32 bits
        a.chunks = uint32_t(chunks);
        a.tiles_per_stripe = uint32_t(tps);
        a.total_tiles = uint32_t(total);
        // 4 stripes column-interleaved: +1-4 % over stripe-major at 1 MiB
        // cells (profiles/r01_probe_tile_order.log)
        a.group = g_tune_group > 0 ? uint32_t(g_tune_group) : 4u;
        const void* fn = burst_fn ? burst_fn
                         : sh.rpipe ? pick_pipe(a.k, a.r, sh.unroll)
                         : sh.dma ? pick_dma(a.k, a.r, sh.unroll, sh.block)
                                  : (sh.nt ? pick_shape<true>(a.k, a.r, sh.unroll, sh.block, sh.map)
                                           : pick_shape<false>(a.k, a.r, sh.unroll, sh.block, sh.map));
        uint64_t grid = g_tune_grid ? uint64_t(g_tune_grid) : uint64_t(cus) * sh.blocks_per_cu;
        if (grid > total) grid = total;
        a.xcd_remap = (g_tune_xcd_remap && grid % 8 == 0) ? 1u : 0u;
        void* args[] = {&a};
        const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(sh.block), args, 0, stream);
        if (e != hipSuccess) return int(e);
    }
    const uint64_t begin = chunks * 16;
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

template <int K, int R, bool RES>
const void* mixed_fn() {
    if constexpr (K > 6)
        return reinterpret_cast<const void*>(&gf_decode_mixed<K, R, 2, 512, RES>);
    else
        return reinterpret_cast<const void*>(&gf_decode_mixed<K, R, 4, 256, RES>);
}

template <int K>
const void* mixed_pick_r(int r, bool res) {
    switch (r) {
        case 1: return res ? mixed_fn<K, 1, true>() : mixed_fn<K, 1, false>();
        case 2: return res ? mixed_fn<K, 2, true>() : mixed_fn<K, 2, false>();
        case 3: return res ? mixed_fn<K, 3, true>() : mixed_fn<K, 3, false>();
        default: return res ? mixed_fn<K, 4, true>() : mixed_fn<K, 4, false>();
    }
}

constexpr uint32_t kResidentBlobMax = 64u << 10;  // LDS budget for resident plans

}  // namespace

int launch_decode_mixed(const MixedArgs& in, int rows, int device, hipStream_t stream) {
    MixedArgs a = in;
    if (a.cell_len % 16 != 0 || a.cell_len / 16 > 0xFFFFFFFFull) return -1;
    const bool res = a.blob_bytes <= kResidentBlobMax && a.blob_bytes % 4 == 0;
    const void* fn = nullptr;
    switch (a.k) {
        case 2: fn = mixed_pick_r<2>(rows, res); break;
        case 3: fn = mixed_pick_r<3>(rows, res); break;
        case 6: fn = mixed_pick_r<6>(rows, res); break;
        case 10: fn = mixed_pick_r<10>(rows, res); break;
        default: return -1;
    }
    const int U = a.k > 6 ? 2 : 4, BS = a.k > 6 ? 512 : 256;
    // K > 6: a grid of 8 per CU (one resident): RS(10,4) mixed decode 3216-3234
    // -> 3524-3621 GiB/s against 2 per CU
    const int bpc = g_tune_blocks_per_cu ? g_tune_blocks_per_cu : (a.k > 6 ? 8 : 1);
    const uint64_t chunks = a.cell_len / 16;
    const uint64_t tile = uint64_t(BS) * U;
    const uint64_t tps = (chunks + tile - 1) / tile;
    const uint64_t total = tps * a.stripes;
    if (total > 0xFFFFFFFFull) return -1;
    if (total == 0) return 0;
    a.chunks = uint32_t(chunks);
    a.tiles_per_stripe = uint32_t(tps);
    a.total_tiles = uint32_t(total);
    a.group = g_tune_group > 0 ? uint32_t(g_tune_group) : 4u;
    uint64_t grid = uint64_t(num_cus(device)) * bpc;
    if (grid > total) grid = total;
    void* args[] = {&a};
    const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(BS), args, res ? a.blob_bytes : 0, stream);
    return e == hipSuccess ? 0 : int(e);
}

}  // namespace hec
