// ec_experimental.hip -- kernel variants that were measured on MI355X and
// rejected, kept buildable for re-measurement.  Compiled only into the
// HEC_EXPERIMENTAL library (make exp -> lib/libhdfs_ec_amd_exp.so) and
// selected with tune key 5 (3 = register pipe, 4 = output bursts, 5 =
// register double buffering); the default library never contains them.
// Results (same-box A/B logs under profiles/):
//  * pipe: -1 % RS(6,3), -5 % RS(10,4) (r01d_probe_pipe_*.log)
//  * output bursts: -3 % .. -30 % (r01e_probe_burst_*.log)
//  * store cache policies of the pipe kernel: no gain (r01d_probe_pipe_k6.log)
//  * double buffering with both register sets drain-free: -7 % RS(6,3),
//    -10 % RS(10,4) at 256 stripes (r02_probe_db_*.log)
#ifndef HEC_EXPERIMENTAL
#error "ec_experimental.hip is built only with -DHEC_EXPERIMENTAL"
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "ec_kernels.hpp"
#include "gf_device.hpp"

namespace hec {

namespace {
// Store cache policy (measurement knob, tune key 13): 0 = nt (default),
// 1 = sc1, 2 = sc0 sc1, 3 = nt sc1, 4 = plain.  nt / plain keep the written
// line in the XCD's L2 until it is evicted; sc1 drops it (MI355X_MICROARCH
// "stores of each flavour").  The asm forms are invisible to the waitcnt
// pass: later compiler waits on loads only over-wait (older stores retire
// first), and the s_nop covers the >8-byte store-data VALU-write hazard.
template <int POL>
__device__ __forceinline__ void store16p(uint8_t* p, u32x4 v) {
    if constexpr (POL == 0)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else if constexpr (POL == 4)
        *reinterpret_cast<u32x4*>(p) = v;
    else if constexpr (POL == 1)
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2)
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}


}  // namespace

// ---------------------------------------------------------------------------
// Register double-buffered kernel (compile-time K).  Two register sets of
// K x U chunks alternate: tile t+grid's loads are issued before tile t is
// computed, so a wave keeps a whole tile of loads in flight through its GF
// math and its stores (tile time ~ max(latency, math) instead of their sum).
// Two accumulator sets as well: the accumulators written by a tile's math
// are the store data of the tile two half-steps back, long retired, so the
// waitcnt pass never drains in-flight stores to protect their data VGPRs.
// ---------------------------------------------------------------------------
template <int K, int U, int BS>
__device__ __forceinline__ void db_load(const MatmulArgs& a, uint32_t tile, u32x4 (&x)[U][K], uint32_t& stripe,
                                        uint32_t& tcol) {
    tile_coords(tile, a, stripe, tcol);
    const uint32_t chunks = a.chunks;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t col = tcol * (BS * U) + u * BS + threadIdx.x;
        const uint32_t off = (col < chunks ? col : 0u) * 16u;  // dead lanes read chunk 0, never stored
#pragma unroll
        for (int i = 0; i < K; i++) x[u][i] = load16<true>((a.in[i] + uint64_t(stripe) * a.in_stride[i]) + off);
    }
}

template <int K, int R, int U>
__device__ __forceinline__ void db_compute(const u32x4 (&x)[U][K], const PermTable (*s_tab)[kMaxK],
                                           u32x4 (&acc)[U][R]) {
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
        Sel s[U][4];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int d = 0; d < 4; d++) s[u][d] = make_sel(x[u][i][d]);
#pragma unroll
        for (int j = 0; j < R; j++) {
            const PermTable& t = *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
            const uint32_t t0lo = t.t0lo, t0hi = t.t0hi, t1lo = t.t1lo, t1hi = t.t1hi, t2 = t.t2;
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    const uint32_t p = gf_mul4(t0lo, t0hi, t1lo, t1hi, t2, s[u][d].s0, s[u][d].s1, s[u][d].s2);
                    acc[u][j][d] = i == 0 ? p : (acc[u][j][d] ^ p);
                }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]));
}

template <int R, int U, int BS>
__device__ __forceinline__ void db_store(const MatmulArgs& a, uint32_t stripe, uint32_t tcol, const u32x4 (&acc)[U][R]) {
    const uint32_t chunks = a.chunks;
    if ((tcol + 1) * (BS * U) <= chunks) {  // block-uniform: the whole tile lies inside the cell
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++)
                store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + (tcol * (BS * U) + u * BS + threadIdx.x) * 16u,
                              acc[u][j]);
    } else {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t col = tcol * (BS * U) + u * BS + threadIdx.x;
            if (col >= chunks) continue;
#pragma unroll
            for (int j = 0; j < R; j++) store16<true>((a.out[j] + uint64_t(stripe) * a.out_stride[j]) + col * 16u, acc[u][j]);
        }
    }
}

template <int K, int R, int U, int BS>
__global__ __launch_bounds__(BS) void gf_matmul_db(MatmulArgs a) {
    static_assert(K > 0, "double-buffered kernel needs a compile-time input count");
    __shared__ PermTable s_tab[R][kMaxK];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    prologue<R, BS>(a, K, s_tab, s_exp, s_log, s_coef);
    const uint32_t total = a.total_tiles, step = gridDim.x;
    uint32_t tile = blockIdx.x;
    if (tile >= total) return;
    u32x4 xa[U][K], xb[U][K], acca[U][R], accb[U][R];
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
        for (int j = 0; j < R; j++) accb[u][j] = u32x4{0, 0, 0, 0};
    uint32_t sa, ca, sb = 0, cb = 0;
    db_load<K, U, BS>(a, tile, xa, sa, ca);
    for (;;) {
        // unconditional loads (a branch around them would make the waitcnt
        // pass count them as absent and wait for the prefetch too); past the
        // end the block re-reads its current tile and stores nothing from it
        const bool more_b = tile + step < total;  // block-uniform
        db_load<K, U, BS>(a, more_b ? tile + step : tile, xb, sb, cb);
        // the other set's accumulators (store data of the previous half) stay
        // allocated through the loads' address math: no temporary lands in a
        // register an in-flight store still reads
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" ::"v"(accb[u][j]));
        __builtin_amdgcn_sched_barrier(0);
        db_compute<K, R, U>(xa, s_tab, acca);
        db_store<R, U, BS>(a, sa, ca, acca);
        __builtin_amdgcn_sched_barrier(0);
        if (!more_b) break;
        const bool more_a = tile + 2 * step < total;
        db_load<K, U, BS>(a, more_a ? tile + 2 * step : tile + step, xa, sa, ca);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int j = 0; j < R; j++) asm volatile("" ::"v"(acca[u][j]));
        __builtin_amdgcn_sched_barrier(0);
        db_compute<K, R, U>(xb, s_tab, accb);
        db_store<R, U, BS>(a, sb, cb, accb);
        __builtin_amdgcn_sched_barrier(0);
        if (!more_a) break;
        tile += 2 * step;
    }
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


namespace {

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

template <int K, int U, int BS>
const void* db_pick_r(int r) {
    switch (r) {
        case 1: return reinterpret_cast<const void*>(&gf_matmul_db<K, 1, U, BS>);
        case 2: return reinterpret_cast<const void*>(&gf_matmul_db<K, 2, U, BS>);
        case 3: return reinterpret_cast<const void*>(&gf_matmul_db<K, 3, U, BS>);
        default: return reinterpret_cast<const void*>(&gf_matmul_db<K, 4, U, BS>);
    }
}

// Double-buffered register kernel: K in {2,3,6} at (U, BS) in {(4,256),
// (2,256)}; K = 10 at (2,256) and (1,512).  nullptr: shape not compiled.
const void* pick_db(int k, int r, int unroll, int bs) {
    switch (k) {
        case 2: return unroll >= 4 ? db_pick_r<2, 4, 256>(r) : db_pick_r<2, 2, 256>(r);
        case 3: return unroll >= 4 ? db_pick_r<3, 4, 256>(r) : db_pick_r<3, 2, 256>(r);
        case 6: return unroll >= 4 ? db_pick_r<6, 4, 256>(r) : db_pick_r<6, 2, 256>(r);
        case 10: return bs == 512 ? db_pick_r<10, 1, 512>(r) : db_pick_r<10, 2, 256>(r);
        default: return nullptr;
    }
}

const void* pick_pipe(int k, int r, int unroll, int store_pol) {
    // store-policy variants only at the bench shapes (RS(6,3), RS(10,4))
    if (store_pol > 0 && unroll <= 2 && ((k == 6 && r == 3) || (k == 10 && r == 4))) {
        if (k == 6) return unroll == 2 ? pipe_pol<6, 3, 2>(store_pol) : pipe_pol<6, 3, 1>(store_pol);
        return unroll == 2 ? pipe_pol<10, 4, 2>(store_pol) : pipe_pol<10, 4, 1>(store_pol);
    }
    if (k == 10) return unroll >= 2 ? pipe_pick_r<10, 2>(r) : pipe_pick_r<10, 1>(r);
    if (unroll >= 3) return pipe_pick_k<3>(k, r);
    if (unroll == 2) return pipe_pick_k<2>(k, r);
    return pipe_pick_k<1>(k, r);
}
}  // namespace

bool experimental_matmul(const Tune& t, int k, int r, ExpKernel* out) {
    if (!(k == 2 || k == 3 || k == 6 || k == 10)) return false;
    ExpKernel e{nullptr, t.unroll ? t.unroll : 4, 256, 1, 1};
    if (t.pipeline == 3) {  // register pipe (double-buffered, drains before stores)
        e.unroll = std::min(e.unroll, k == 10 ? 2 : 3);
        e.fn = pick_pipe(k, r, e.unroll, t.store_pol);
    } else if (t.pipeline == 4) {  // output bursts of T column tiles
        const int T = t.burst_tiles == 3 ? 3 : 2;
        e.unroll = 4;
        e.tile_mult = T;
        e.fn = T == 3 ? burst_pick<3>(k, r) : burst_pick<2>(k, r);
    } else if (t.pipeline == 5) {  // drain-free register double buffering
        if (k == 10) {
            e.block = t.block == 512 ? 512 : 256;
            e.unroll = e.block == 512 ? 1 : 2;
        } else {
            e.unroll = e.unroll >= 4 ? 4 : 2;
        }
        e.blocks_per_cu = e.block == 512 ? 2 : 1;
        e.fn = pick_db(k, r, e.unroll, e.block);
    }
    if (!e.fn) return false;
    *out = e;
    return true;
}

}  // namespace hec
