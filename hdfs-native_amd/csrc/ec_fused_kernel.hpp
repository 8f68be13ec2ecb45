// ec_fused_kernel.hpp -- the fused stripe multiply + chunk checksum kernel
// template, shared by the ahead-of-time build (ec_fused.hip)
// and the plan-time JIT (jit.cpp: decode + verify with the decode plan's own
// bit-sliced XOR network, compiled by hiprtc from this header).  See
// ec_fused.hip for the design and the launcher.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>

#include <cstdint>
#endif

#include "bitslice.hpp"
#include "checksum.hpp"
#include "checksum_device.hpp"
#include "checksum_tables.hpp"
#include "ec_kernels.hpp"
#include "gf_device.hpp"
#include "xor_networks.hpp"

namespace hec {

// Parity math of the fused kernel: PermNet = the v_perm product tables of
// the launch's coefficient rows (any matrix, read from the kernel
// arguments); a network type (kBsl = true) = bit-sliced XOR networks,
// absorb_at(i, planes, acc) folding input i's 8 bit planes into the R * 8
// accumulator planes (input 0 initialises them).  RsNet = the RS coding
// matrix's parity rows (xor_networks.hpp); jit.cpp generates one per decode
// plan.
struct PermNet {
    static constexpr bool kBsl = false;
};

template <int K, int R>
struct RsNet {
    static constexpr bool kBsl = true;
    __device__ __forceinline__ static void absorb_at(int i, const uint32_t (&p)[8], uint32_t (&acc)[R * 8]) {
        bitslice::rs_absorb_at<K, R>(i, p, acc);
    }
};

namespace {  // per translation unit (each code object has its own tables)
__constant__ crc::Tables<crc::kCrc32c> kFusedCrc32c = crc::Tables<crc::kCrc32c>();
__constant__ crc::Tables<crc::kCksum> kFusedCksum = crc::Tables<crc::kCksum>();

template <int KIND>
__device__ __forceinline__ const crc::Tables<KIND>& fused_tables() {
    if constexpr (KIND == crc::kCrc32c)
        return kFusedCrc32c;
    else
        return kFusedCksum;
}

// scheme 15's slicing-by-32 tables (32 KiB), emitted only where a scheme-15
// kernel is instantiated
template <int KIND>
__device__ __forceinline__ const uint32_t* fused_slice32() {
    static constexpr crc::Slice32<KIND> kT{};
    return &kT.t[0][0];
}
}  // namespace

// Layout: a wave owns SLABS KiB (SLABS slabs of 1 KiB, one 16-B load per
// lane per slab) of every cell of its stripe; one checksum round is 64
// quarters = 8 pieces = 8/SLABS shards' share, over a 9-KiB image (as in
// checksum.hip).  Inputs stream shard by shard (the next one prefetched
// into registers when the budget allows) while being accumulated into the
// r output registers and staged for the round; then (encode) each parity
// shard is stored and staged, or (VERIFY) each rebuilt cell is only stored.
// SLABS = 8 (one shard per round) when the r x 8 accumulators fit 2 waves
// per SIMD, else 4 (two shards per round; an odd shard count leaves one
// half-empty round).  9 KiB of image per wave -> 8 waves per CU.
//   encode (VERIFY = false): checksummed shards 0..K+R-1 = inputs then
//     outputs; sums[(stripe * n_total + shard_id[s]) * nck + chunk].
//   VERIFY: checksummed shards 0..K-1 = the survivors; their expected sums
//     sit at the same index (shard_id = survivor shard numbers), a mismatch
//     sets bad[stripe * n_total + shard_id[s]].
// BSL (encode with the RS coding matrix, K in {3, 6, 10}): the parity is
// computed bit-sliced -- each input's 8-dword groups transposed into bit
// planes (bitslice.hpp) and folded into the accumulator planes by the
// generated XOR network of the RS parity rows (xor_networks.hpp), the planes
// transposed back at the end -- instead of through the v_perm product
// tables: RS(6,3) 650 instead of 960 VALU per 8 dwords of every shard,
// RS(10,4) 1155 instead of 2000.  The kernel is VALU-issue bound.
// WQ: tiles are wave-tiles (SLABS KiB of one stripe's cells per wave) from
// the work queue (gf_device.hpp WaveQueue, a.queue) instead of block tiles in
// a fixed order.
template <int K, int R, int SLABS, int SCHEME, int KIND, bool VERIFY, int WPE = 2, bool PAIR = false,
          class NET = PermNet, int PFD = 1, bool WQ = false>
__global__ __launch_bounds__(crcdev::sliced(SCHEME) ? 128 * WPE * (WPE - 1) : 512)
    __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void gf_fused_crc(
    MatmulArgs a, FusedCrcArgs cs) {
    constexpr bool BSL = NET::kBsl;
    static_assert(!BSL || SLABS % 2 == 0, "bit-sliced parity: 8-dword groups");
    using TL = crcdev::TableLayout<SCHEME>;
    using Spec = crc::Spec<KIND>;
    constexpr bool REFL = Spec::kReflected;
    // sliced schemes: WPE = 2 -> 256-thread blocks, two per CU; WPE = 3 ->
    // one 768-thread block per CU (12 waves, 3 per SIMD)
    constexpr int BS = crcdev::sliced(SCHEME) ? 128 * WPE * (WPE - 1) : 512, WAVES = BS / 64;
    constexpr int PITCH = 144, STAGE = 64 * PITCH, SPR = 8 / SLABS;
    constexpr int NSUM = VERIFY ? K : K + R;  // checksummed shards
    // VERIFY with PFD = 4: the tile's expected chunk sums (CPS per survivor
    // per wave) are loaded with its first input, NWANT per lane, and each CRC
    // round takes its own from them by a lane shuffle instead of a global load
    // whose latency the round would wait for
    constexpr bool WANT_PF = VERIFY && PFD == 4;
    // VERIFY with PFD = 5 (default shapes: inputs one at a time, or in pairs
    // with one pair ahead): the rebuilt rows are stored, and the next tile's
    // first inputs loaded, BEFORE the last input's CRC round, which then
    // covers their latency; otherwise the next tile's first loads queue
    // behind this tile's stores (vmcnt retires in order) with nothing to do
    constexpr bool EARLY_OUT = VERIFY && PFD == 5;
    constexpr int CPS = SLABS * 2, NWANT = WANT_PF ? (NSUM * CPS + 63) / 64 : 1;
    constexpr uint32_t WAVE_BYTES = SLABS * 1024u, TILE_BYTES = WQ ? WAVE_BYTES : WAVES * WAVE_BYTES;
    constexpr bool PF = R * SLABS <= 24;  // register prefetch of the next shard
    __shared__ PermTable s_tab[R][K];  // K columns: scheme 11 needs 2 x 79 KiB per CU
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    __shared__ uint32_t s_ctabs[TL::kWords];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[WAVES * STAGE];
    prologue<R, BS, K>(a, K, s_tab, s_exp, s_log, s_coef);
    crcdev::stage_tables<SCHEME, BS>(s_ctabs, fused_tables<KIND>());
    if constexpr (SCHEME == 15) {
        static_assert(KIND == crc::kCrc32c, "scheme 15 folds the reflected register");
        const uint32_t* t32 = fused_slice32<KIND>();
        for (int t = threadIdx.x; t < 32 * 256; t += BS) s_ctabs[t] = t32[t];
    }
    __syncthreads();
    const uint32_t kfinal = fused_tables<KIND>().final512;

    const uint64_t cell_len = a.cell_len;
    const uint64_t nck = (cell_len + 511) / 512;  // checksum chunks per cell
    const uint32_t total = a.total_tiles;
    // wave index as a scalar: the wave's byte offset, the shard bases and the
    // stage pointer then stay in SGPRs (saddr + 32-bit lane offset loads and
    // stores, no per-access 64-bit VALU address)
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x / 64)), lane = threadIdx.x & 63;
    // this lane's quarter in a round: row `lane` = piece lane/8 = (shard
    // slot sir, slab), chunk half (lane/4)&1 of that slab, quarter qi
    const int qi = lane & 3, piece = lane >> 3, sir = piece / SLABS, pslab = piece % SLABS, half = (lane >> 2) & 1;
    uint8_t* stage = s_stage + wave * STAGE;
    uint32_t* out_sums = reinterpret_cast<uint32_t*>(cs.sums);
    const uint32_t* exp_sums = reinterpret_cast<const uint32_t*>(cs.expected);

    // tile -> (stripe, column), with the columns of stripe s rotated by
    // s * col_rot (measurement: concurrent stripes of a tile-order group then
    // sit at different offsets of their cells)
    auto coords = [&](uint32_t t, uint32_t& stripe, uint32_t& tcol) {
        tile_coords(t, a, stripe, tcol);
        if (a.col_rot) {
            tcol += (stripe * a.col_rot) % a.tiles_per_stripe;
            if (tcol >= a.tiles_per_stripe) tcol -= a.tiles_per_stripe;
        }
    };
    // PFD = 3: x already holds this tile's input 0 (loaded during the
    // previous tile's outputs)
    bool have_next = false;
    u32x4 x[SLABS], xn[SLABS];
    WaveQueue wq;
    if constexpr (WQ) {
        queue_zero_next(a.queue_zero);
        wq.init(a.queue, total);
    }
    // the wave's byte offset inside a block tile (WQ: a wave-tile is the wave's own)
    const uint32_t wave_off = WQ ? 0u : uint32_t(wave) * WAVE_BYTES;
    for (uint32_t tile = WQ ? wq.next() : blockIdx.x; tile < total; tile = WQ ? wq.next() : tile + gridDim.x) {
        uint32_t stripe, tcol;
        coords(tile, stripe, tcol);
        const uint64_t wbyte = uint64_t(tcol) * TILE_BYTES + wave_off;  // wave's first byte
        if (wbyte >= cell_len) continue;  // wave-uniform (never a prefetched tile: those are full)
        // 32-bit lane offsets from a wave-uniform per-shard base (saddr +
        // voffset addressing); dead slabs of a short last tile read slab 0
        // (compared in 32 bits: a 64-bit compare shares the offsets' zero
        // extension with the address adds, which then lose the saddr form
        // and hold every offset as a 64-bit VGPR pair)
        const uint64_t left = cell_len - wbyte;
        const uint32_t left32 = left > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(left);
        uint32_t voff[SLABS];
        bool live[SLABS];
#pragma unroll
        for (int u = 0; u < SLABS; u++) {
            const uint32_t o = uint32_t(u) * 1024u + uint32_t(lane) * 16u;
            live[u] = o < left32;
            voff[u] = live[u] ? o : 0u;
        }
        const uint64_t cbyte = wbyte + uint64_t(pslab) * 1024u + uint64_t(half) * 512u;
        const bool in_cell = cbyte < cell_len;
        const bool full = in_cell && cell_len - cbyte >= 512u;  // same for a chunk's 4 lanes

        uint32_t wreg[NWANT];  // WANT_PF: the tile's expected sums (filled with input 0's loads)
        // `first` is a compile-time constant at every (unrolled) call site,
        // so the shard ids are scalar kernarg reads
        auto sum_cell = [&](int first) {
            if constexpr (!VERIFY) return uint64_t(stripe) * (K + R) + first + sir;  // encode: identity layout
            const uint32_t sid = (SPR > 1 && sir > 0 && first + 1 < NSUM) ? cs.shard_id[first + 1] : cs.shard_id[first];
            return uint64_t(stripe) * cs.n_total + sid;
        };
        auto crc_round = [&](int first, int count) {
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            const bool live_c = in_cell && sir < count;
            uint32_t want = 0;
            if constexpr (WANT_PF) {
                // from the tile's prefetched sums: entry (first + sir) * CPS + chunk
                const int f = (first + sir) * CPS + pslab * 2 + half;
#pragma unroll
                for (int h = 0; h < NWANT; h++) {
                    const uint32_t v = uint32_t(__shfl(int(wreg[h]), f & 63));
                    if ((f >> 6) == h) want = v;
                }
            } else if (VERIFY && live_c && qi == 0) {
                want = exp_sums[sum_cell(first) * nck + cbyte / 512];  // issued before the lookups
            }
            uint32_t val = 0;
            if (full && sir < count) {
                uint32_t r = crcdev::quarter<SCHEME, REFL>(s_ctabs, stage + lane * PITCH, lane);
                if (qi < 3) r = crcdev::shift_quarter<SCHEME>(s_ctabs, qi, r);
                val = r;
            } else if (live_c && qi == 0) {
                // short last chunk of the cell: this lane walks it whole, bytewise
                const uint32_t len = uint32_t(cell_len - cbyte);
                uint32_t r = Spec::kInit;
                for (uint32_t b = 0; b < len; b++)
                    r = crcdev::byte_step<REFL, crcdev::ByteTable<SCHEME>::stride, crcdev::ByteTable<SCHEME>::bswap>(
                        s_ctabs + crcdev::ByteTable<SCHEME>::off, r, stage[(lane + b / 128) * PITCH + (b % 128)]);
                val = r ^ Spec::kXorout;
            }
            val ^= __shfl_xor(val, 1);
            val ^= __shfl_xor(val, 2);
            if (live_c && qi == 0) {
                const uint32_t be = __builtin_bswap32(full ? (val ^ kfinal) : val);
                if constexpr (VERIFY) {
                    if (be != want) cs.bad[sum_cell(first)] = 1;
                } else {
                    if (cs.sums_nt)
                        __builtin_nontemporal_store(be, out_sums + sum_cell(first) * nck + cbyte / 512);
                    else
                        out_sums[sum_cell(first) * nck + cbyte / 512] = be;
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        };
        // slab u of the shard in round slot `slot`: lane l's 16 B -> row
        // 8*(slot*SLABS + u) + l/8, byte 16*(l%8)
        auto stage_piece = [&](int slot, int u, const u32x4& v) {
            *reinterpret_cast<u32x4*>(stage + (8 * (slot * SLABS + u) + lane / 8) * PITCH + 16 * (lane % 8)) = v;
        };
        // this lane's own 16 B of slab u in round slot `slot`, read back
        auto staged_piece = [&](int slot, int u) {
            return *reinterpret_cast<const u32x4*>(stage + (8 * (slot * SLABS + u) + lane / 8) * PITCH + 16 * (lane % 8));
        };
        auto after_stage = [&](int shard) {
            if (shard % SPR == SPR - 1 || shard == NSUM - 1) crc_round(shard - shard % SPR, shard % SPR + 1);
        };

        u32x4 acc[BSL ? 1 : SLABS][R];
        if constexpr (!BSL) {
#pragma unroll
            for (int u = 0; u < SLABS; u++)
#pragma unroll
                for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
        }
        // BSL: group g = slabs 2g, 2g+1 (8 dwords) as R*8 bit planes
        uint32_t accp[BSL ? SLABS / 2 : 1][BSL ? R * 8 : 1];
        // input i's share of the parity, bit-sliced (input 0 initialises accp);
        // fetch(g, lo, hi) yields group g's two slabs
        auto bsl_absorb_from = [&](int i, auto&& fetch) {
            if constexpr (BSL) {
#pragma unroll
                for (int g = 0; g < SLABS / 2; g++) {
                    u32x4 lo, hi;
                    fetch(g, lo, hi);
                    uint32_t pl[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    if (i > 0) {
                        // opaque per input: keeps the XOR chains of the
                        // accumulators from being reassociated across inputs
#pragma unroll
                        for (int t = 0; t < R * 8; t++) asm volatile("" : "+v"(accp[g][t]));
                    }
                    bitslice::transpose8(pl);
                    NET::absorb_at(i, pl, accp[g]);
                    // one group's planes and network temporaries live at a time
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
        auto bsl_absorb = [&](int i, const u32x4 (&xi)[SLABS]) {
            bsl_absorb_from(i, [&](int g, u32x4& lo, u32x4& hi) {
                lo = xi[2 * g];
                hi = xi[2 * g + 1];
            });
        };
        // parity row j's slabs back from the planes (the transpose is its own inverse)
        auto bsl_output = [&](int j, u32x4 (&o)[SLABS]) {
            if constexpr (BSL) {
#pragma unroll
                for (int g = 0; g < SLABS / 2; g++) {
                    uint32_t q[8];
#pragma unroll
                    for (int t = 0; t < 8; t++) q[t] = accp[g][8 * j + t];
                    bitslice::transpose8(q);
                    o[2 * g] = u32x4{q[0], q[1], q[2], q[3]};
                    o[2 * g + 1] = u32x4{q[4], q[5], q[6], q[7]};
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
        const bool pref = have_next;  // x (and xn with pairs, EARLY_OUT) hold this tile's first inputs
        if (!pref) {
#pragma unroll
            for (int u = 0; u < SLABS; u++)
                x[u] = load16<true>(a.in[0] + (uint64_t(stripe) * a.in_stride[0] + wbyte) + voff[u]);
        }
        have_next = false;
        if constexpr (WANT_PF) {
            const uint64_t c0 = wbyte / 512;
#pragma unroll
            for (int h = 0; h < NWANT; h++) {
                const int f = lane + 64 * h, s = f / CPS, c = f % CPS;
                uint32_t sid = 0;
#pragma unroll
                for (int t = 0; t < NSUM; t++) sid = s == t ? cs.shard_id[t] : sid;
                const bool ok = s < NSUM && wbyte + uint64_t(c) * 512u < cell_len;
                wreg[h] = ok ? exp_sums[(uint64_t(stripe) * cs.n_total + sid) * nck + c0 + uint64_t(c)] : 0u;
            }
        }
        auto load_in = [&](int i, u32x4 (&dst)[SLABS]) {
#pragma unroll
            for (int u = 0; u < SLABS; u++)
                dst[u] = load16<true>(a.in[i] + (uint64_t(stripe) * a.in_stride[i] + wbyte) + voff[u]);
        };
        // the next tile's input 0 (and 1: `two`) into x (xn) when that tile is
        // full for this wave (its lane offsets are then the constant ones)
        auto prefetch_next = [&](bool two) {
            const uint32_t nt = WQ ? wq.peek() : tile + gridDim.x;
            if (nt < total) {
                uint32_t ns, ncol;
                coords(nt, ns, ncol);
                const uint64_t nw = uint64_t(ncol) * TILE_BYTES + wave_off;
                if (nw + WAVE_BYTES <= cell_len) {  // wave-uniform
#pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        x[u] = load16<true>(a.in[0] + (uint64_t(ns) * a.in_stride[0] + nw) + uint32_t(u) * 1024u +
                                            uint32_t(lane) * 16u);
                    if (two) {
#pragma unroll
                        for (int u = 0; u < SLABS; u++)
                            xn[u] = load16<true>(a.in[1] + (uint64_t(ns) * a.in_stride[1] + nw) + uint32_t(u) * 1024u +
                                                 uint32_t(lane) * 16u);
                    }
                    have_next = true;
                }
            }
        };
        // the R output rows: stored (encode: and checksummed, one round each)
        auto emit_outputs = [&]() {
#pragma unroll
            for (int j = 0; j < R; j++) {
                u32x4 o[SLABS];
                if constexpr (BSL) {
                    bsl_output(j, o);
                } else {
#pragma unroll
                    for (int u = 0; u < SLABS; u++) o[u] = acc[u][j];
                }
#pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    if (live[u]) store16<true>(a.out[j] + (uint64_t(stripe) * a.out_stride[j] + wbyte) + voff[u], o[u]);
                    if constexpr (!VERIFY) stage_piece((K + j) % SPR, u, o[u]);
                }
                if constexpr (!VERIFY) after_stage(K + j);
            }
        };
        if constexpr (BSL && !PAIR && PFD == 3) {
            // Bit-sliced parity, one input at a time, loads issued a phase
            // earlier: input i is staged to LDS first, so its registers take
            // input i + 1's loads BEFORE the parity math, which reads input i
            // back from the stage (its own 16-B pieces: no barrier); the loads
            // are in flight across the network and the CRC round instead of
            // the CRC round only.  The next tile's input 0 is loaded during
            // this tile's outputs (when that tile is full for this wave, so its
            // lane offsets are the constant ones).
#pragma unroll
            for (int i = 0; i < K; i++) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < SLABS; u++) stage_piece(i % SPR, u, x[u]);
                __builtin_amdgcn_sched_barrier(0);
                if (i + 1 < K) load_in(i + 1, x);
                __builtin_amdgcn_sched_barrier(0);
                bsl_absorb_from(i, [&](int g, u32x4& lo, u32x4& hi) {
                    lo = staged_piece(i % SPR, 2 * g);
                    hi = staged_piece(i % SPR, 2 * g + 1);
                });
                __builtin_amdgcn_sched_barrier(0);
                after_stage(i);
                __builtin_amdgcn_sched_barrier(0);
            }
            prefetch_next(false);
        } else if constexpr (BSL && PAIR && SPR == 2 && PFD == 2) {
            // Bit-sliced parity, inputs two at a time, loads TWO pairs ahead:
            // pair p lives in buf[p & 1]; once its planes are absorbed the
            // buffer is refilled with pair p + 2 before the CRC round, so two
            // pairs' loads (16 KiB per wave at 4 slabs) are in flight across
            // it instead of one.  The smaller bit-sliced accumulators (4
            // slabs: R x 8 planes x 2 groups) leave the VGPRs for it.
            u32x4 buf[2][2][SLABS];
#pragma unroll
            for (int u = 0; u < SLABS; u++) buf[0][0][u] = x[u];
            if (K > 1) load_in(1, buf[0][1]);
            if (K > 2) load_in(2, buf[1][0]);
            if (K > 3) load_in(3, buf[1][1]);
#pragma unroll
            for (int i = 0; i < K; i += 2) {
                const bool two = i + 1 < K;
                auto& cur = buf[(i / 2) & 1];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    stage_piece(0, u, cur[0][u]);
                    if (two) stage_piece(1, u, cur[1][u]);
                }
                bsl_absorb(i, cur[0]);
                if (two) bsl_absorb(i + 1, cur[1]);
                __builtin_amdgcn_sched_barrier(0);
                if (i + 4 < K) load_in(i + 4, cur[0]);
                if (i + 5 < K) load_in(i + 5, cur[1]);
                __builtin_amdgcn_sched_barrier(0);
                after_stage(two ? i + 1 : i);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if constexpr (PAIR && SPR == 2 && PF) {
            // Inputs two at a time (one CRC round): both shards' products go
            // into the accumulators through one chain of 3-input XORs, 3 ops
            // per (dword, output) for the pair instead of 4.  The next pair's
            // loads are issued after this pair's GF math, before its round.
            if (K > 1 && !(EARLY_OUT && pref)) {
#pragma unroll
                for (int u = 0; u < SLABS; u++)
                    xn[u] = load16<true>(a.in[1] + (uint64_t(stripe) * a.in_stride[1] + wbyte) + voff[u]);
            }
#pragma unroll
            for (int i = 0; i < K; i += 2) {
                const bool two = i + 1 < K;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    stage_piece(0, u, x[u]);
                    if (two) stage_piece(1, u, xn[u]);
                }
                if constexpr (BSL) {
                    bsl_absorb(i, x);
                    if (two) bsl_absorb(i + 1, xn);
                } else {
                uint32_t toff = uint32_t(i) * uint32_t(sizeof(PermTable));
                asm volatile("" : "+v"(toff));
#pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    asm volatile("" : "+v"(x[u]), "+v"(xn[u]));
#pragma unroll
                    for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
                }
                uint32_t ta[R][5], tq[R][5];
#pragma unroll
                for (int j = 0; j < R; j++) {
                    const PermTable& t =
                        *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
                    ta[j][0] = t.t0lo;
                    ta[j][1] = t.t0hi;
                    ta[j][2] = t.t1lo;
                    ta[j][3] = t.t1hi;
                    ta[j][4] = t.t2;
                    if (two) {
                        const PermTable& q = (&t)[1];
                        tq[j][0] = q.t0lo;
                        tq[j][1] = q.t0hi;
                        tq[j][2] = q.t1lo;
                        tq[j][3] = q.t1hi;
                        tq[j][4] = q.t2;
                    }
                }
#pragma unroll
                for (int u = 0; u < SLABS; u++)
#pragma unroll
                    for (int d = 0; d < 4; d++) {
                        const Sel sa = make_sel(x[u][d]);
                        if (two) {
                            const Sel sb = make_sel(xn[u][d]);
#pragma unroll
                            for (int j = 0; j < R; j++) {
                                const uint32_t a0 = __builtin_amdgcn_perm(ta[j][1], ta[j][0], sa.s0);
                                const uint32_t a1 = __builtin_amdgcn_perm(ta[j][3], ta[j][2], sa.s1);
                                const uint32_t a2 = __builtin_amdgcn_perm(ta[j][4], ta[j][4], sa.s2);
                                const uint32_t b0 = __builtin_amdgcn_perm(tq[j][1], tq[j][0], sb.s0);
                                const uint32_t b1 = __builtin_amdgcn_perm(tq[j][3], tq[j][2], sb.s1);
                                const uint32_t b2 = __builtin_amdgcn_perm(tq[j][4], tq[j][4], sb.s2);
                                acc[u][j][d] = xor3(xor3(xor3(acc[u][j][d], a0, a1), a2, b0), b1, b2);
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < R; j++)
                                acc[u][j][d] ^= gf_mul4(ta[j][0], ta[j][1], ta[j][2], ta[j][3], ta[j][4], sa.s0,
                                                        sa.s1, sa.s2);
                        }
                    }
                }  // !BSL
                __builtin_amdgcn_sched_barrier(0);
                if (i + 2 < K) {
#pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        x[u] = load16<true>(a.in[i + 2] + (uint64_t(stripe) * a.in_stride[i + 2] + wbyte) + voff[u]);
                }
                if (i + 3 < K) {
#pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        xn[u] = load16<true>(a.in[i + 3] + (uint64_t(stripe) * a.in_stride[i + 3] + wbyte) + voff[u]);
                }
                if constexpr (EARLY_OUT) {
                    if (i + 2 >= K) {  // last pair: rows out and the next tile's loads before its round
                        __builtin_amdgcn_sched_barrier(0);
                        emit_outputs();
                        prefetch_next(K > 1);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                after_stage(two ? i + 1 : i);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < K; i++) {
                if (PF && !BSL && i + 1 < K) {
    #pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        xn[u] = load16<true>(a.in[i + 1] + (uint64_t(stripe) * a.in_stride[i + 1] + wbyte) + voff[u]);
                }
                __builtin_amdgcn_sched_barrier(0);
    #pragma unroll
                for (int u = 0; u < SLABS; u++) stage_piece(i % SPR, u, x[u]);
                if constexpr (BSL) {
                    bsl_absorb(i, x);
                } else {
                // opaque per-input table offset threaded through the
                // accumulators: keeps the table reads (and the GF math) of input
                // i from being hoisted next to those of the other inputs
                uint32_t toff = uint32_t(i) * uint32_t(sizeof(PermTable));
                asm volatile("" : "+v"(toff));
    #pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    asm volatile("" : "+v"(x[u]));
    #pragma unroll
                    for (int j = 0; j < R; j++) asm volatile("" : "+v"(acc[u][j]) : "v"(toff));
                }
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
                for (int u = 0; u < SLABS; u++)
    #pragma unroll
                    for (int d = 0; d < 4; d++) {
                        const Sel sl = make_sel(x[u][d]);
    #pragma unroll
                        for (int j = 0; j < R; j++)
                            acc[u][j][d] ^= gf_mul4(tb[j][0], tb[j][1], tb[j][2], tb[j][3], tb[j][4], sl.s0, sl.s1, sl.s2);
                    }
                }  // !BSL
                __builtin_amdgcn_sched_barrier(0);
                // BSL: the next shard's loads go out after this shard's GF
                // math (x is dead by then), in flight across the CRC round
                if (BSL && i + 1 < K) {
    #pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        x[u] = load16<true>(a.in[i + 1] + (uint64_t(stripe) * a.in_stride[i + 1] + wbyte) + voff[u]);
                }
                if constexpr (EARLY_OUT) {
                    if (i + 1 == K) {  // last input: rows out and the next tile's input 0 before its round
                        __builtin_amdgcn_sched_barrier(0);
                        emit_outputs();
                        prefetch_next(false);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                after_stage(i);
                __builtin_amdgcn_sched_barrier(0);
                if (!BSL && i + 1 < K) {
    #pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        x[u] = PF ? xn[u]
                                  : load16<true>(a.in[i + 1] + (uint64_t(stripe) * a.in_stride[i + 1] + wbyte) + voff[u]);
                }
            }
        }
        if constexpr (!EARLY_OUT) {
#pragma unroll
            for (int j = 0; j < R; j++) {
                u32x4 o[SLABS];
                if constexpr (BSL) {
                    bsl_output(j, o);
                } else {
#pragma unroll
                    for (int u = 0; u < SLABS; u++) o[u] = acc[u][j];
                }
#pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    if (live[u]) store16<true>(a.out[j] + (uint64_t(stripe) * a.out_stride[j] + wbyte) + voff[u], o[u]);
                    if constexpr (!VERIFY) stage_piece((K + j) % SPR, u, o[u]);
                }
                if constexpr (!VERIFY) after_stage(K + j);
            }
        }
    }
}

}  // namespace hec
