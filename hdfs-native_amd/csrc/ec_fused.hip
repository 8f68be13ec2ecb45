// ec_fused.hip -- the GF(2^8) stripe multiply fused with the per-chunk
// checksums of the cells it streams, so that a striped
// write or read touches HBM once:
//   * encode: parity of the k data cells plus the CRC32C of all k+m cells
//     (CellBuffer::encode, block_writer.rs:817-851, feeding k+m packet
//     streams whose WritePacket::calculate_checksum, connection.rs:568-584,
//     puts one CRC32C per 512-B chunk);
//   * decode + verify: the read side (block_reader.rs:480-525 -> ec_decode):
//     the k survivors' chunk checksums (CRC32C or CRC32 = CRC_32_CKSUM,
//     ReadPacket::get_data, connection.rs:477-504) are checked against the
//     sums that came with their packets while the missing data cells are
//     rebuilt from the same registers; a mismatch flags the cell
//     (HdfsError::ChecksumError), and the host re-plans that stripe.
// Register GF math as in gf_matmul_v16 (ec_kernels.hip); each wave drops its
// 1-KiB pieces -- each exactly two chunk-aligned 512-B chunks -- into a
// wave-private LDS image of 144-B quarter rows and runs the quarter-chunk
// checksum of checksum.hip over it in rounds of 64 quarters.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "checksum.hpp"
#include "checksum_device.hpp"
#include "checksum_tables.hpp"
#include "bitslice.hpp"
#include "ec_kernels.hpp"
#include "gf_device.hpp"
#include "xor_networks.hpp"

namespace hec {

namespace {
__constant__ crc::Tables<crc::kCrc32c> kFusedCrc32c = crc::Tables<crc::kCrc32c>();
__constant__ crc::Tables<crc::kCksum> kFusedCksum = crc::Tables<crc::kCksum>();

template <int KIND>
__device__ __forceinline__ const crc::Tables<KIND>& fused_tables() {
    if constexpr (KIND == crc::kCrc32c)
        return kFusedCrc32c;
    else
        return kFusedCksum;
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
template <int K, int R, int SLABS, int SCHEME, int KIND, bool VERIFY, int WPE = 2, bool PAIR = false,
          bool BSL = false>
__global__ __launch_bounds__(crcdev::sliced(SCHEME) ? 128 * WPE * (WPE - 1) : 512)
    __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void gf_fused_crc(
    MatmulArgs a, FusedCrcArgs cs) {
    static_assert(!BSL || (!VERIFY && bitslice::rs_net_available<K, R>() && SLABS % 2 == 0), "bit-sliced encode");
    using TL = crcdev::TableLayout<SCHEME>;
    using Spec = crc::Spec<KIND>;
    constexpr bool REFL = Spec::kReflected;
    // sliced schemes: WPE = 2 -> 256-thread blocks, two per CU; WPE = 3 ->
    // one 768-thread block per CU (12 waves, 3 per SIMD)
    constexpr int BS = crcdev::sliced(SCHEME) ? 128 * WPE * (WPE - 1) : 512, WAVES = BS / 64;
    constexpr int PITCH = 144, STAGE = 64 * PITCH, SPR = 8 / SLABS;
    constexpr int NSUM = VERIFY ? K : K + R;  // checksummed shards
    constexpr uint32_t WAVE_BYTES = SLABS * 1024u, TILE_BYTES = WAVES * WAVE_BYTES;
    constexpr bool PF = R * SLABS <= 24;  // register prefetch of the next shard
    __shared__ PermTable s_tab[R][K];  // K columns: scheme 11 needs 2 x 79 KiB per CU
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    __shared__ uint32_t s_ctabs[TL::kWords];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[WAVES * STAGE];
    prologue<R, BS, K>(a, K, s_tab, s_exp, s_log, s_coef);
    crcdev::stage_tables<SCHEME, BS>(s_ctabs, fused_tables<KIND>());
    __syncthreads();
    const uint32_t kfinal = fused_tables<KIND>().final512;

    const uint64_t cell_len = a.cell_len;
    const uint64_t nck = (cell_len + 511) / 512;  // checksum chunks per cell
    const uint32_t total = a.total_tiles;
    const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
    // this lane's quarter in a round: row `lane` = piece lane/8 = (shard
    // slot sir, slab), chunk half (lane/4)&1 of that slab, quarter qi
    const int qi = lane & 3, piece = lane >> 3, sir = piece / SLABS, pslab = piece % SLABS, half = (lane >> 2) & 1;
    uint8_t* stage = s_stage + wave * STAGE;
    uint32_t* out_sums = reinterpret_cast<uint32_t*>(cs.sums);
    const uint32_t* exp_sums = reinterpret_cast<const uint32_t*>(cs.expected);

    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        uint32_t stripe, tcol;
        tile_coords(tile, a, stripe, tcol);
        const uint64_t wbyte = uint64_t(tcol) * TILE_BYTES + uint64_t(wave) * WAVE_BYTES;  // wave's first byte
        if (wbyte >= cell_len) continue;  // wave-uniform
        // 32-bit lane offsets from a wave-uniform per-shard base (saddr +
        // voffset addressing); dead slabs of a short last tile read slab 0
        const uint64_t left = cell_len - wbyte;
        uint32_t voff[SLABS];
        bool live[SLABS];
#pragma unroll
        for (int u = 0; u < SLABS; u++) {
            const uint32_t o = uint32_t(u) * 1024u + uint32_t(lane) * 16u;
            live[u] = o < left;
            voff[u] = live[u] ? o : 0u;
        }
        const uint64_t cbyte = wbyte + uint64_t(pslab) * 1024u + uint64_t(half) * 512u;
        const bool in_cell = cbyte < cell_len;
        const bool full = in_cell && cell_len - cbyte >= 512u;  // same for a chunk's 4 lanes

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
            if (VERIFY && live_c && qi == 0) want = exp_sums[sum_cell(first) * nck + cbyte / 512];  // issued before the lookups
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
        // input i's share of the parity, bit-sliced (input 0 initialises accp)
        auto bsl_absorb = [&](int i, const u32x4 (&xi)[SLABS]) {
            if constexpr (BSL) {
#pragma unroll
                for (int g = 0; g < SLABS / 2; g++) {
                    uint32_t pl[8] = {xi[2 * g][0],     xi[2 * g][1],     xi[2 * g][2],     xi[2 * g][3],
                                      xi[2 * g + 1][0], xi[2 * g + 1][1], xi[2 * g + 1][2], xi[2 * g + 1][3]};
                    if (i > 0) {
                        // opaque per input: keeps the XOR chains of the
                        // accumulators from being reassociated across inputs
#pragma unroll
                        for (int t = 0; t < R * 8; t++) asm volatile("" : "+v"(accp[g][t]));
                    }
                    bitslice::transpose8(pl);
                    bitslice::rs_absorb_at<K, R>(i, pl, accp[g]);
                    // one group's planes and network temporaries live at a time
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
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
        u32x4 x[SLABS], xn[SLABS];
#pragma unroll
        for (int u = 0; u < SLABS; u++) x[u] = load16<true>(a.in[0] + (uint64_t(stripe) * a.in_stride[0] + wbyte) + voff[u]);
        if constexpr (PAIR && SPR == 2 && PF) {
            // Inputs two at a time (one CRC round): both shards' products go
            // into the accumulators through one chain of 3-input XORs, 3 ops
            // per (dword, output) for the pair instead of 4.  The next pair's
            // loads are issued after this pair's GF math, before its round.
            if (K > 1) {
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

#ifdef HEC_EXPERIMENTAL
// Role-split variant: one 512-thread block per CU, waves 0-3 are GF waves and
// waves 4-7 CRC waves; wave w and w + 4 share a SIMD (a workgroup's waves go
// to the SIMDs cyclically), so every SIMD always holds one wave issuing the
// VALU-heavy GF math and one issuing the LDS-heavy lookups, instead of two
// waves that alternate between the phases.  A pair owns 8 KiB of every cell
// of the stripe (as SLABS = 8) and two 9-KiB images: in round n the GF wave
// loads / multiplies / stages shard n into image n & 1 (parity rounds store
// and stage an output) while the CRC wave checksums round n - 1 from the
// other image; one block barrier ends a round.  Rounds run on across tiles;
// a last round flushes the CRC of the block's last tile.  Every wave runs
// the same rounds and barriers, whatever its role.
// Rejected (same-box A/B, profiles/r02g/probe_split_rs*.log): RS(6,3) x 1024
// encode + CRC 2.68 vs 2.23 ms, decode + verify 2.27-2.33 vs 2.08 ms; RS(10,4)
// x 512 2.23-2.28 vs 1.96 ms and 1.98-2.09 vs 1.84 ms.  One CRC wave per SIMD
// cannot keep the table lookups in flight (ds_read_b32 needs ~4 waves per
// SIMD for its full rate), and the per-round barrier exposes the GF wave's
// load latency.  Measurement build: RS(6,3) and RS(10,4) only.
template <int K, int R, int KIND, bool VERIFY, bool PRIO>
__global__ __launch_bounds__(512) void gf_fused_crc_split(MatmulArgs a, FusedCrcArgs cs) {
    constexpr int SCHEME = 11;
    using TL = crcdev::TableLayout<SCHEME>;
    using Spec = crc::Spec<KIND>;
    constexpr bool REFL = Spec::kReflected;
    constexpr int BS = 512, SLABS = 8, PITCH = 144, STAGE = 64 * PITCH;
    constexpr int NSUM = VERIFY ? K : K + R;
    constexpr uint32_t WAVE_BYTES = SLABS * 1024u, TILE_BYTES = 4u * WAVE_BYTES;
    __shared__ PermTable s_tab[R][K];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ uint8_t s_coef[R * kMaxK];
    __shared__ uint32_t s_ctabs[TL::kWords];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[4][2][STAGE];
    prologue<R, BS, K>(a, K, s_tab, s_exp, s_log, s_coef);
    crcdev::stage_tables<SCHEME, BS>(s_ctabs, fused_tables<KIND>());
    __syncthreads();
    const uint32_t kfinal = fused_tables<KIND>().final512;

    const uint64_t cell_len = a.cell_len;
    const uint64_t nck = (cell_len + 511) / 512;
    const uint32_t total = a.total_tiles;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x & 63;
    const bool gf = wave < 4;
    const int pw = wave & 3;
    if constexpr (PRIO) {
        if (!gf) __builtin_amdgcn_s_setprio(1);
    }
    // CRC role: this lane's quarter row = lane = (slab lane/8, half (lane/4)&1, quarter lane&3)
    const int qi = lane & 3, pslab = lane >> 3, half = (lane >> 2) & 1;
    uint32_t* out_sums = reinterpret_cast<uint32_t*>(cs.sums);
    const uint32_t* exp_sums = reinterpret_cast<const uint32_t*>(cs.expected);

    // LDS writes of this wave done, then the block barrier (no vmcnt wait:
    // the GF wave's loads and stores stay in flight across rounds)
    auto round_end = [&]() {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };

    // CRC of one staged round: shard `sh` of stripe `stripe`, wave bytes from `wbyte`
    auto crc_round = [&](const uint8_t* img, uint32_t stripe, uint64_t wbyte, int sh) {
        const uint64_t cbyte = wbyte + uint64_t(pslab) * 1024u + uint64_t(half) * 512u;
        const bool in_cell = cbyte < cell_len;
        const bool full = in_cell && cell_len - cbyte >= 512u;
        const uint64_t cell = VERIFY ? uint64_t(stripe) * cs.n_total + cs.shard_id[sh]
                                     : uint64_t(stripe) * (K + R) + uint64_t(sh);
        uint32_t want = 0;
        if (VERIFY && in_cell && qi == 0) want = exp_sums[cell * nck + cbyte / 512];
        uint32_t val = 0;
        if (full) {
            uint32_t r = crcdev::quarter<SCHEME, REFL>(s_ctabs, img + lane * PITCH, lane);
            if (qi < 3) r = crcdev::shift_quarter<SCHEME>(s_ctabs, qi, r);
            val = r;
        } else if (in_cell && qi == 0) {
            const uint32_t len = uint32_t(cell_len - cbyte);
            uint32_t r = Spec::kInit;
            for (uint32_t b = 0; b < len; b++)
                r = crcdev::byte_step<REFL, crcdev::ByteTable<SCHEME>::stride, crcdev::ByteTable<SCHEME>::bswap>(
                    s_ctabs + crcdev::ByteTable<SCHEME>::off, r, img[(lane + b / 128) * PITCH + (b % 128)]);
            val = r ^ Spec::kXorout;
        }
        val ^= __shfl_xor(val, 1);
        val ^= __shfl_xor(val, 2);
        if (in_cell && qi == 0) {
            const uint32_t be = __builtin_bswap32(full ? (val ^ kfinal) : val);
            if constexpr (VERIFY) {
                if (be != want) cs.bad[cell] = 1;
            } else {
                out_sums[cell * nck + cbyte / 512] = be;
            }
        }
    };
    auto stage_piece = [&](uint8_t* img, int u, const u32x4& v) {
        *reinterpret_cast<u32x4*>(img + (8 * u + lane / 8) * PITCH + 16 * (lane % 8)) = v;
    };

    // the pair's share of a tile: its first byte, and whether any of it is in the cell
    auto pair_start = [&](uint32_t tile, uint32_t& stripe, uint64_t& wbyte) {
        uint32_t tcol;
        tile_coords(tile, a, stripe, tcol);
        wbyte = uint64_t(tcol) * TILE_BYTES + uint64_t(pw) * WAVE_BYTES;
        return wbyte < cell_len;  // wave-uniform, the same for both waves of a pair
    };

    // The two roles run separate loops (separate register lives) over the same
    // tiles, NSUM rounds each, one barrier per round.
    if (!gf) {
        uint32_t n = 0;  // round counter: image n & 1
        uint32_t p_stripe = 0;
        uint64_t p_wbyte = 0;
        int p_sh = 0;
        bool p_live = false;  // the round staged one round earlier
        for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
            uint32_t stripe;
            uint64_t wbyte;
            const bool work = pair_start(tile, stripe, wbyte);
            for (int s = 0; s < NSUM; s++) {
                if (p_live) crc_round(s_stage[pw][(n - 1) & 1], p_stripe, p_wbyte, p_sh);
                p_stripe = stripe;
                p_wbyte = wbyte;
                p_sh = s;
                p_live = work;
                n++;
                round_end();
            }
        }
        if (p_live) crc_round(s_stage[pw][(n - 1) & 1], p_stripe, p_wbyte, p_sh);  // flush
        return;
    }

    uint32_t n = 0;
    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        uint32_t stripe;
        uint64_t wbyte;
        const bool work = pair_start(tile, stripe, wbyte);
        if (!work) {
            for (int s = 0; s < NSUM; s++) round_end();
            n += NSUM;
            continue;
        }
        const uint64_t left = cell_len - wbyte;
        uint32_t voff[SLABS];
        bool live[SLABS];
        u32x4 acc[SLABS][R];
        u32x4 x[SLABS];
#pragma unroll
        for (int u = 0; u < SLABS; u++) {
            const uint32_t o = uint32_t(u) * 1024u + uint32_t(lane) * 16u;
            live[u] = o < left;
            voff[u] = live[u] ? o : 0u;
#pragma unroll
            for (int j = 0; j < R; j++) acc[u][j] = u32x4{0, 0, 0, 0};
            x[u] = load16<true>(a.in[0] + (uint64_t(stripe) * a.in_stride[0] + wbyte) + voff[u]);
        }
#pragma unroll
        for (int i = 0; i < K; i++) {
            // input i; its loads were issued in the last round and land while
            // the wave waits at the barrier
            uint8_t* img = s_stage[pw][(n + i) & 1];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < SLABS; u++) stage_piece(img, u, x[u]);
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
                const PermTable& t = *reinterpret_cast<const PermTable*>(reinterpret_cast<const char*>(&s_tab[j][0]) + toff);
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
            __builtin_amdgcn_sched_barrier(0);
            if (i + 1 < K) {
#pragma unroll
                for (int u = 0; u < SLABS; u++)
                    x[u] = load16<true>(a.in[i + 1] + (uint64_t(stripe) * a.in_stride[i + 1] + wbyte) + voff[u]);
            }
            if (VERIFY && i == K - 1) {
#pragma unroll
                for (int j = 0; j < R; j++)
#pragma unroll
                    for (int u = 0; u < SLABS; u++)
                        if (live[u])
                            store16<true>(a.out[j] + (uint64_t(stripe) * a.out_stride[j] + wbyte) + voff[u], acc[u][j]);
            }
            __builtin_amdgcn_sched_barrier(0);
            round_end();
        }
        if constexpr (!VERIFY) {
#pragma unroll
            for (int j = 0; j < R; j++) {
                uint8_t* img = s_stage[pw][(n + K + j) & 1];
#pragma unroll
                for (int u = 0; u < SLABS; u++) {
                    if (live[u]) store16<true>(a.out[j] + (uint64_t(stripe) * a.out_stride[j] + wbyte) + voff[u], acc[u][j]);
                    stage_piece(img, u, acc[u][j]);
                }
                round_end();
            }
        }
        n += NSUM;
    }
}

#endif  // HEC_EXPERIMENTAL

namespace {

// 8 slabs per wave while the r x 8 accumulators fit (k <= 6, r <= 3), else 4
constexpr int fused_slabs(int k, int r) { return (r <= 3 && k <= 6) ? 8 : 4; }

template <int K, int R, int SCHEME, int WPE = 2>
const void* encode_sl(int slabs, bool pair = false) {
    if constexpr (WPE == 3) return reinterpret_cast<const void*>(&gf_fused_crc<K, R, 4, SCHEME, crc::kCrc32c, false, 3>);
    if (slabs == 4 && pair)
        return reinterpret_cast<const void*>(&gf_fused_crc<K, R, 4, SCHEME, crc::kCrc32c, false, 2, true>);
    return slabs == 4 ? reinterpret_cast<const void*>(&gf_fused_crc<K, R, 4, SCHEME, crc::kCrc32c, false>)
                      : reinterpret_cast<const void*>(&gf_fused_crc<K, R, 8, SCHEME, crc::kCrc32c, false>);
}

template <int K, int R, int SCHEME, int WPE = 2>
const void* verify_kind(int kind, bool pair = false) {
    constexpr int SL = WPE == 3 ? 4 : fused_slabs(K, R);
    if constexpr (SL == 4 && WPE == 2) {
        if (pair)
            return kind == crc::kCrc32c
                       ? reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCrc32c, true, 2, true>)
                       : reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCksum, true, 2, true>);
    }
    return kind == crc::kCrc32c ? reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCrc32c, true, WPE>)
                                : reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCksum, true, WPE>);
}

// scheme 12 (default) = the fold + 11-bit slicing of the tail; the
// measurement build adds 11 = 11-bit slicing (tune key 11 = 5), 1 =
// slicing-by-8 (key 11 = 1), the rejected schemes and shapes.  The product
// library compiles the default slab count / pairing of each (K, R) only.
// the bit-sliced parity (BSL) for the RS coding matrix of (K, R) with a
// generated network; RS(2,1) keeps the v_perm tables (no gain: 162 vs 160 VALU)
template <int K, int R>
constexpr bool bsl_shape() {
    return bitslice::rs_net_available<K, R>() && K > 2;
}

template <int K, int R, int SCHEME, bool PAIR>
const void* encode_bsl(bool bsl) {
    constexpr int SL = fused_slabs(K, R);
    if constexpr (bsl_shape<K, R>())
        if (bsl) return reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCrc32c, false, 2, PAIR, true>);
    return reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCrc32c, false, 2, PAIR>);
}

template <int K, int R>
const void* encode_fn(int slabs, int scheme, int wpe, bool pair, bool bsl) {
#ifndef HEC_EXPERIMENTAL
    (void)slabs;
    (void)scheme;
    (void)wpe;
    (void)pair;
    constexpr int SL = fused_slabs(K, R);
    return encode_bsl<K, R, 12, SL == 4>(bsl);
#else
    // bit-sliced parity at the default slab count (tune key 22 = 1: off)
    if (bsl && scheme == 12 && wpe != 3 && slabs == fused_slabs(K, R) && (slabs == 8 || pair))
        return encode_bsl<K, R, 12, fused_slabs(K, R) == 4>(true);
    // fold depth 16 / 20 dwords (key 11 = 10 / 11), RS(6,3) and RS(10,4) only
    if constexpr ((K == 6 && R == 3) || (K == 10 && R == 4)) {
        if ((scheme == 13 || scheme == 14) && bsl && wpe != 3 && slabs == fused_slabs(K, R) && (slabs == 8 || pair))
            return scheme == 13 ? encode_bsl<K, R, 13, fused_slabs(K, R) == 4>(true)
                                : encode_bsl<K, R, 14, fused_slabs(K, R) == 4>(true);
    }
    if (scheme == 13 || scheme == 14) return nullptr;
    // bit-sliced parity at 4 slabs in one 768-thread block per CU (3 waves per
    // SIMD; tune key 16 = 3), RS(6,3) and RS(10,4)
    if constexpr ((K == 6 && R == 3) || (K == 10 && R == 4)) {
        if (bsl && scheme == 12 && wpe == 3)
            return reinterpret_cast<const void*>(&gf_fused_crc<K, R, 4, 12, crc::kCrc32c, false, 3, false, true>);
    }
    // rejected (same-box A/B, profiles/r01_probe_fused_scheme.log,
    // r02_probe_fused_rep2.log, r02_probe_fused_wpe3_*.log):
    // bank-replicated slicing-by-1 (4 chains) and slicing-by-2 (tune key 11
    // = 2 / 6), one 768-thread block per CU at 3 waves per SIMD (key 16 = 3)
    if (scheme == 4) return encode_sl<K, R, 4>(slabs);
    if (scheme == 22) return encode_sl<K, R, 22>(slabs);
    if (wpe == 3) return scheme == 11 ? encode_sl<K, R, 11, 3>(slabs) : encode_sl<K, R, 1, 3>(slabs);
    if (scheme == 12) return encode_sl<K, R, 12>(slabs, pair);
    return scheme == 11 ? encode_sl<K, R, 11>(slabs, pair) : encode_sl<K, R, 1>(slabs, pair);
#endif
}

template <int K, int R>
const void* verify_fn(int kind, int scheme, int wpe, bool pair) {
#ifndef HEC_EXPERIMENTAL
    (void)scheme;
    (void)wpe;
    (void)pair;
    constexpr int SL = fused_slabs(K, R);
    return kind == crc::kCrc32c
               ? reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, 12, crc::kCrc32c, true, 2, SL == 4>)
               : reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, 12, crc::kCksum, true, 2, SL == 4>);
#else
    if (scheme == 22) return verify_kind<K, R, 22>(kind);
    if constexpr ((K == 6 && R == 3) || (K == 10 && R == 4)) {
        constexpr int SL = fused_slabs(K, R);
        if ((scheme == 13 || scheme == 14) && wpe != 3 && kind == crc::kCrc32c)
            return scheme == 13
                       ? reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, 13, crc::kCrc32c, true, 2, SL == 4>)
                       : reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, 14, crc::kCrc32c, true, 2, SL == 4>);
    }
    if (scheme == 13 || scheme == 14) return nullptr;
    if (wpe == 3) return scheme == 11 ? verify_kind<K, R, 11, 3>(kind) : verify_kind<K, R, 1, 3>(kind);
    if (scheme == 12) return verify_kind<K, R, 12>(kind, pair);
    return scheme == 11 ? verify_kind<K, R, 11>(kind, pair) : verify_kind<K, R, 1>(kind, pair);
#endif
}

#ifdef HEC_EXPERIMENTAL
// role-split kernel (tune key 21 = 2, or 3 with the CRC waves at raised priority)
template <int K, int R>
const void* split_fn(bool verify, int kind, bool prio) {
    if (!verify)
        return prio ? reinterpret_cast<const void*>(&gf_fused_crc_split<K, R, crc::kCrc32c, false, true>)
                    : reinterpret_cast<const void*>(&gf_fused_crc_split<K, R, crc::kCrc32c, false, false>);
    if (kind == crc::kCrc32c)
        return prio ? reinterpret_cast<const void*>(&gf_fused_crc_split<K, R, crc::kCrc32c, true, true>)
                    : reinterpret_cast<const void*>(&gf_fused_crc_split<K, R, crc::kCrc32c, true, false>);
    return prio ? reinterpret_cast<const void*>(&gf_fused_crc_split<K, R, crc::kCksum, true, true>)
                : reinterpret_cast<const void*>(&gf_fused_crc_split<K, R, crc::kCksum, true, false>);
}

template <int K>
const void* pick_split(bool verify, int r, int kind, bool prio) {
    if (K == 6 && r == 3) return split_fn<6, 3>(verify, kind, prio);
    if (K == 10 && r == 4) return split_fn<10, 4>(verify, kind, prio);
    return nullptr;
}

#endif

template <int K>
const void* pick_r(bool verify, int r, int slabs, int scheme, int kind, int wpe, bool pair, bool bsl) {
    switch (r) {
        case 1: return verify ? verify_fn<K, 1>(kind, scheme, wpe, pair) : encode_fn<K, 1>(slabs, scheme, wpe, pair, bsl);
        case 2: return verify ? verify_fn<K, 2>(kind, scheme, wpe, pair) : encode_fn<K, 2>(slabs, scheme, wpe, pair, bsl);
        case 3: return verify ? verify_fn<K, 3>(kind, scheme, wpe, pair) : encode_fn<K, 3>(slabs, scheme, wpe, pair, bsl);
        default: return verify ? verify_fn<K, 4>(kind, scheme, wpe, pair) : encode_fn<K, 4>(slabs, scheme, wpe, pair, bsl);
    }
}

int launch_fused(const MatmulArgs& in, const FusedCrcArgs& cs, bool verify, int device, hipStream_t stream) {
    MatmulArgs a = in;
    const Tune tn = tune_snapshot();
    const void* sums = verify ? static_cast<const void*>(cs.expected) : static_cast<const void*>(cs.sums);
    bool aligned = a.cell_len % 16 == 0 && sums && (reinterpret_cast<uintptr_t>(sums) & 3u) == 0 && a.r >= 1 &&
                   a.r <= kMaxR && (!verify || cs.bad);
    for (int i = 0; i < a.k; i++)
        aligned &= ((reinterpret_cast<uintptr_t>(a.in[i]) | a.in_stride[i]) & 15u) == 0;
    for (int j = 0; j < a.r; j++)
        aligned &= ((reinterpret_cast<uintptr_t>(a.out[j]) | a.out_stride[j]) & 15u) == 0;
    if (cs.kind != crc::kCrc32c && (cs.kind != crc::kCksum || !verify)) return -1;
    const int slabs = tn.fused_wpe == 3                                    ? 4
                      : verify                                               ? fused_slabs(a.k, a.r)
                      : (tn.fused_slabs == 4 || tn.fused_slabs == 8) ? tn.fused_slabs
                                                                             : fused_slabs(a.k, a.r);
    // checksum lookups (checksum_device.hpp): 11-bit slicing (6 lookups per
    // 8 bytes; the default before the fold), slicing-by-8 on tune key 11 = 1; both in 256-thread
    // blocks, 2 per CU.  Same-box A/B (profiles/r02_probe_fused_w11_*.log):
    // encode + CRC 5-7 % faster with 11-bit slicing, decode + verify within
    // +-1 %.  The kernel is bound by its VALU/issue stream more than by the
    // LDS: the bank-replicated tables (conflict-free, half the LDS cycles,
    // 1.5x the VALU) lose 10-20 % (r02_probe_fused_rep2.log).
    // Default since round 2 (session k): the fold (scheme 12, checksum_device.hpp
    // quarter_fold), 24 lookups per 128-B quarter instead of 96; same box,
    // RS(6,3) x 1024 (profiles/r02k_fold/crc63_v*.json): encode + CRC 2.18-2.21
    // -> 1.96-1.97 ms (4.38-4.43 -> 4.90-4.94 TB/s), decode + verify 1.96-1.99
    // -> 1.82 ms.  11-bit slicing on key 11 = 5.
    // measurement: fold depth 16 / 20 dwords (key 11 = 10 / 11)
    const int scheme = tn.crc_variant == 10             ? 13
                       : tn.crc_variant == 11           ? 14
                       : (!verify && tn.crc_variant == 2) ? 4
                       : tn.crc_variant == 6            ? 22
                       : tn.crc_variant == 1            ? 1
                       : tn.crc_variant == 5            ? 11
                                                        : 12;
    const int wpe = (tn.fused_wpe == 3 && crcdev::sliced(scheme)) ? 3 : 2;
    // at 4 slabs (two shards per round) the inputs go two at a time: same-box
    // A/B (profiles/r02_probe_fused_pair.log) RS(10,4) x 512 encode + CRC
    // 1.950 -> 1.915 ms, decode + verify 1.878 -> 1.818 ms; at k <= 6 the
    // 8-slab kernel (no pairs) stays faster than 4 slabs with pairs
    const bool pair = tn.fused_pair != 1;
#ifdef HEC_EXPERIMENTAL
    // role-split GF / CRC waves (tune key 21 = 2 / 3): rejected, see the kernel
    const bool split = tn.fused_split == 2 || tn.fused_split == 3;
    const bool prio = tn.fused_split == 3;
#else
    constexpr bool split = false;
#endif
    const int waves = split ? 8 : !crcdev::sliced(scheme) ? 8 : wpe == 3 ? 12 : 4;
    const void* fn = nullptr;
    if (split) {
#ifdef HEC_EXPERIMENTAL
        switch (a.k) {
            case 6: fn = pick_split<6>(verify, a.r, cs.kind, prio); break;
            case 10: fn = pick_split<10>(verify, a.r, cs.kind, prio); break;
            default: return -1;
        }
        if (!fn) return -1;
#endif
    } else {
        // encode with the RS matrix: the bit-sliced parity (tune key 22 = 1: the
        // v_perm tables, measurement build)
        const bool bsl = !verify && tn.fused_bsl != 1 && rs_parity_matrix(a);
        switch (a.k) {
            case 2: fn = pick_r<2>(verify, a.r, slabs, scheme, cs.kind, wpe, pair, bsl); break;
            case 3: fn = pick_r<3>(verify, a.r, slabs, scheme, cs.kind, wpe, pair, bsl); break;
            case 6: fn = pick_r<6>(verify, a.r, slabs, scheme, cs.kind, wpe, pair, bsl); break;
            case 10: fn = pick_r<10>(verify, a.r, slabs, scheme, cs.kind, wpe, pair, bsl); break;
            default: return -1;
        }
        if (!fn) return -1;  // a measurement scheme not compiled for this shape
    }
    if (!aligned) return -1;
    const uint64_t chunks = a.cell_len / 16;
    // split: 4 GF waves x 8 KiB per tile; else waves x slabs x 1 KiB
    const uint64_t tile_bytes = split ? 4u * 8192u : 1024u * uint64_t(slabs) * uint64_t(waves);
    const uint64_t tps = (a.cell_len + tile_bytes - 1) / tile_bytes;
    const uint64_t total = tps * a.stripes;
    if (chunks > 0xFFFFFFFFull || total > 0xFFFFFFFFull) return -1;
    if (total == 0) return 0;
    a.chunks = uint32_t(chunks);
    a.tiles_per_stripe = uint32_t(tps);
    a.total_tiles = uint32_t(total);
    tile_order(a.stripes, a.tiles_per_stripe, tn.group > 0 ? uint32_t(tn.group) : 4u, a.group, a.grouped_tiles);
    // LDS: ~61 KiB per 256-thread block (two per CU) / ~131 KiB per 512-thread block (one)
    // a grid of 8 blocks per CU (2 or 1 resident): finer-grained dynamic
    // scheduling beats exactly the resident blocks by 3 % (RS(6,3)) to 5 %
    // (RS(10,4))
    uint64_t grid = tn.grid ? uint64_t(tn.grid) : uint64_t(num_cus(device)) * ((split || wpe == 3) ? 4 : 8);
    if (grid > total) grid = total;
    FusedCrcArgs c = cs;
    void* args[] = {&a, &c};
    const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(uint32_t(waves * 64)), args, 0, stream);
    return e == hipSuccess ? 0 : int(e);
}

}  // namespace

int launch_encode_crc(const MatmulArgs& a, const FusedCrcArgs& c, int device, hipStream_t stream) {
    return launch_fused(a, c, false, device, stream);
}

int launch_decode_verify(const MatmulArgs& a, const FusedCrcArgs& c, int device, hipStream_t stream) {
    return launch_fused(a, c, true, device, stream);
}

}  // namespace hec
