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

#include "ec_fused_kernel.hpp"
#include "jit.hpp"

namespace hec {

// The role-split variant (GF waves and CRC waves paired on each SIMD; tune
// key 21 = 2 / 3) lost 10-20 % (profiles/r02g/probe_split_rs*.log) and was
// removed in round 6 (git history keeps it).

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
        if (bsl) return reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCrc32c, false, 2, PAIR, RsNet<K, R>>);
    return reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, SCHEME, crc::kCrc32c, false, 2, PAIR>);
}

// encode + CRC with the work queue of wave-tiles (gf_device.hpp WaveQueue),
// the default bit-sliced shape; the product compiles it for k = 3 and 10
// (launch_fused: the k it wins at)
template <int K, int R>
const void* encode_wq_fn(int slabs = 0) {
    constexpr int SL = fused_slabs(K, R);
#ifdef HEC_EXPERIMENTAL
    // measurement: 4 slabs with the inputs in pairs where the default is 8
    // (tune keys 28 = 1, 10 = 4)
    if constexpr (bsl_shape<K, R>() && SL == 8)
        if (slabs == 4)
            return reinterpret_cast<const void*>(
                &gf_fused_crc<K, R, 4, 12, crc::kCrc32c, false, 2, true, RsNet<K, R>, 1, true>);
#endif
    (void)slabs;
    if constexpr (bsl_shape<K, R>() && (kExperimental || K != 6))
        return reinterpret_cast<const void*>(
            &gf_fused_crc<K, R, SL, 12, crc::kCrc32c, false, 2, SL == 4, RsNet<K, R>, 1, true>);
    return nullptr;
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
    // bit-sliced parity at 4 slabs with the inputs in pairs where the default
    // is 8 (RS(3,2), RS(6,3); tune key 10 = 4), one or two pairs loaded ahead
    // (key 24 = 2): the measurement twin of the specialised decode + verify shapes
    if constexpr (bsl_shape<K, R>() && fused_slabs(K, R) == 8) {
        // key 24 = 3: the default 8-slab shape with each input's loads issued
        // before its parity math (the parity reads the staged copy)
        if (bsl && scheme == 12 && wpe == 2 && slabs == 8 && tune_snapshot().jit_pfd == 3)
            return reinterpret_cast<const void*>(
                &gf_fused_crc<K, R, 8, 12, crc::kCrc32c, false, 2, false, RsNet<K, R>, 3>);
        if (bsl && scheme == 12 && wpe == 2 && slabs == 4 && pair)
            return tune_snapshot().jit_pfd == 2
                       ? reinterpret_cast<const void*>(
                             &gf_fused_crc<K, R, 4, 12, crc::kCrc32c, false, 2, true, RsNet<K, R>, 2>)
                       : reinterpret_cast<const void*>(
                             &gf_fused_crc<K, R, 4, 12, crc::kCrc32c, false, 2, true, RsNet<K, R>, 1>);
    }
    // fold depth 16 / 20 dwords (key 11 = 10 / 11), RS(6,3) and RS(10,4) only
    if constexpr ((K == 6 && R == 3) || (K == 10 && R == 4)) {
        if ((scheme == 13 || scheme == 14) && bsl && wpe != 3 && slabs == fused_slabs(K, R) && (slabs == 8 || pair))
            return scheme == 13 ? encode_bsl<K, R, 13, fused_slabs(K, R) == 4>(true)
                                : encode_bsl<K, R, 14, fused_slabs(K, R) == 4>(true);
        // slicing-by-32 CRC tail (key 11 = 12)
        if (scheme == 15 && bsl && wpe != 3 && slabs == fused_slabs(K, R) && (slabs == 8 || pair))
            return encode_bsl<K, R, 15, fused_slabs(K, R) == 4>(true);
    }
    if (scheme == 13 || scheme == 14 || scheme == 15) return nullptr;
    // bit-sliced parity at 4 slabs in one 768-thread block per CU (3 waves per
    // SIMD; tune key 16 = 3), RS(6,3) and RS(10,4)
    if constexpr ((K == 6 && R == 3) || (K == 10 && R == 4)) {
        if (bsl && scheme == 12 && wpe == 3)
            return reinterpret_cast<const void*>(&gf_fused_crc<K, R, 4, 12, crc::kCrc32c, false, 3, false, RsNet<K, R>>);
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
        if (scheme == 15 && wpe != 3 && kind == crc::kCrc32c)
            return reinterpret_cast<const void*>(&gf_fused_crc<K, R, SL, 15, crc::kCrc32c, true, 2, SL == 4>);
    }
    if (scheme == 13 || scheme == 14 || scheme == 15) return nullptr;
    if (wpe == 3) return scheme == 11 ? verify_kind<K, R, 11, 3>(kind) : verify_kind<K, R, 1, 3>(kind);
    if (scheme == 12) return verify_kind<K, R, 12>(kind, pair);
    return scheme == 11 ? verify_kind<K, R, 11>(kind, pair) : verify_kind<K, R, 1>(kind, pair);
#endif
}


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
                       : tn.crc_variant == 12           ? 15
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
    constexpr bool split = false;  // the role-split kernel is gone (round 6); key 21 is retired
    const int waves = !crcdev::sliced(scheme) ? 8 : wpe == 3 ? 12 : 4;
    const void* fn = nullptr;
    {
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
        // a measurement scheme not compiled for this shape (decode + verify:
        // unless its specialised kernel is ready, below)
        if (!fn && !verify) return -1;
    }
    if (!aligned) return -1;
    // decode + verify at the default scheme: the plan's own bit-sliced network
    // when its specialised kernel is compiled (jit.hpp), same block; its slab
    // count is jit::default_slabs (4; measurement build: tune key 10), the
    // tile geometry below follows it
    jit::VerifyKernel vk;
    int use_slabs = slabs;
    bool vwq = false;  // the specialised kernel takes the work queue (tune key 28 / jit::default_wq)
    if (verify && !split && (scheme == 12 || (scheme == 15 && cs.kind == crc::kCrc32c))) {
        uint8_t mat[kMaxR * kMaxK];
        for (int j = 0; j < a.r; j++)
            for (int i = 0; i < a.k; i++) mat[j * a.k + i] = a.coef[j * kMaxK + i];
        const int js = (tn.fused_slabs == 4 || tn.fused_slabs == 8) ? tn.fused_slabs : jit::default_slabs(a.k, a.r);
        const int jp = jit::pick_pfd(tn.jit_pfd, js, a.k, a.r);
        // (3 waves per SIMD: tune key 16 = 3 with key 10 = 4; the launch's
        // `waves` and grid already follow wpe)
        vwq = (kExperimental && tn.fused_wq) ? tn.fused_wq == 1 : jit::default_wq(a.k, a.r);
        if (jit::verify_kernel(device, a.k, a.r, cs.kind, js, wpe, jp, mat, false, &vk, scheme, vwq)) use_slabs = js;
    }
    // Encode + CRC with the work queue of wave-tiles at k = 3 and 10; k = 6
    // keeps the block tiles (decode + verify: the queue at every k,
    // jit::default_wq).  Same process and buffers, 2 sets x 5 alternated
    // rounds (scripts/probe_fused_wq.py, profiles/r05z): RS(10,4) x 256
    // 0.675-0.683 of HBM peak vs 0.627-0.628, RS(3,2) x 1024 0.721-0.724 vs
    // 0.697-0.698, RS(6,3) x 1024 0.697-0.709 vs 0.703-0.712.  Tune key 28
    // (measurement build): 1 = the queue at k = 3, 6, 10; 2 = block tiles.
    bool wq = false;
    QueueLease lease;  // work-queue counters (held until the launch is enqueued)
    const bool wq_want = kExperimental && tn.fused_wq ? tn.fused_wq == 1 : (a.k == 3 || a.k == 10);
    const bool wq_shape = slabs == fused_slabs(a.k, a.r) || (kExperimental && slabs == 4);
    if (wq_want && !verify && !split && fn && scheme == 12 && wpe == 2 && !vk.fn && wq_shape &&
        rs_parity_matrix(a) && tn.fused_bsl != 1) {
        const void* f = nullptr;
        switch (a.k * 16 + a.r) {
            case 3 * 16 + 2: f = encode_wq_fn<3, 2>(slabs); break;
            case 6 * 16 + 3: f = encode_wq_fn<6, 3>(slabs); break;
            case 10 * 16 + 4: f = encode_wq_fn<10, 4>(slabs); break;
            default: break;
        }
        if (f) lease = queue_lease(device, stream);
        if (lease) {
            fn = f;
            wq = true;
        }
    }
    if (vk.fn && vwq) {
        lease = queue_lease(device, stream);
        if (lease)
            wq = true;
        else
            vk.fn = nullptr;  // no counters: the generic kernel (below) instead
        if (!vk.fn) use_slabs = slabs;
    }
    a.queue = lease.use;
    a.queue_zero = lease.zero;
    if (!fn && !vk.fn) return -1;
    const uint64_t chunks = a.cell_len / 16;
    // split: 4 GF waves x 8 KiB per tile; else waves x slabs x 1 KiB (work
    // queue: one wave's slabs)
    const uint64_t tile_bytes =
        split ? 4u * 8192u : 1024u * uint64_t(use_slabs) * uint64_t(wq ? 1 : waves);
    const uint64_t tps = (a.cell_len + tile_bytes - 1) / tile_bytes;
    const uint64_t total = tps * a.stripes;
    if (chunks > 0xFFFFFFFFull || total > 0xFFFFFFFFull) return -1;
    if (total == 0) return 0;
    a.chunks = uint32_t(chunks);
    a.tiles_per_stripe = uint32_t(tps);
    a.total_tiles = uint32_t(total);
    // tile order: groups of 8 stripes (the register kernels keep 4); same
    // buffers, 3 placements x 3 rounds (profiles/r04p): with 32 blocks per CU,
    // encode + CRC 1.720 vs 1.727 ms for 4-stripe groups, 1.737-1.759 at 16
    // blocks per CU; decode + verify level
    tile_order(a.stripes, a.tiles_per_stripe, tn.group > 0 ? uint32_t(tn.group) : 8u, a.group, a.grouped_tiles);
    a.col_rot = uint32_t(tn.col_rot);  // measurement (key 25); 0 in the product
    // LDS: ~61 KiB per 256-thread block (two per CU) / ~131 KiB per 512-thread block (one)
    // a grid of 32 blocks per CU (2 resident): finer-grained dynamic
    // scheduling beats exactly the resident blocks by 3 % (RS(6,3)) to 5 %
    // (RS(10,4)) at 8 per CU; on the same buffers 16 beats 8
    // by 1-2 % (profiles/r04n: decode + verify 1.728 vs 1.747 ms, encode +
    // CRC 1.776 vs 1.803), 32 beats 8 by 1.5-2 % (r04o) and ties 16 (r04p;
    // 64: 1-2 % slower)
    uint64_t grid = tn.grid ? uint64_t(tn.grid) : uint64_t(num_cus(device)) * ((split || wpe == 3) ? 4 : 32);
    if (wq && !tn.grid) grid = uint64_t(num_cus(device)) * (wpe == 3 ? 1 : 2);  // the resident blocks drain the queue
    if (grid > total) grid = total;
    FusedCrcArgs c = cs;
    c.sums_nt = tn.crc_sums_nt == 1 ? 1u : 0u;  // measurement (key 30)
    void* args[] = {&a, &c};
    if (vk.fn) {
        jit::count_launch();
        const hipError_t e =
            hipModuleLaunchKernel(vk.fn, uint32_t(grid), 1, 1, uint32_t(waves * 64), 1, 1, 0, stream, args, nullptr);
        if (e != hipSuccess) return int(e);
        lease.launched();
        return 0;
    }
    const hipError_t e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(uint32_t(waves * 64)), args, 0, stream);
    if (e != hipSuccess) return int(e);
    lease.launched();
    return 0;
}

}  // namespace

int launch_encode_crc(const MatmulArgs& a, const FusedCrcArgs& c, int device, hipStream_t stream) {
    return launch_fused(a, c, false, device, stream);
}

int launch_decode_verify(const MatmulArgs& a, const FusedCrcArgs& c, int device, hipStream_t stream) {
    return launch_fused(a, c, true, device, stream);
}

}  // namespace hec
