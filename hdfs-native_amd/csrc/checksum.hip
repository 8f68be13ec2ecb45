// checksum.hip -- per-chunk checksums on gfx950.
//
// Reference: every DataTransferProtocol packet carries one checksum per
// bytes_per_checksum chunk of its data: CRC32C on write
// (WritePacket::calculate_checksum, rust/src/hdfs/connection.rs:568-584),
// CRC32C or CRC32 verified on read (ReadPacket::get_data, :477-504; a
// mismatch is HdfsError::ChecksumError).  CRC32C = crc 3.4 CRC_32_ISCSI,
// CRC32 = CRC_32_CKSUM (connection.rs:37-38; parameters in
// checksum_tables.hpp); sums are big-endian (put_u32 / get_u32).  Shards
// are written as whole cells, so the chunks of a cell are exactly the
// chunks of its block stream.  Compute mode writes the sums; verify mode
// compares them with the expected sums and flags the cell.
//
// Fast kernel (512-B chunks): a wave owns 16 consecutive chunks (8 KiB) of
// one cell ("task") and each lane a QUARTER chunk (128 B):
//  1. the task's 8 coalesced 16-B-per-lane loads were issued PF tasks ago
//     into registers; they are written to a wave-private LDS image
//     [quarter][128 + 16 B pad] (the pad makes both the ds_write_b128 fill
//     and the per-lane ds_read_b128 walk bank-conflict free) and the
//     registers are refilled with the loads of task + PF;
//  2. each lane computes the linear CRC of its 128 B from state 0 with one
//     of two lookup SCHEMEs (below), moves it to its place in the chunk with
//     an "append 384/256/128 zero bytes" byte table (CRC is linear over
//     GF(2)), two XOR shuffles combine the 4 quarters and the init/xorout
//     constant of a 512-B chunk is folded in.
// SCHEME 1 (default): slicing-by-8 from 8 KiB of tables, 256-thread blocks,
//   2 per CU.  Random table indices hit the 32 banks of a ds_read_b32
//   half-wave ~3-4 ways deep (PMC: LDS array 85 % busy, 60 % of it conflict
//   cycles).
// SCHEME 4 / 8: slicing-by-1 from a table REPLICATED across the 32 banks
//   (lane l reads column l%32: conflict free), the quarter as 4 / 8
//   independent segment chains (latency) combined with "append 16*j zero
//   bytes" tables; 72 KiB of tables, 512-thread blocks, 1 per CU.  Halves
//   the LDS-array cycles but not the time: with 2 waves per SIMD the byte
//   chain's latency, not LDS throughput, sets the pace (all schemes measure
//   4.6-4.9 TB/s against 6.4 for the kernel's loads alone).
// No cross-wave traffic and no block barrier after the table prologue.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "checksum.hpp"
#include "checksum_device.hpp"
#include "checksum_tables.hpp"
#include "ec_kernels.hpp"
#include "work_queue.hpp"

namespace hec {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t v4u_ __attribute__((ext_vector_type(4)));

constexpr int kCrcBlock = 256;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__constant__ crc::Tables<crc::kCrc32c> kTablesCrc32c = crc::Tables<crc::kCrc32c>();
__constant__ crc::Tables<crc::kCksum> kTablesCksum = crc::Tables<crc::kCksum>();

template <int KIND>
__device__ __forceinline__ const crc::Tables<KIND>& tables() {
    if constexpr (KIND == crc::kCrc32c)
        return kTablesCrc32c;
    else
        return kTablesCksum;
}

// Compute mode: store the big-endian sum.  Verify mode: flag the cell on a
// mismatch (every flagging lane stores the same byte).
__device__ __forceinline__ void emit_sum(const CrcArgs& a, uint64_t cell_idx, uint64_t chunk, uint32_t crc) {
    uint64_t cell = cell_idx;
    if (a.mapped) {  // launch cells are a subset of the sums layout
        const uint64_t s = cell_idx / a.n_shards;
        const uint64_t stripe = a.stripe_list ? a.stripe_list[s] : s;
        cell = stripe * a.n_total + a.sid[cell_idx - s * a.n_shards];
    }
    const uint64_t at = cell * a.chunks_per_cell + chunk;
    if (a.expected) {
        if (reinterpret_cast<const uint32_t*>(a.expected)[at] != bswap32(crc)) a.bad[cell] = 1;
    } else if (a.sums_nt) {
        __builtin_nontemporal_store(bswap32(crc), reinterpret_cast<uint32_t*>(a.out) + at);
    } else {
        reinterpret_cast<uint32_t*>(a.out)[at] = bswap32(crc);
    }
}

// One wave's task: 16 chunks (8 KiB) of one cell, 8 coalesced 1-KiB loads.
// `task` is wave-uniform (scalar base/stride loads); the loads are
// unconditional with dead lanes clamped to the cell start -- a conditional
// load with a zero default makes hipcc copy the result out of the load's
// registers behind an s_waitcnt vmcnt(0), which serialises the prefetch.
// Dead lanes' bytes are never checksummed.
__device__ __forceinline__ void load_task(const CrcArgs& a, uint64_t groups, uint64_t task, int lane, u32x4 (&v)[8]) {
    const uint64_t cell_idx = task / groups;
    const uint64_t g = task - cell_idx * groups;
    const uint64_t s = cell_idx / a.n_shards;
    const uint32_t shard = uint32_t(cell_idx - s * a.n_shards);
    const uint64_t stripe = a.stripe_list ? a.stripe_list[s] : s;
    const uint8_t* base = a.base[shard] + stripe * a.stride[shard] + g * 16u * 512u;
    const uint64_t left = a.cell_len - g * 16u * 512u;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t off = uint32_t(t) * 1024u + uint32_t(lane) * 16u;
        v[t] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (off < left ? off : 0u)));
    }
}

template <int SCHEME>
struct CrcShape : crcdev::TableLayout<SCHEME> {
    static constexpr int kBlock = SCHEME == 16 ? 1024 : (SCHEME <= 1 || crcdev::w11(SCHEME)) ? 256 : 512;
    static constexpr int kWaves = kBlock / 64;
};

// WQ > 0 (PF = 1 only): tasks come from the work queue of wave-tiles
// (work_queue.hpp, a.queue) in units of WQ consecutive tasks of one cell,
// one unit per atomic; the next task is still loaded during this one.
// BLK > 0 (measurement, tune key 33): BLK-thread blocks instead of the
// scheme's; 768 = one block per CU with the tables staged once for 12 waves
// (3 per SIMD, 149.5 KiB of LDS), 50 % more tasks in flight than two
// 256-thread blocks.
template <int KIND, int SCHEME, int PF, int WQ = 0, int BLK = 0>
__global__ __launch_bounds__(BLK ? BLK : CrcShape<SCHEME>::kBlock) void checksum_chunks512(CrcArgs a) {
    static_assert(WQ == 0 || PF == 1, "the queue (and the runs, WQ < 0) run one task of prefetch");
    using Sh = CrcShape<SCHEME>;
    using Spec = crc::Spec<KIND>;
    constexpr bool REFL = Spec::kReflected;
    constexpr int CH = 512, Q = CH / 4, PITCH = Q + 16, STAGE = 64 * PITCH, BS = BLK ? BLK : Sh::kBlock;
    constexpr int WAVES = BS / 64;
    __shared__ uint32_t s_tables[Sh::kWords];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[WAVES * STAGE];
    uint32_t* s_main = s_tables;
    crcdev::stage_tables<SCHEME, BS>(s_tables, tables<KIND>());
    __syncthreads();
    const uint32_t kfinal = tables<KIND>().final512;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x & 63;
    const int qi = lane & 3, c = lane >> 2;  // quarter, chunk within the task
    uint8_t* stage = s_stage + wave * STAGE;
    const uint64_t groups = a.groups_per_cell;
    const uint64_t tasks = groups * a.n_shards * a.stripes;
    const uint64_t step = uint64_t(gridDim.x) * WAVES;

    // stage v (task's data), refill v with task `next`'s loads, checksum
    auto run_task = [&](uint64_t task, u32x4 (&v)[8], uint64_t next) {
        const uint64_t cell_idx = task / groups;
        const uint64_t g = task - cell_idx * groups;
        const uint64_t start = g * 16u * CH;
#pragma unroll
        for (int t = 0; t < 8; t++) {
            const uint32_t off = uint32_t(t) * 1024u + uint32_t(lane) * 16u;
            *reinterpret_cast<u32x4*>(stage + (off / Q) * PITCH + (off % Q)) = v[t];
        }
        if (next < tasks) load_task(a, groups, next, lane, v);
        // lanes read what other lanes of the SAME wave wrote: a wave's LDS ops
        // complete in order; only the compiler must not hoist the reads
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");

        const uint64_t cstart = start + uint64_t(c) * CH;
        const bool live = cstart < a.cell_len;
        const bool full = live && a.cell_len - cstart >= uint64_t(CH);  // same for the chunk's 4 lanes
        uint32_t val = 0;
        if constexpr (SCHEME == 0) {
            // measurement only: the task's loads + staging, no CRC math
            val = *reinterpret_cast<const uint32_t*>(stage + lane * PITCH);
        } else if (full) {
            uint32_t r = crcdev::quarter<SCHEME, REFL>(s_main, stage + lane * PITCH, lane);
            if (qi < 3) r = crcdev::shift_quarter<SCHEME>(s_tables, qi, r);
            val = r;
        } else if (live && qi == 0) {
            // short last chunk of the cell: this lane walks it whole, bytewise
            const uint32_t len = uint32_t(a.cell_len - cstart);
            uint32_t r = Spec::kInit;
            for (uint32_t p = 0; p < len; p++)
                r = crcdev::byte_step<REFL, crcdev::ByteTable<SCHEME>::stride, crcdev::ByteTable<SCHEME>::bswap>(
                    s_main + crcdev::ByteTable<SCHEME>::off, r,
                                                                              stage[(4 * c + p / Q) * PITCH + (p % Q)]);
            val = r ^ Spec::kXorout;
        }
        val ^= __shfl_xor(val, 1);
        val ^= __shfl_xor(val, 2);
        if (live && qi == 0) emit_sum(a, cell_idx, g * 16u + c, full ? (val ^ kfinal) : val);
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
    };

    if constexpr (WQ > 0) {
        // units of WQ tasks; the launcher keeps the unit count below 2^32
        const uint32_t units = uint32_t((tasks + WQ - 1) / WQ);
        queue_zero_next(a.queue_zero);
        WaveQueue q;
        q.init(a.queue, units);
        auto task_of = [&](uint32_t u) { return u < units ? uint64_t(u) * WQ : tasks; };
        uint64_t task = task_of(q.next());
        u32x4 v[8];
        if (task < tasks) load_task(a, groups, task, lane, v);
        while (task < tasks) {
            const bool unit_end = (task % WQ) == WQ - 1 || task + 1 >= tasks;
            run_task(task, v, unit_end ? task_of(q.peek()) : task + 1);
            task = unit_end ? task_of(q.next()) : task + 1;
        }
        return;
    }
    if constexpr (WQ < 0) {
        // measurement (tune key 31): fixed order in runs of -WQ consecutive
        // tasks of one cell per wave, so a wave writes whole lines of sums
        constexpr uint64_t SEQ = uint64_t(-WQ);
        const uint64_t wstep = SEQ * step;
        uint64_t task = (uint64_t(blockIdx.x) * WAVES + wave) * SEQ;
        auto next_of = [&](uint64_t t) { return (t % SEQ) != SEQ - 1 ? t + 1 : t - (SEQ - 1) + wstep; };
        u32x4 v[8];
        if (task < tasks) load_task(a, groups, task, lane, v);
        while (task < tasks) {
            const uint64_t nt = next_of(task);
            run_task(task, v, nt);
            task = nt;
        }
        return;
    }
    // PF register sets in flight: task t's loads are issued while task t-PF
    // is checksummed
    uint64_t task = uint64_t(blockIdx.x) * WAVES + wave;
    u32x4 va[8], vb[8];
    if (task < tasks) load_task(a, groups, task, lane, va);
    if (PF == 2 && task + step < tasks) load_task(a, groups, task + step, lane, vb);
    while (task < tasks) {
        run_task(task, va, task + PF * step);
        task += step;
        if constexpr (PF == 2) {
            if (task >= tasks) break;
            run_task(task, vb, task + 2 * step);
            task += step;
        }
    }
}

// The LDS-DMA CRC kernel (tasks landed in LDS by global_load_lds_dwordx4,
// key 11 = 13; round 5) lost 4-14 % on the bench's buffers
// (profiles/r05n) and was removed in round 6; scripts/probe_crc_dma.hip keeps
// its standalone probe form.

// Generic path: any chunk size / alignment.  One lane per chunk, bytes from
// global memory, slice-by-1.
template <int KIND>
__global__ __launch_bounds__(kCrcBlock) void checksum_chunks_bytes(CrcArgs a) {
    using Spec = crc::Spec<KIND>;
    __shared__ uint32_t s_tab[256];
    for (int t = threadIdx.x; t < 256; t += kCrcBlock) s_tab[t] = tables<KIND>().slice[0][t];
    __syncthreads();
    const uint64_t total = a.chunks_per_cell * a.n_shards * a.stripes;
    for (uint64_t gidx = uint64_t(blockIdx.x) * kCrcBlock + threadIdx.x; gidx < total;
         gidx += uint64_t(gridDim.x) * kCrcBlock) {
        const uint64_t cell_idx = gidx / a.chunks_per_cell;
        const uint64_t chunk = gidx - cell_idx * a.chunks_per_cell;
        const uint64_t s = cell_idx / a.n_shards;
        const uint32_t shard = uint32_t(cell_idx - s * a.n_shards);
        const uint64_t stripe = a.stripe_list ? a.stripe_list[s] : s;
        const uint8_t* p = a.base[shard] + stripe * a.stride[shard] + chunk * a.bytes_per_checksum;
        const uint64_t cs = chunk * a.bytes_per_checksum;
        const uint64_t len = a.cell_len - cs < a.bytes_per_checksum ? a.cell_len - cs : a.bytes_per_checksum;
        uint32_t crc = Spec::kInit;
        for (uint64_t i = 0; i < len; i++) crc = crcdev::byte_step<Spec::kReflected, 1>(s_tab, crc, p[i]);
        emit_sum(a, cell_idx, chunk, crc ^ Spec::kXorout);
    }
}

template <int KIND, int SCHEME>
const void* crc_fn(int pf) {
    return pf == 2 ? reinterpret_cast<const void*>(&checksum_chunks512<KIND, SCHEME, 2>)
                   : reinterpret_cast<const void*>(&checksum_chunks512<KIND, SCHEME, 1>);
}

template <int KIND>
const void* crc_pick(int scheme, int pf) {
#ifdef HEC_EXPERIMENTAL
    // rejected schemes (profiles/r01_probe_crc.log, r01d_probe_crc_1024.log):
    // bank-replicated slicing-by-1 with 4 / 8 chains, slicing-by-8 at 4 waves
    // per SIMD, and the memory side alone (scheme 0: WRONG sums)
    if (scheme == 16) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 16, 1>);
    if (scheme == 4) return crc_fn<KIND, 4>(pf);
    if (scheme == 8) return crc_fn<KIND, 8>(pf);
    if (scheme == 0) return crc_fn<KIND, 0>(pf);
    // bank-replicated slicing-by-2, 4 chains: 5.14 vs 5.37 TB/s
    // (profiles/r02_probe_crc_rep2.log)
    if (scheme == 22) return crc_fn<KIND, 22>(pf);
    // fold depth 16 / 20 dwords (CRC32C; the MSB-first kind has no fold)
    if (scheme == 13 || scheme == 14) {
        if constexpr (KIND == crc::kCrc32c) return scheme == 13 ? crc_fn<KIND, 13>(pf) : crc_fn<KIND, 14>(pf);
        return crc_fn<KIND, 12>(pf);
    }
#endif
#ifdef HEC_EXPERIMENTAL
    // the fold with the work queue (tune key 29 = 1 / 2 / 4 / 8 / 16 tasks per unit)
    if (scheme == 12 && pf < 0) {
        if constexpr (KIND == crc::kCrc32c) {
            if (pf == -1) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, 1>);
            if (pf == -2) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, 2>);
            if (pf == -4) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, 4>);
            if (pf == -8) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, 8>);
            if (pf == -16) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, 16>);
            if (pf == -102) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, -2>);
            if (pf == -104) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, -4>);
            if (pf == -108) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, -8>);
            if (pf == -116) return reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1, -16>);
        }
        return nullptr;
    }
#endif
#ifndef HEC_EXPERIMENTAL
    // product: the fold (CRC32C, one task of prefetch) / 11-bit slicing inside
    // scheme 12 (CRC32, two tasks)
    (void)scheme;
    (void)pf;
    return KIND == crc::kCrc32c ? reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 1>)
                                : reinterpret_cast<const void*>(&checksum_chunks512<KIND, 12, 2>);
#else
    if (scheme == 12) return crc_fn<KIND, 12>(pf);
    return scheme == 1 ? crc_fn<KIND, 1>(pf) : crc_fn<KIND, 11>(pf);
#endif
}

}  // namespace

int launch_checksum(const CrcArgs& in, int device, hipStream_t stream) {
    CrcArgs a = in;
    if (a.bytes_per_checksum == 0 || a.cell_len == 0 || a.n_shards == 0) return -1;
    if (a.kind != crc::kCrc32c && a.kind != crc::kCksum) return -1;
    if (a.expected && !a.bad) return -1;
    // sums are read / written as u32 by every path (fast and byte kernels)
    if ((reinterpret_cast<uintptr_t>(a.out) | reinterpret_cast<uintptr_t>(a.expected)) & 3u) return -1;
    if (a.n_shards > uint32_t(kCrcMaxShards) || a.n_total < a.n_shards) return -1;
    a.mapped = a.n_total != a.n_shards || a.stripe_list != nullptr;
    for (uint32_t i = 0; i < a.n_shards; i++) {
        if (a.sid[i] >= a.n_total) return -1;
        a.mapped |= a.sid[i] != i;
    }
    a.chunks_per_cell = (a.cell_len + a.bytes_per_checksum - 1) / a.bytes_per_checksum;
    if (a.stripes == 0) return 0;
    bool aligned = a.cell_len % 16 == 0;
    for (uint32_t i = 0; i < a.n_shards; i++)
        aligned &= ((reinterpret_cast<uintptr_t>(a.base[i]) | a.stride[i]) & 15u) == 0;
    const int cus = num_cus(device);
    const Tune tn = tune_snapshot();
    a.sums_nt = tn.crc_sums_nt == 1 ? 1u : 0u;  // measurement (key 30)
    void* args[] = {&a};
    hipError_t e;
    QueueLease lease;  // work-queue counters (held until the launch is enqueued)
    if (aligned && a.bytes_per_checksum == 512) {
        a.groups_per_cell = (a.chunks_per_cell + 15) / 16;
        const uint64_t tasks = a.groups_per_cell * a.n_shards * a.stripes;
        // 11-bit slicing (6 LDS lookups per 8 bytes), 2 tasks of prefetch,
        // was the default until the fold.  Interleaved A/B (profiles/r01d_probe_crc_w11.log): 5.32
        // TB/s vs 4.84-4.89 for slicing-by-8 (profiles/r01_probe_crc.log: 4.91
        // vs 4.80 replicated, 4 chains, and 4.64, 8 chains; 4.64 for
        // slicing-by-8 at 4 waves per SIMD, r01d_probe_crc_1024.log); the
        // memory side alone reaches 6.4.
        // default since round 2 (session k): the fold (scheme 12, CRC32C; the
        // MSB-first kind runs 11-bit slicing inside it) with one task of
        // prefetch: same box, 9 x 1 MiB x 1024, 1.598 ms (6.05 TB/s) vs 1.804
        // (5.36) for 11-bit slicing at its best prefetch
        // (profiles/r02k_fold/probe_crc.log); 11-bit slicing on key 11 = 5
        const int scheme = tn.crc_variant == 10  ? 13
                           : tn.crc_variant == 11 ? 14
                           : tn.crc_variant == 1   ? 1
                           : tn.crc_variant == 2 ? 4
                           : tn.crc_variant == 3 ? 8
                           : tn.crc_variant == 4 ? 16
                           : tn.crc_variant == 9 ? 0
                           : tn.crc_variant == 6 ? 22
                           : tn.crc_variant == 5 ? 11
                                                 : 12;
        // prefetch depth: key 12 (0 = the scheme's default: 1 for the CRC32C
        // fold, 2 otherwise -- the MSB-first CRC32 kind has no fold and runs
        // 11-bit slicing inside scheme 12, whose best depth is 2)
        const int pf = tn.crc_prefetch == 1   ? 1
                       : tn.crc_prefetch == 2 ? 2
                       : (scheme == 12 && a.kind == crc::kCrc32c) ? 1
                                                                    : 2;
        // scheme 16: always 1 (128 VGPRs at 4 waves/SIMD)
        const int waves = scheme == 16 ? CrcShape<16>::kWaves : crcdev::sliced(scheme) ? CrcShape<1>::kWaves : CrcShape<4>::kWaves;
        const int per_cu = (crcdev::sliced(scheme) && scheme != 16) ? 2 : 1;  // LDS: 56 / 77.5 KiB; ~144 / ~154 KiB
        uint64_t grid = (tasks + waves - 1) / waves;
        const uint64_t cap = tn.grid ? uint64_t(tn.grid) : uint64_t(cus) * per_cu;
        if (grid > cap) grid = cap;
        const void* fn = a.kind == crc::kCrc32c ? crc_pick<crc::kCrc32c>(scheme, pf) : crc_pick<crc::kCksum>(scheme, pf);
#ifdef HEC_EXPERIMENTAL
        // tune key 33 = 768: the fold kernel (CRC32C, one task of prefetch) in
        // one 768-thread block per CU, 3 waves per SIMD
        if (tn.crc_block == 768 && scheme == 12 && a.kind == crc::kCrc32c && pf == 1 && !tn.crc_runs && !tn.crc_wq) {
            fn = reinterpret_cast<const void*>(&checksum_chunks512<crc::kCrc32c, 12, 1, 0, 768>);
            const uint64_t g = (tasks + 11) / 12;
            grid = g < uint64_t(cus) ? g : uint64_t(cus);
            e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(768), args, 0, stream);
            return e == hipSuccess ? 0 : int(e);
        }
        // tune key 31: the fold kernel in runs of 2 / 4 consecutive tasks per wave
        if (tn.crc_runs && scheme == 12 && a.kind == crc::kCrc32c && pf == 1) {
            const void* f = crc_pick<crc::kCrc32c>(12, -100 - tn.crc_runs);
            if (f) fn = f;
        }
        // tune key 29: the fold kernel with the work queue, 1 / 2 / 4 tasks per
        // unit, the resident blocks only
        if (tn.crc_wq && scheme == 12 && a.kind == crc::kCrc32c && pf == 1 &&
            (tasks + uint64_t(tn.crc_wq) - 1) / uint64_t(tn.crc_wq) < (uint64_t(1) << 32)) {
            const void* f = crc_pick<crc::kCrc32c>(12, -tn.crc_wq);
            if (f) lease = queue_lease(device, stream);
            a.queue = lease.use;
            a.queue_zero = lease.zero;
            if (a.queue) {
                fn = f;
                grid = uint64_t(cus) * per_cu;
                const uint64_t units = (tasks + uint64_t(tn.crc_wq) - 1) / uint64_t(tn.crc_wq);
                if (grid > units) grid = units;
            }
        }
#endif
        e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(uint32_t(waves * 64)), args, 0, stream);
        if (e == hipSuccess) lease.launched();
    } else {
        const uint64_t total = a.chunks_per_cell * a.n_shards * a.stripes;
        uint64_t grid = (total + kCrcBlock - 1) / kCrcBlock;
        if (grid > uint64_t(cus) * 4) grid = uint64_t(cus) * 4;
        const void* fn = a.kind == crc::kCrc32c ? reinterpret_cast<const void*>(&checksum_chunks_bytes<crc::kCrc32c>)
                                                : reinterpret_cast<const void*>(&checksum_chunks_bytes<crc::kCksum>);
        e = hipLaunchKernel(fn, dim3(uint32_t(grid)), dim3(kCrcBlock), args, 0, stream);
    }
    return e == hipSuccess ? 0 : int(e);
}

}  // namespace hec
