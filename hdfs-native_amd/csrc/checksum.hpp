// checksum.hpp -- chunk-checksum kernel arguments (see checksum.hip).
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (jit.cpp) provides the HIP runtime itself
#include <hip/hip_runtime.h>
#else
typedef struct ihipStream_t* hipStream_t;  // the launchers below are host code: declarations only
#endif

#include <cstdint>

namespace hec {

constexpr int kCrcMaxShards = 48;

struct CrcArgs {
    const uint8_t* base[kCrcMaxShards];  // shard i of stripe s at base[i] + s*stride[i]
    uint64_t stride[kCrcMaxShards];
    // Cell (stripe s, launch shard i) has index s * n_total + sid[i] in the
    // sums and flag layouts ([stripe][n_total][chunk]; identity: sid[i] = i,
    // n_total = n_shards).  Compute mode (expected == nullptr): big-endian
    // u32 per chunk to out.  Verify mode: compare against expected and set
    // bad[cell] = 1 on any mismatch in that cell (ReadPacket::get_data,
    // connection.rs:477-504); out unused.
    uint8_t sid[kCrcMaxShards];
    // optional: launch stripe s is batch stripe stripe_list[s] (addresses,
    // sums and flags); null = identity.  `stripes` counts the list.
    const uint32_t* stripe_list;
    uint32_t n_total;
    uint32_t mapped;  // filled by the launcher: sid is not the identity
    uint8_t* out;
    const uint8_t* expected;
    uint8_t* bad;
    int32_t kind;  // crc::Kind: 0 = CRC32C, 1 = CRC32 (CRC_32_CKSUM)
    uint32_t n_shards;
    uint64_t cell_len;
    uint64_t stripes;
    uint64_t bytes_per_checksum;
    uint64_t chunks_per_cell;  // filled by the launcher
    uint64_t groups_per_cell;  // filled by the launcher (fast path)
    uint32_t* queue;           // work-queue variant: this launch's counters (zero when it starts)
    uint32_t* queue_zero;      // the set this launch zeroes for the stream's next launch (nullptr: none)
    uint32_t sums_nt;          // compute mode: non-temporal sum stores (measurement build, key 30)
};

// 0 ok, -1 invalid sizes, >0 hipError_t.
int launch_checksum(const CrcArgs& a, int device, hipStream_t stream);

struct MatmulArgs;

// Checksum side of the fused coding kernels: which cells are checksummed
// and where their chunk sums go (encode) or come from (verify).
struct FusedCrcArgs {
    uint8_t* sums;            // encode: written, [stripe][n_total][nchunks] big-endian
    const uint8_t* expected;  // verify: read, same layout
    uint8_t* bad;             // verify: bad[stripe * n_total + shard] = 1 on mismatch
    uint32_t n_total;         // shards per stripe in the sums layout (k + m)
    int32_t kind;             // crc::Kind
    uint8_t shard_id[64];     // sums index of launch input i (verify: survivor shard ids) / output K + j
    uint32_t sums_nt;         // encode: non-temporal sum stores (measurement build, key 30)
};

// Fused encode + CRC32C of all k inputs and r outputs per 512-B chunk.
// Needs k in {2,3,6,10}, r <= 4, 16-B aligned layout and cell_len % 16 == 0;
// returns -1 otherwise.
int launch_encode_crc(const MatmulArgs& a, const FusedCrcArgs& c, int device, hipStream_t stream);

// Fused decode + checksum verify of the k survivors (a.in) while the e = a.r
// missing rows are rebuilt (a.out); CRC32C or CRC32, 512-B chunks.  Same
// shape limits as launch_encode_crc (-1 otherwise).
int launch_decode_verify(const MatmulArgs& a, const FusedCrcArgs& c, int device, hipStream_t stream);

}  // namespace hec
