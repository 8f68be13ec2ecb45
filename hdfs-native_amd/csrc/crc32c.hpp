// crc32c.hpp -- CRC32C-per-chunk kernel arguments (see crc32c.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hec {

constexpr int kCrcMaxShards = 48;

struct CrcArgs {
    const uint8_t* base[kCrcMaxShards];  // shard i of stripe s at base[i] + s*stride[i]
    uint64_t stride[kCrcMaxShards];
    uint8_t* out;                        // big-endian u32 per chunk: [stripe][shard][chunk]
    uint32_t n_shards;
    uint64_t cell_len;
    uint64_t stripes;
    uint64_t bytes_per_checksum;
    uint64_t chunks_per_cell;  // filled by the launcher
    uint64_t groups_per_cell;  // filled by the launcher (fast path)
};

// 0 ok, -1 invalid sizes, >0 hipError_t.
int launch_crc32c(const CrcArgs& a, int device, hipStream_t stream);

struct MatmulArgs;
// Fused encode + CRC32C of all k inputs and r outputs per 512-B chunk (sums
// [stripe][k+r][nchunks] big-endian).  Needs k in {2,3,6,10}, r <= 4,
// 16-B aligned layout and cell_len % 16 == 0; returns -1 otherwise.
int launch_encode_crc(const MatmulArgs& a, uint8_t* sums, int device, hipStream_t stream);

}  // namespace hec
