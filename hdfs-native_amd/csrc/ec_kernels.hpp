// ec_kernels.hpp -- kernel argument block and launcher for the GF(2^8)
// stripe-cell matrix multiply (see ec_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hec {

constexpr int kBlock = 256;  // threads per block (4 waves)
constexpr int kMaxK = 32;    // inputs per launch (HEC_MAX_DATA_UNITS)
constexpr int kMaxR = 4;     // outputs per launch (more rows are split)

// Passed by value as the kernel argument (kernarg segment, ~800 B).
struct MatmulArgs {
    const uint8_t* in[kMaxK];
    uint64_t in_stride[kMaxK];  // bytes between stripes for input i
    uint8_t* out[kMaxR];
    uint64_t out_stride[kMaxR];
    uint8_t coef[kMaxR * kMaxK];  // row j, column i at [j*kMaxK + i]
    int32_t k;                    // inputs used
    int32_t r;                    // outputs used (1..kMaxR)
    uint64_t cell_len;            // bytes per cell
    uint64_t stripes;
    uint64_t byte_begin;          // byte kernel: first byte handled
    uint32_t chunks;              // vec kernel: 16-B chunks per cell
    uint32_t tiles_per_stripe;
    uint32_t total_tiles;
    uint32_t group;               // tile order: G stripes column-interleaved (1 = stripe-major)
    uint32_t xcd_remap;           // register kernel: 1 = the 8 XCDs' blocks take contiguous tile runs
};

// One coefficient's v_perm_b32 product tables (see ec_kernels.hip): c*x =
// perm(t0hi,t0lo,x&7) ^ perm(t1hi,t1lo,(x>>3)&7) ^ perm(t2,t2,x>>6), 32 B.
struct PermTable {
    uint32_t t0lo, t0hi, t1lo, t1hi, t2, pad0, pad1, pad2;
};

// ---- heterogeneous per-stripe erasure patterns ---------------------------
constexpr int kMaxShards = kMaxK + 16;  // k + m <= 48

// Plan blob entry (device workspace): header, then e x k PermTables.
struct DevPlanHeader {
    uint32_t e;              // missing data shards
    uint8_t surv[kMaxK];     // survivor shard indices (first k present)
    uint8_t miss[16];        // missing data indices, ascending
    uint8_t pad[12];
};
static_assert(sizeof(DevPlanHeader) == 64, "plan header is 64 B");

struct MixedArgs {
    const uint8_t* base[kMaxShards];  // all k+m shard bases
    uint64_t stride[kMaxShards];
    uint8_t* out[kMaxK];              // reconstructed data shard i -> out[i]
    uint64_t out_stride[kMaxK];
    const uint8_t* plans;             // blob: plan p at plans + plan_off[p]
    uint32_t blob_bytes;              // size of the blob (LDS-resident when <= 64 KiB)
    const uint32_t* plan_off;
    const uint16_t* stripe_plan;      // per stripe; 0xFFFF = nothing missing
    int32_t k;
    int32_t row0;                     // first missing row handled by this launch
    uint64_t cell_len;
    uint64_t stripes;
    uint32_t chunks, tiles_per_stripe, total_tiles, group;
};

// Mixed-pattern decode of one group of missing rows row0 .. row0+rows-1
// (rows <= kMaxR).  Requires k in {2,3,6,10}, 16-B aligned bases/strides
// and cell_len % 16 == 0.  0 ok, -1 unsupported, >0 hipError_t.
int launch_decode_mixed(const MixedArgs& a, int rows, int device, hipStream_t stream);

// Launches the multiply for one group of <= kMaxR output rows.  0 on
// success, -1 invalid sizes, otherwise the (positive) hipError_t.
int launch_gf_matmul(const MatmulArgs& a, int device, hipStream_t stream);

// Tuning knobs (set through hec_tune_set).
extern int g_tune_unroll;         // 0 = default, else 1|2|4
extern int g_tune_nt;             // -1 = default, else 0|1
extern int g_tune_blocks_per_cu;  // 0 = default
extern int g_tune_block;          // 0 = default, else 256|512
extern int g_tune_pipeline;       // 0 = default, 1 = register kernel, 2 = LDS-DMA kernel
extern int g_tune_map;            // 0 = default, 1|2 = chunk mapping 0|1
extern int g_tune_grid;           // 0 = default, else absolute grid size
extern int g_tune_group;          // 0 = default, else stripes per tile-order group
extern int g_tune_crc_unfused;    // 1 = encode + separate CRC pass
extern int g_tune_crc_variant;    // 0 = default, 1 = slice-by-8, 2/3 = bank-replicated slice-by-1, 4/8 chains
extern int g_tune_crc_prefetch;   // 0 = default, 1 / 2 tasks of register prefetch (CRC kernel)
extern int g_tune_fused_slabs;    // 0 = default, else 4 / 8 slabs per wave (fused encode+CRC)
extern int g_tune_xcd_remap;           // 1 = XCD-contiguous block -> tile mapping (register kernel)
extern int g_tune_burst_tiles;          // output-burst kernel (key 5 = 4): tiles per burst, 2 or 3
extern int g_tune_host_copy_threads;  // 0 = default (4): hec_decode_host_batch's host copy threads
extern int g_tune_store_pol;      // 0 = nt stores, 1..4 = sc1 | sc0 sc1 | nt sc1 | plain (pipelined kernel)

}  // namespace hec
