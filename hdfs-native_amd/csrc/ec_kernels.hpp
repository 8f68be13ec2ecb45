// ec_kernels.hpp -- kernel argument block and launcher for the GF(2^8)
// stripe-cell matrix multiply (see ec_kernels.hip).
#pragma once

#ifndef __HIPCC_RTC__  // hiprtc (jit.cpp) provides the HIP runtime itself
#include <hip/hip_runtime.h>
#else
typedef struct ihipStream_t* hipStream_t;  // the launchers below are host code: declarations only
#endif

#include <cstdint>

#include "tuning.hpp"

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
    uint32_t grouped_tiles;       // tiles of the whole G-stripe groups; the remainder stripes go stripe-major
    uint32_t drain;               // register kernel: 1 = wait for the tile's stores before the next tile's loads
    uint32_t col_rot = 0;         // tile order: stripe s starts its columns at (s * col_rot) % tiles (0 = none)
    uint32_t* queue = nullptr;       // work-queue kernels: this launch's counters (zero when it starts)
    uint32_t* queue_zero = nullptr;  // the set this launch zeroes for the stream's next launch (nullptr: none)
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

constexpr uint32_t kNoPlan = 0xFFFFFFFFu;  // stripe with no missing data shard

// Workspace (device): [per-stripe plan offset: u32 x stripes][plan blob]
// [kMixedQueueBytes: zeroed tile counters, kMixedQueues per launch, one per
// kMixedQueueStride bytes];
// plan = DevPlanHeader + e x k PermTables (row r, input i at r*k + i).
constexpr uint32_t kMixedQueues = 8, kMixedQueueStride = 256;
constexpr size_t kMixedQueueBytes = size_t(16) * kMixedQueues * kMixedQueueStride;  // up to 16 launches (64 rows)
struct MixedArgs {
    const uint8_t* base[kMaxShards];  // all k+m shard bases
    uint64_t stride[kMaxShards];
    uint8_t* out[kMaxK];              // reconstructed data shard i -> out[i]
    uint64_t out_stride[kMaxK];
    const uint8_t* plans;             // blob: plan of stripe s at plans + stripe_off[s]
    const uint32_t* stripe_off;       // per stripe; kNoPlan = nothing missing
    uint32_t blob_bytes;              // size of the blob
    int32_t k;
    int32_t row0;                     // first missing row handled by this launch
    uint64_t cell_len;
    uint64_t stripes;
    uint32_t chunks, tiles_per_stripe, total_tiles, group, grouped_tiles;
    uint32_t drain;                   // 1 = wait for a tile's stores before the next tile (tune key 6)
    uint32_t* queue;                  // this launch's zeroed tile counters (work-queue variant, key 26)
};

#ifndef __HIPCC_RTC__
// The work-queue counter sets of one launch (ec_kernels.hip, DESIGN.md §3.1
// "Counter sets").  A direct launch takes its stream's current set (`use`,
// zero) and zeroes the stream's other set (`zero`) for the next launch; the
// stream is held (its sets' lock) from queue_lease() until the lease ends, so
// launches from several threads on one stream still alternate in their
// stream order.  A launch into a stream that is being captured gets a set of
// its own (the graph keeps it for good) zeroed by a memset node captured
// just before the kernel; `zero` is then nullptr.  An empty lease (use ==
// nullptr) means: launch the fixed-order kernel.
struct QueueLease {
    uint32_t* use = nullptr;
    uint32_t* zero = nullptr;
    QueueLease() = default;
    QueueLease(QueueLease&& o) noexcept;
    QueueLease& operator=(QueueLease&& o) noexcept;
    QueueLease(const QueueLease&) = delete;
    QueueLease& operator=(const QueueLease&) = delete;
    ~QueueLease();
    explicit operator bool() const { return use != nullptr; }
    // The kernel was enqueued: the stream's next launch takes `zero`.  A lease
    // whose kernel was not enqueued leaves the stream on `use` (still zero).
    void launched();
    void* st_ = nullptr;  // the stream's sets (held while the lease lives)
};
QueueLease queue_lease(int device, hipStream_t stream);
// Allocates the device's pool of graph-capture sets, outside any capture
// (hec_coder_create calls it); a capture with no set left launches the
// fixed-order kernels.
void queue_reserve(int device);
// Counter sets in use on a device: {direct streams, graph sets handed out}.
void queue_stats(int device, uint64_t* streams, uint64_t* graph_sets);
// 1 when streams are told apart by hipStreamGetId, 0 when by handle.
int queue_keyed_by_id();
#endif

// Mixed-pattern decode of one group of missing rows row0 .. row0+rows-1
// (rows <= kMaxR).  Requires k in {2,3,6,10}, 16-B aligned bases/strides
// and cell_len % 16 == 0.  0 ok, -1 unsupported, >0 hipError_t.
int launch_decode_mixed(const MixedArgs& a, int rows, int device, hipStream_t stream);

// True when the launch's coefficients are the RS coding matrix's parity rows
// (gen_rs_matrix, gf256.rs:40-57) for its (k, r): the encode kernels then
// run the bit-sliced XOR networks of xor_networks.hpp.
bool rs_parity_matrix(const MatmulArgs& a);

// Launches the multiply for one group of <= kMaxR output rows.  0 on
// success, -1 invalid sizes, otherwise the (positive) hipError_t.
int launch_gf_matmul(const MatmulArgs& a, int device, hipStream_t stream);


}  // namespace hec
