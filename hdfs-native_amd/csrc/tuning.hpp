// tuning.hpp -- launch-shape knobs for measurement (hec_tune_set) and the
// per-device CU count cache.  Host code only.
//
// The knobs are process-wide std::atomic<int>s; every launcher reads one
// consistent snapshot (relaxed loads) at its start, so a concurrent
// hec_tune_set never races with a launch -- it affects launches that start
// after it.  Variants that were measured and rejected (register double
// buffering, output bursts, store cache policies, bank-replicated and
// memory-only CRC schemes) exist only in the HEC_EXPERIMENTAL build
// (lib/libhdfs_ec_amd_exp.so); the default library rejects their keys.
#pragma once

namespace hec {

struct Tune {
    int unroll;             // key 1: 16-B chunks per lane (0 = per-shape default)
    int nt;                 // key 2: non-temporal loads/stores (-1 = default on)
    int blocks_per_cu;      // key 3: grid = blocks_per_cu x CUs (0 = default)
    int block;              // key 4: threads per block (0 = default)
    int pipeline;           // key 5: 0 default, 1 register, 2 LDS-DMA (exp: 3 pipe, 4 burst, 5 double-buffered)
    int drain;              // key 6: store drain per tile in the register kernels (0 default = yes, 1 no, 2 yes)
    int grid;               // key 7: absolute grid size (0 = default)
    int group;              // key 8: stripes per tile-order group (0 = default 4)
    int crc_unfused;        // key 9: 1 = hec_encode_crc_device as encode + checksum passes
    int fused_slabs;        // key 10: fused encode+CRC slabs per wave (0, 4, 8)
    int crc_variant;        // key 11: 0 default (fold, = 7), 1 slicing-by-8, 5 11-bit (exp: 2, 3, 4, 6, 9)
    int crc_prefetch;       // key 12: CRC kernel register prefetch depth (0 = 2, 1, 2)
    int store_pol;          // key 13 (exp): store cache policy of the pipe kernel
    int host_copy_threads;  // key 14: hec_decode_host_batch host copy threads (0 = 4)
    int burst_tiles;        // key 15 (exp): tiles per output burst (2, 3)
    int call_piece_kib;     // key 17: per-call drop-in pipeline piece, KiB per shard (0 = 256)
    int unaligned;          // key 18: unaligned layouts: 0 default = dword kernel + byte tail, 1 = byte kernel only
    int fused_pair;         // key 19: fused kernels at 4 slabs: 0 default / 2 = inputs two at a time, 1 = one at a time
    int mixed_skip;         // key 20: mixed decode rows past a stripe's e: 0 default (skip for k <= 6), 1 compute all, 2 skip
    int fused_split;        // key 21: fused kernels' wave roles: 0 default = 1 = every wave alternates (exp: 2 / 3 role-split GF / CRC waves)
    int fused_wpe;          // key 16: fused kernels' waves per SIMD (0 default = 2; exp: 3, one 768-thread block per CU)
};

// One consistent view of every knob (relaxed atomic loads).
Tune tune_snapshot();

// Validates and stores one knob; returns an HEC_* status.
int tune_store(int key, int value);

// Multiprocessor count of a device (cached per device, thread-safe).
int num_cus(int device);

}  // namespace hec
