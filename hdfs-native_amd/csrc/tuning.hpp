// tuning.hpp -- launch-shape knobs and the per-device CU count cache.  Host
// code only.
//
// The product library (lib/libhdfs_ec_amd.so) has NO knobs: tune_snapshot()
// returns the defaults below, every launcher picks the measured default
// shape, and only the kernels those defaults use are instantiated.  The
// knobs exist in the HEC_EXPERIMENTAL measurement build
// (lib/libhdfs_ec_amd_exp.so, `make exp`): there they are process-wide
// std::atomic<int>s set through hec_tune_set (include/hdfs_ec_amd_exp.h);
// every launcher reads one consistent snapshot (relaxed loads) at its start,
// so a concurrent hec_tune_set only affects launches that start after it.
// That build also holds some measured-and-rejected variants (bank-replicated
// and memory-only CRC schemes, slicing-by-8, ...); those that lost by more
// than 3 % were removed in round 6 (git keeps them).
#pragma once

namespace hec {

#ifdef HEC_EXPERIMENTAL
constexpr bool kExperimental = true;
#else
constexpr bool kExperimental = false;
#endif

struct Tune {
    int unroll = 0;             // key 1: 16-B chunks per lane (0 = per-shape default)
    int nt = -1;                // key 2: non-temporal loads/stores (-1 = default on)
    int blocks_per_cu = 0;      // key 3: grid = blocks_per_cu x CUs (0 = default)
    int block = 0;              // key 4: threads per block (0 = default)
    int pipeline = 0;           // key 5: 0 default, 1 register, 2 LDS-DMA
    int drain = 0;              // key 6: store drain per tile in the register kernels (0 default = yes, 1 no, 2 yes)
    int grid = 0;               // key 7: absolute grid size (0 = default)
    int group = 0;              // key 8: stripes per tile-order group (0 = default 4)
    int crc_unfused = 0;        // key 9: 1 = hec_encode_crc_device as encode + checksum passes
    int fused_slabs = 0;        // key 10: fused encode+CRC slabs per wave (0, 4, 8)
    int crc_variant = 0;        // key 11: 0 default (the fold), 1 slicing-by-8, 5 11-bit, 12 slicing-by-32 tail, 2/3/4/6/9 rejected schemes
    int crc_prefetch = 0;       // key 12: CRC kernel register prefetch depth (0 = scheme default: 1 for the CRC32C fold, else 2; 1, 2)
    int store_pol = 0;          // key 13: retired (the pipe kernel's store policy, round 6 pruning)
    int host_copy_threads = 0;  // key 14: hec_decode_host_batch host copy threads (0 = 4)
    int burst_tiles = 0;        // key 15: retired (output bursts, round 6 pruning)
    int fused_wpe = 0;          // key 16: fused kernels' waves per SIMD (0 default = 2; 3 = one 768-thread block per CU)
    int call_piece_kib = 0;     // key 17: per-call drop-in pipeline piece, KiB per shard (0 = 256)
    int unaligned = 0;          // key 18: unaligned layouts: 0 default = dword kernel + byte tail, 1 = byte kernel only
    int fused_pair = 0;         // key 19: fused kernels at 4 slabs: 0 default / 2 = inputs two at a time, 1 = one at a time
    int mixed_skip = 0;         // key 20: mixed decode rows past a stripe's e: 0 default = 2 = skip, 1 compute all
    int fused_split = 0;        // key 21: fused kernels' wave roles: 0 / 1 = every wave alternates (role split retired)
    int fused_bsl = 0;          // key 22: fused encode parity: 0 default = bit-sliced for the RS matrix, 1 = v_perm tables
    int matmul_bsl = 0;         // key 23: register / LDS-DMA encode: 0 default = v_perm tables, 1 = bit-sliced RS parity (rejected)
    int col_rot = 0;            // key 25: fused kernels' per-stripe column rotation (tiles per stripe index; 0 = none)
    int jit_pfd = 0;            // key 24: fused load schedule (0 default, 2 = two pairs ahead at 4 slabs, 3 = early issue at 8, 4 = sums per tile, 5 = early outputs)
    int matmul_wq = 0;          // key 27: register kernel's work queue of wave-tiles (0 = default: 2 rounds per atomic for k <= 3, 1 for k = 6, 10; 1 / 2 forced; 3 = the fixed tile order)
    int fused_wq = 0;           // key 28: fused kernels' work queue (0 = default: encode + CRC at k = 3, 10, decode + verify at every k; 1 = everywhere; 2 = block tiles)
    int crc_wq = 0;             // key 29: CRC32C checksum kernel with the work queue (0 = off; 1 / 2 / 4 / 8 / 16 tasks per unit)
    int crc_sums_nt = 0;        // key 30: 1 = the CRC kernels store the sums non-temporal (measurement)
    int crc_runs = 0;           // key 31: CRC32C checksum kernel in runs of 2 / 4 consecutive tasks per wave (measurement)
    int matmul_pair = 0;        // key 32: 1 = the wave-pair register kernel for k = 10 (measurement)
    int crc_block = 0;          // key 33: CRC32C checksum kernel threads per block (0 = 256; 768 = 3 waves per SIMD)
    int mixed_wq = 0;           // key 26: mixed decode work queue of wave-tiles (0 = default: 1 round of wave-tiles per atomic for k >= 6, 4 below; 1 / 2 / 4 forced; 3 = the fixed tile order)
};

#ifdef HEC_EXPERIMENTAL
// One consistent view of every knob (relaxed atomic loads).
Tune tune_snapshot();

// Validates and stores one knob; returns an HEC_* status.
int tune_store(int key, int value);
#else
// Product build: the defaults, always.
inline Tune tune_snapshot() { return Tune{}; }
#endif

// Multiprocessor count of a device (cached per device, thread-safe).
int num_cus(int device);

}  // namespace hec
