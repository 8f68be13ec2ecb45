/*
 * hdfs_ec_amd_exp.h -- measurement knobs of the HEC_EXPERIMENTAL build
 * (hdfs-native_amd/lib/libhdfs_ec_amd_exp.so, `make -C hdfs-native_amd exp`).
 *
 * NOT part of the drop-in interface (include/hdfs_ec_amd.h) and not exported
 * by the product library: lib/libhdfs_ec_amd.so always runs the measured
 * default launch shapes and compiles only their kernels.  The measurement
 * build adds the measured-and-rejected kernel variants and lets a harness
 * (bench.py --tune, scripts/, tests/test_gpu_experimental.py) pick shapes and
 * variants for same-box A/B runs.  Knobs are process-wide atomics; every
 * launch reads one consistent snapshot at its start, so a concurrent
 * hec_tune_set only affects launches made after it.
 *
 * key 1: 16-B column chunks per lane per tile (1, 2, 3, 4; 8 for k <= 3; 0 = default)
 * key 2: non-temporal global loads/stores (0 or 1; -1 = default on)
 * key 3: blocks per CU for the grid (1..16; 0 = default)
 * key 4: threads per block (256 or 512; 0 = default)
 * key 5: kernel pipeline: 1 = register, 2 = LDS-DMA prefetch, 0 = default
 *        (3 / 4 / 5 -- register double buffering, output bursts, double-
 *        buffered tiles -- were removed in round 6)
 * key 6: store drain per tile in the register kernels: 1 = no drain,
 *        0 / 2 = drain (default)
 * key 7: absolute grid size in blocks (0 = default)
 * key 8: tile order, stripes interleaved per group (1 = stripe-major; 0 = default 4)
 * key 9: 1 = hec_encode_crc_device as encode + separate CRC pass (0 = fused)
 * key 10: fused encode+CRC slabs per wave: 0 = default, 4 or 8
 * key 11: CRC lookups: 0 = default (CRC32C: each 128-B quarter folded by a
 *         sparse multiple of the polynomial, then 11-bit slicing over its
 *         tail; CRC32: 11-bit slicing), 7 = the same as 0, 1 = slice-by-8, 5 =
 *         11-bit slicing everywhere, 2 / 3 = bank-replicated slice-by-1 with
 *         4 / 8 chains, 4 = slice-by-8 at 4 waves per SIMD (checksum
 *         kernel), 6 = bank-replicated slice-by-2, 9 = memory side only
 *         (WRONG sums), 10 / 11 = the fold over 16 / 20 of the quarter's 32
 *         dwords (512- / 384-bit tail of lookups; CRC32C, RS(6,3) and
 *         RS(10,4) in the fused kernels), 12 = the fold with a
 *         slicing-by-32 tail (32 independent lookups; CRC32C, the same
 *         fused shapes and the specialised decode + verify)
 * key 12: CRC register prefetch depth in 8-KiB tasks: 0 = default (1 for the
 *         CRC32C fold, else 2), 1 or 2
 * key 13: retired in round 6 (store cache policy of the removed pipe kernel)
 * key 14: host threads that copy the present data cells in hec_decode_host_batch
 *         (0 = default 4)
 * key 15: retired in round 6 (the removed output-burst kernel)
 * key 16: fused kernels' waves per SIMD: 0 / 2 = default; 3
 * key 17: per-call drop-in (hec_encode / hec_decode) pipeline piece in KiB per
 *         shard, a multiple of 4 (0 = default 256)
 * key 18: unaligned layouts: 0 = default (dword-realigning kernel + byte tail),
 *         1 = the byte kernel alone
 * key 19: fused kernels at 4 slabs per wave: 0 / 2 = inputs two at a time
 *         (default), 1 = one at a time
 * key 20: mixed-pattern decode, rows past a stripe's erasure count: 0 / 2 =
 *         skipped (default), 1 = computed and dropped at the store
 * key 21: fused kernels' wave roles: 0 / 1 = every wave alternates GF math
 *         and CRC rounds (the only form since round 6 removed the role split)
 * key 22: fused encode + CRC parity: 0 = default (bit-sliced XOR network of
 *         the RS matrix for RS(3,2), RS(6,3), RS(10,4)), 1 = v_perm tables
 * key 23: register / LDS-DMA encode kernels: 0 = default (v_perm tables),
 *         1 = bit-sliced XOR network of the RS matrix (gf_encode_bsl, and
 *         gf_matmul_dma's BSL form; RS(3,2), RS(6,3), RS(10,4); measured
 *         slower at RS(6,3) 1 MiB, not kept)
 * key 24: fused kernels' load schedule: 0 / 1 = default; 2 = at 4 slabs
 *         (key 10 = 4; JIT decode + verify, bit-sliced encode twins) two
 *         input pairs loaded ahead; 3 = at 8 slabs (JIT decode + verify, the
 *         bit-sliced encode) each input's loads issued before the parity
 *         math of the previous one, which reads its staged copy; 4 = (JIT
 *         decode + verify) the expected chunk sums loaded once per tile and
 *         shuffled to the CRC rounds; 5 = (JIT decode + verify) the rebuilt
 *         rows stored and the next tile's first inputs loaded before the
 *         last input's CRC round
 * key 25: fused kernels: stripe s starts its tile columns at (s * value) mod
 *         the tiles per stripe (0 = default, no rotation; up to 4096)
 * key 26: mixed-pattern decode work queue: 0 = default (1 round of wave-tiles
 *         per atomic for k >= 6, 4 below); 1 / 2 / 4 forced; 3 = fixed order
 * key 27: register kernel work queue: 0 = default (2 rounds per atomic for
 *         k <= 3, 1 for k = 6, 10); 1 / 2 forced; 3 = the fixed tile order
 * key 28: fused kernels' work queue: 0 = default (encode + CRC at k = 3, 10,
 *         decode + verify at every k); 1 = everywhere; 2 = block tiles
 * key 29: CRC32C checksum kernel on the work queue, 1 / 2 / 4 / 8 / 16 tasks
 *         per unit (0 = default: the fixed order)
 * key 30: 1 = the CRC kernels store their sums non-temporal
 * key 31: CRC32C checksum kernel in runs of 2 / 4 / 8 / 16 consecutive tasks
 *         of one cell per wave (fixed order)
 * key 32: 1 = the wave-pair register kernel for k = 10 (gf_matmul_pair: two
 *         waves per wave-tile, 5 inputs each, partials exchanged in LDS);
 *         key 3 sets its 128-thread blocks per CU (0 = 4: two waves per SIMD)
 * key 33: 768 = the CRC32C checksum kernel (the fold, compute and verify) in
 *         one 768-thread block per CU: 3 waves per SIMD (0 = default: two
 *         256-thread blocks per CU)
 * Returns HEC_OK, or HEC_ERR_INVALID_ARG for an unknown key / value.
 */
#ifndef HDFS_EC_AMD_EXP_H
#define HDFS_EC_AMD_EXP_H

#ifdef __cplusplus
extern "C" {
#endif

int hec_tune_set(int key, int value);

#ifdef __cplusplus
}
#endif

#endif /* HDFS_EC_AMD_EXP_H */
