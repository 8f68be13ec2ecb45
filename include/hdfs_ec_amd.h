/*
 * hdfs_ec_amd.h -- C ABI of the MI355X-native Reed-Solomon erasure-coding
 * engine that drops in behind hdfs-native's internal EC functions.
 *
 * Reference interface replaced (hdfs-native 0.14.1, Rust; public under the
 * `benchmark` feature, rust/src/lib.rs:49-52):
 *   hdfs_native::ec::gf256::Coder::new            rust/src/ec/gf256.rs:32-38
 *   hdfs_native::ec::gf256::Coder::gen_rs_matrix  rust/src/ec/gf256.rs:40-57
 *   hdfs_native::ec::gf256::Coder::encode         rust/src/ec/gf256.rs:61-80
 *   hdfs_native::ec::gf256::Coder::decode         rust/src/ec/gf256.rs:84-137
 *   Matrix::select_rows / Matrix::invert          rust/src/ec/matrix.rs:74-84, :101-162
 *   Mul<&[&[u8]]> for Matrix (the hot loop)       rust/src/ec/matrix.rs:204-231
 * Callers in the reference: CellBuffer::encode (rust/src/hdfs/block_writer.rs:838),
 * EcSchema::ec_decode (rust/src/ec/mod.rs:71-72), rust/benches/ec.rs.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every function returns an int status
 *    (HEC_OK == 0) and never aborts or throws across the ABI.
 *  - GF(2^8) modulo 0x11D, Hadoop Cauchy coding matrix: results are
 *    bit-identical to the reference Coder on the same inputs.
 *  - A coder is bound to one HIP device.  The host-buffer calls
 *    (hec_encode/hec_decode) are synchronous and serialised per coder by an
 *    internal lock (one coder may be shared by threads; use one coder per
 *    thread for concurrency).  The device calls are asynchronous: they only
 *    enqueue work on the caller's HIP stream (`hip_stream` is a hipStream_t
 *    passed as void*; NULL = the null stream).  Their only lock is the
 *    stream's work-queue counter-set lock, held from choosing the launch's
 *    counter set to enqueuing its kernel (see hec_queue_stats).
 */
#ifndef HDFS_EC_AMD_H
#define HDFS_EC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HEC_ABI_VERSION 5

/* Status codes */
#define HEC_OK 0
#define HEC_ERR_INVALID_ARG (-1)       /* reference: assert!/panic (gf256.rs:62-65, matrix.rs:57) */
#define HEC_ERR_NOT_ENOUGH_SHARDS (-2) /* HdfsError::ErasureCodingError("Not enough valid shards") gf256.rs:107-111 */
#define HEC_ERR_UNSUPPORTED_CODEC (-3) /* HdfsError::UnsupportedErasureCodingPolicy mod.rs:74-78 */
#define HEC_ERR_DEVICE (-4)            /* HIP runtime / launch failure */
#define HEC_ERR_NO_MEMORY (-5)         /* host or device allocation failed */
#define HEC_ERR_SINGULAR (-6)          /* reference panics "Matrix is singular" matrix.rs:121-123 */
#define HEC_ERR_CHECKSUM (-7)          /* HdfsError::ChecksumError connection.rs:497-499 */

/* Chunk checksum types: ChecksumTypeProto values (rust/src/proto/hadoop.hdfs.rs:1363),
 * mapped to algorithms by ReadPacket::get_data (rust/src/hdfs/connection.rs:483-487). */
#define HEC_CHECKSUM_NULL 0   /* CHECKSUM_NULL: no verification */
#define HEC_CHECKSUM_CRC32 1  /* crc 3.4 CRC_32_CKSUM (connection.rs:37): MSB-first 0x04C11DB7, init 0, xorout ~0 */
#define HEC_CHECKSUM_CRC32C 2 /* crc 3.4 CRC_32_ISCSI (connection.rs:38): Castagnoli, reflected, init/xorout ~0 */

/* Limits of this engine (the reference has k+m <= 256 through `r as u8`). */
#define HEC_MAX_DATA_UNITS 32
#define HEC_MAX_PARITY_UNITS 16

typedef struct hec_coder hec_coder_t;

/* Human-readable text for a status code (static storage). */
const char *hec_strerror(int status);
int hec_abi_version(void);
/* Detail of the last failing HIP call made by this thread ("" if none). */
const char *hec_last_error(void);

/* ---- Field / matrix helpers (host only, no device needed) ------------- */

/* Coder::gen_rs_matrix (gf256.rs:40-57): writes the (k+m) x k coding matrix,
 * row-major, into out[(k+m)*k]. */
int hec_gen_rs_matrix(size_t data_units, size_t parity_units, uint8_t *out);

/* The same for a codec name as hec_coder_create_codec ("rs", "xor",
 * "rs-legacy"): the (k+m) x k matrix a coder of that codec encodes and
 * decodes with.  HEC_ERR_UNSUPPORTED_CODEC for other names. */
int hec_gen_codec_matrix(const char *codec, size_t data_units, size_t parity_units, uint8_t *out);

/* Matrix::invert (matrix.rs:101-162): in-place inverse of an n x n
 * row-major matrix over GF(2^8).  HEC_ERR_SINGULAR where the reference panics. */
int hec_matrix_invert(uint8_t *mat, size_t n);

/* The decode plan of Coder::decode (gf256.rs:84-126) for a presence mask.
 * present[k+m]: non-zero = shard available.  On HEC_OK:
 *   *n_missing   = e, the number of missing DATA shards (0 => nothing to do);
 *   survivors[k] = the first k present shard indices, ascending;
 *   missing[e]   = the missing data indices, ascending;
 *   matrix[e*k]  = rows of inverse(select_rows(encode_matrix, survivors))
 *                  for the missing indices (row-major).
 * Returns HEC_ERR_NOT_ENOUGH_SHARDS when e > 0 and fewer than k are present. */
int hec_decode_plan(size_t data_units, size_t parity_units, const uint8_t *present,
                    size_t *n_missing, size_t *survivors, size_t *missing, uint8_t *matrix);

/* ---- Coder lifecycle (Coder::new, gf256.rs:32-38) --------------------- */

/* `device` value of a host-only coder: no HIP call is made (creation cannot
 * fail for want of a GPU).  hec_encode / hec_decode and the host-batch calls
 * (hec_encode_host_batch, hec_decode_host_batch, hec_*_rows_host) run the
 * engine's host routine (hec_gf_matmul_host) whatever the host limit; the
 * device-resident calls return HEC_ERR_DEVICE.  This keeps the reference's
 * infallible Coder::new (gf256.rs:32-38) on a host without a visible GPU. */
#define HEC_DEVICE_HOST (-2)

/* Creates a coder for RS(data_units, parity_units) on HIP device `device`
 * (or HEC_DEVICE_HOST).
 * 1 <= data_units <= HEC_MAX_DATA_UNITS, 1 <= parity_units <= HEC_MAX_PARITY_UNITS. */
int hec_coder_create(size_t data_units, size_t parity_units, int device, hec_coder_t **out);
/* Same with a codec name: "rs" (the default above), "xor" (Hadoop XOR-k-1:
 * parity = XOR of the data units; parity_units must be 1) or "rs-legacy"
 * (Hadoop RSRawEncoderLegacy: systematic cyclic RS, generator roots 2^0 ..
 * 2^(m-1), data unit i at degree m+i; policy 3, RS-LEGACY-6-3-1024k).  The
 * reference resolves policies 3 and 4 (ec/mod.rs:118-131) but decodes only
 * "rs" (mod.rs:69-78); this engine codes all three on the same kernels.  Any
 * other name -> HEC_ERR_UNSUPPORTED_CODEC. */
int hec_coder_create_codec(const char *codec, size_t data_units, size_t parity_units, int device,
                           hec_coder_t **out);
void hec_coder_destroy(hec_coder_t *coder);
size_t hec_coder_data_units(const hec_coder_t *coder);
size_t hec_coder_parity_units(const hec_coder_t *coder);
int hec_coder_device(const hec_coder_t *coder);

/* Pooled coders for callers that build a Coder per row: the reference
 * constructs one per decoded row (ec/mod.rs:71-72, Coder::new gf256.rs:32-38)
 * and one per block writer (block_writer.rs:787).  hec_coder_acquire hands
 * out an idle coder of the same (codec, data_units, parity_units, device)
 * from a process-wide pool, or creates one; hec_coder_release returns it (at
 * most 64 idle per key are kept, the rest destroyed).  An acquired coder is
 * the caller's alone until released; steady state costs a mutex and a
 * vector pop -- no stream, event or buffer creation.  device -1 = any device
 * (round-robin over the visible ones; a host-only coder, HEC_DEVICE_HOST, when
 * no GPU is visible), HEC_DEVICE_HOST = host-only.  Release resets the coder's host
 * limit to the default (a setting never carries over to the next acquirer)
 * and ignores a second release of a coder that is already idle in the pool.
 * hec_coder_release on a coder from hec_coder_create destroys it.
 * hec_coder_pool_trim destroys every idle pooled coder and returns how many. */
int hec_coder_acquire(const char *codec, size_t data_units, size_t parity_units, int device, hec_coder_t **out);
void hec_coder_release(hec_coder_t *coder);
size_t hec_coder_pool_trim(void);

/* Routing of the host-buffer drop-ins below (hec_encode / hec_decode on
 * pageable buffers): rows of at most `max_shard_len` bytes per shard are coded
 * by the engine's host routine (hec_gf_matmul_host; rows of >= 256 KiB per
 * shard split over $HEC_HOST_THREADS threads, default 4), longer ones go
 * through the device (pinned bounce buffers, H2D, kernel, D2H).  Per coder;
 * default SIZE_MAX = every row on the host: measured per size, cold and hot,
 * the PCIe round trip of a pageable row never paid for itself;
 * 0 = always the device.  The batched and device-resident calls are not
 * affected. */
int hec_coder_set_host_limit(hec_coder_t *coder, size_t max_shard_len);
size_t hec_coder_host_limit(const hec_coder_t *coder);

/* ---- Host-buffer drop-ins (synchronous) -------------------------------- */

/* Coder::encode (gf256.rs:61-80).  data[k] host buffers of shard_len bytes
 * each; parity[m] caller-allocated host buffers of shard_len bytes, fully
 * overwritten.  shard_len == 0 -> HEC_ERR_INVALID_ARG (the reference panics,
 * matrix.rs:57).  Any shard_len >= 1 is accepted, including tails that are not
 * a multiple of 16. */
int hec_encode(hec_coder_t *coder, const uint8_t *const *data, size_t shard_len,
               uint8_t *const *parity);

/* Coder::decode (gf256.rs:84-137).  shards[k+m] host buffers of shard_len
 * bytes, NULL = missing.  For every missing DATA index i (< k) out[i] must
 * point to shard_len writable bytes and receives the reconstructed shard;
 * out[] entries for present shards and for parity indices are never touched
 * (missing parity is not regenerated, gf256.rs:96-97).  Survivors are the
 * first k present shards in index order.  Returns HEC_OK without writing when
 * no data shard is missing, HEC_ERR_NOT_ENOUGH_SHARDS when fewer than k
 * shards are present. */
int hec_decode(hec_coder_t *coder, const uint8_t *const *shards, size_t shard_len,
               uint8_t *const *out);

/* The hot loop Mul<&[&[u8]]> (matrix.rs:204-231) on the host, for rows too
 * small for the device: out[j] = sum_i matrix[j*cols + i] * in[i], len bytes
 * each, any length and alignment; AVX-512BW+GFNI affine transforms (one
 * vgf2p8affineqb per 64 bytes per coefficient), else AVX2 split-nibble
 * shuffles, else scalar tables (hec_host_isa names the one in use).
 * 1 <= cols <= HEC_MAX_DATA_UNITS.  Synchronous, thread-safe, no device. */
int hec_gf_matmul_host(const uint8_t *matrix, size_t rows, size_t cols, const uint8_t *const *in, uint8_t *const *out,
                       size_t len);
const char *hec_host_isa(void);

/* ---- Device-resident batched API (asynchronous, on hip_stream) --------- *
 * A batch is `stripes` independent stripes of cell_len-byte cells.  Shard i
 * of stripe s lives at  base[i] + s * stride[i]  (device pointers).  For the
 * [stripe][shard][cell] layout pass base[i] = buf + i*cell_len and
 * stride[i] = units*cell_len.  The fast path needs every base and stride
 * 16-byte aligned; other layouts run a byte-granular kernel (same results). */

/* Batched Coder::encode: parity[j] = sum_i C[k+j][i] * data[i]. */
int hec_encode_device(hec_coder_t *coder, const uint8_t *const *d_data, const size_t *data_strides,
                      uint8_t *const *d_parity, const size_t *parity_strides, size_t cell_len,
                      size_t stripes, void *hip_stream);

/* Batched Coder::decode with one erasure pattern for the whole batch.
 * d_shards[k+m] (NULL = missing) with shard_strides[k+m]; d_out[k] with
 * out_strides[k], used only for missing data indices.  The decode matrix is
 * computed on the host once per pattern and cached in the coder. */
int hec_decode_device(hec_coder_t *coder, const uint8_t *const *d_shards, const size_t *shard_strides,
                      uint8_t *const *d_out, const size_t *out_strides, size_t cell_len,
                      size_t stripes, void *hip_stream);

/* Batched Coder::decode where every stripe has its OWN erasure pattern, as a
 * striped read over many block groups sees (ec/mod.rs:71 decodes row by
 * row).  d_shards[k+m]/shard_strides[k+m]: storage of every shard index
 * (never NULL; slots a stripe lacks are not read).  present[stripes] (host):
 * bit i set = shard i of that stripe is available.  Reconstructed data shard
 * i of stripe s goes to d_out[i] + s*out_strides[i], only where it is
 * missing.  One plan per distinct pattern (first-k-present survivors, as
 * gf256.rs:84-126) is built on the host, cached in the coder and uploaded to
 * d_workspace (hec_decode_mixed_workspace_size bytes; keep it untouched
 * until the stream reaches the work: the launch also keeps its tile-queue
 * counters there, so calls in flight on different streams need different
 * workspaces).  If any stripe lacks data shards and
 * has fewer than k present, HEC_ERR_NOT_ENOUGH_SHARDS is returned and
 * nothing is launched. */
size_t hec_decode_mixed_workspace_size(const hec_coder_t *coder, size_t stripes);
int hec_decode_device_mixed(hec_coder_t *coder, const uint8_t *const *d_shards, const size_t *shard_strides,
                            uint8_t *const *d_out, const size_t *out_strides, const uint64_t *present,
                            size_t cell_len, size_t stripes, void *d_workspace, size_t workspace_bytes,
                            void *hip_stream);

/* The raw hot loop, Mul<&[&[u8]]> (matrix.rs:204-231), batched:
 * out[j] = sum_i matrix[j*cols + i] * in[i] for j < rows, i < cols.
 * Any rows >= 1 (launched 4 output rows at a time), 1 <= cols <=
 * HEC_MAX_DATA_UNITS.  Runs on the coder's device. */
int hec_gf_matmul_device(hec_coder_t *coder, const uint8_t *matrix, size_t rows, size_t cols,
                         const uint8_t *const *d_in, const size_t *in_strides, uint8_t *const *d_out,
                         const size_t *out_strides, size_t cell_len, size_t stripes, void *hip_stream);

/* ---- Chunk checksums -------------------------------- *
 * WritePacket::calculate_checksum (rust/src/hdfs/connection.rs:568-584) on
 * the device: for each of `n_shards` cells of `stripes` stripes (shard i of
 * stripe s at d_bases[i] + s*strides[i], cell_len bytes), one CRC32C
 * (Castagnoli / crc CRC_32_ISCSI, connection.rs:37-38) per
 * bytes_per_checksum chunk, the last one possibly short, written big-endian
 * (put_u32) to d_out + 4*((s*n_shards + i)*nchunks + c), nchunks =
 * ceil(cell_len / bytes_per_checksum).  Runs on the coder's device; the
 * fast path is bytes_per_checksum == 512 with 16-B aligned cells. */
int hec_crc32c_device(hec_coder_t *coder, const uint8_t *const *d_bases, const size_t *strides, size_t n_shards,
                      size_t cell_len, size_t stripes, size_t bytes_per_checksum, uint8_t *d_out,
                      void *hip_stream);

/* The same for either algorithm the read path accepts: `checksum_type` is
 * HEC_CHECKSUM_CRC32C or HEC_CHECKSUM_CRC32 (HEC_CHECKSUM_NULL is invalid
 * here: there is nothing to compute). */
int hec_checksum_device(hec_coder_t *coder, int checksum_type, const uint8_t *const *d_bases, const size_t *strides,
                        size_t n_shards, size_t cell_len, size_t stripes, size_t bytes_per_checksum,
                        uint8_t *d_out, void *hip_stream);

/* ReadPacket::get_data's check (connection.rs:477-504) over whole cells:
 * recomputes every chunk checksum and compares it with d_expected (same
 * layout as hec_checksum_device's output, big-endian as received).
 * d_bad[s*n_shards + i] is set to 1 when any chunk of cell (s, i)
 * mismatches (the reference's HdfsError::ChecksumError for that packet) and
 * is otherwise left untouched: zero it first.  HEC_CHECKSUM_NULL verifies
 * nothing and returns HEC_OK.  Asynchronous on hip_stream. */
int hec_checksum_verify_device(hec_coder_t *coder, int checksum_type, const uint8_t *const *d_bases,
                               const size_t *strides, size_t n_shards, size_t cell_len, size_t stripes,
                               size_t bytes_per_checksum, const uint8_t *d_expected, uint8_t *d_bad,
                               void *hip_stream);

/* The striped read of one batch of rows (block_reader.rs:480-525 feeding
 * EcSchema::ec_decode, ec/mod.rs:62-89) with every cell it consumes
 * checksum-verified.  d_shards[k+m] as hec_decode_device (NULL = shard not
 * available for the whole batch).  Per stripe the survivors are the first k
 * available shards whose chunk checksums verify against d_sums
 * ([stripe][k+m][nchunks] big-endian, the sums that arrived with the
 * packets); a shard that fails is skipped and the next available one is
 * read instead, as read_slice drops a failing cell reader and starts the
 * next parity reader.  Every data shard that is missing or failed is
 * rebuilt into d_out[i] (out_strides as hec_decode_device; all k slots
 * are required, and a present data shard's slot may be its own input
 * buffer, which then is repaired in place); present data shards that
 * verify are not copied.  d_bad[s*(k+m) + i] = 1 marks the
 * cells that failed (zeroed by the call; device memory).  When every stripe
 * verifies first time this is one fused pass over the survivors (k in
 * {2,3,6,10}, 512-B chunks, 16-B aligned).  Stripes with a failing cell
 * are re-planned on the host together: each round verifies every newly
 * used cell of all of them (one stripe-list checksum launch per shard
 * index, one flag read-back), and one mixed-pattern decode then rebuilds
 * them all (at most m rounds).  Synchronous (it must see the
 * verdicts).  Returns HEC_ERR_NOT_ENOUGH_SHARDS when some stripe has fewer
 * than k shards that verify (its d_bad flags say which; the other stripes
 * are still rebuilt).  HEC_CHECKSUM_NULL decodes without verifying. */
int hec_decode_verify_device(hec_coder_t *coder, int checksum_type, const uint8_t *const *d_shards,
                             const size_t *shard_strides, uint8_t *const *d_out, const size_t *out_strides,
                             size_t cell_len, size_t stripes, size_t bytes_per_checksum, const uint8_t *d_sums,
                             uint8_t *d_bad, void *hip_stream);

/* Plan-time specialisation of the fused decode + verify pass.
 * That pass rebuilds the missing data rows with the decode plan's matrix,
 * known only at run time, through v_perm product tables.  For a plan the
 * engine meets, it generates the matrix's bit-sliced XOR network and compiles
 * the same kernel with it (hiprtc, loaded with dlopen): about a third fewer
 * VALU ops for RS(6,3) with 3 rows lost.  By default the compile runs on a
 * background thread the first time a plan is launched, and launches use the
 * ahead-of-time kernel until it is ready (identical results).  Code objects
 * are cached per process and on disk ($HEC_JIT_CACHE, default
 * ~/.cache/hdfs_ec_amd/jit; "" = none).  HEC_JIT=0 disables it, HEC_JIT=sync
 * compiles on first use.
 *   hec_coder_prepare_decode: compile (or load) the specialised kernel for the
 *     presence mask present[k+m] and checksum type now, synchronously, on the
 *     coder's device; *specialised = 1 when it is ready (0: not available --
 *     no hiprtc, JIT off, no fused shape for this plan, or nothing missing).
 *   hec_jit_warm: the same into the caches only, no device needed (install-
 *     time warm-up).  HEC_ERR_INVALID_ARG for a plan without a fused kernel
 *     (k not in {2,3,6,10}, no or more than 4 data shards missing),
 *     HEC_ERR_DEVICE when hiprtc is absent or the compile fails.
 *   hec_jit_stats: kernels compiled, loaded from the disk cache, failed,
 *     and launches that ran a specialised kernel (process totals). */
int hec_coder_prepare_decode(hec_coder_t *coder, const uint8_t *present, int checksum_type, int *specialised);
int hec_jit_warm(size_t data_units, size_t parity_units, const uint8_t *present, int checksum_type);
void hec_jit_stats(uint64_t *compiled, uint64_t *from_disk, uint64_t *failed, uint64_t *launches);

/* ---- work-queue counter sets (diagnostic) -------------- *
 * The coding kernels deal their tiles from launch counters.  Every stream
 * that launched one has two counter sets it alternates between (each launch
 * zeroes the set of the stream's next launch); a launch into a capturing
 * stream gets a set of its own, zeroed by a memset node in the graph.
 * hec_queue_stats: streams with sets and graph sets handed out on `device`
 * (process totals; past 4096 streams / 256 graph launches per device the
 * kernels fall back to their fixed tile order), and *keyed_by_id = 1 when
 * streams are told apart by hipStreamGetId (HIP >= 7.1 in the process), 0
 * when by handle.  Any pointer may be NULL; all zeros for a device that
 * does not exist. */
void hec_queue_stats(int device, uint64_t *streams, uint64_t *graph_sets, int *keyed_by_id);

/* Encode plus CRC32C of the k data and m parity cells (shard order
 * 0..k+m-1, same output layout as hec_crc32c_device): everything a striped
 * writer needs to emit its k+m packet streams.  One fused pass (the
 * checksums are taken from the registers/LDS the encode already holds) for
 * k in {2,3,6,10}, m <= 4, 512-B chunks and 16-B aligned cells; otherwise an
 * encode followed by hec_crc32c_device. */
int hec_encode_crc_device(hec_coder_t *coder, const uint8_t *const *d_data, const size_t *data_strides,
                          uint8_t *const *d_parity, const size_t *parity_strides, size_t cell_len, size_t stripes,
                          size_t bytes_per_checksum, uint8_t *d_sums, void *hip_stream);

/* ---- Pinned-host pipelined batch (PCIe-inclusive path) ----------------- *
 * Encodes a [stripe][k][cell] host batch into a [stripe][m][cell] host batch,
 * streaming chunks of `chunk_stripes` stripes H2D -> encode -> D2H with
 * copy/compute overlap on the coder's own streams (3 device slots; H2D,
 * compute and D2H of consecutive chunks run concurrently).  Host buffers should be
 * pinned (hipHostMalloc / registered) for full PCIe rate.  Synchronous. */
int hec_encode_host_batch(hec_coder_t *coder, const uint8_t *h_data, uint8_t *h_parity,
                          size_t cell_len, size_t stripes, size_t chunk_stripes);

/* The read side, fused with the cell split (ec/mod.rs:62-89): h_vertical[k+m]
 * are the per-shard "vertical" buffers a striped reader accumulates (shard i
 * = its cells of `rows` consecutive rows, rows*cell_len bytes; NULL =
 * missing).  Writes the k*cell_len*rows file bytes, in file (row) order, to
 * h_file: present data cells are copied, missing ones reconstructed
 * (first-k-present survivors).  The k survivors stream H2D through the same
 * 3-slot pipeline as the encode and only the rebuilt cells come back D2H;
 * the present data cells are copied host-side (up to 4 threads) while the
 * DMA runs.  HEC_ERR_NOT_ENOUGH_SHARDS when a data shard is missing and fewer
 * than k shards are present.  Synchronous. */
int hec_decode_host_batch(hec_coder_t *coder, const uint8_t *const *h_vertical, size_t cell_len, size_t rows,
                          uint8_t *h_file, size_t chunk_rows);

/* ---- Whole files: the last row may be short ------------------------------ *
 * A file of data_len bytes is rows of k cells in file order (CellBuffer::write,
 * block_writer.rs:791-805); the last row may hold L < k*cell_len bytes: cell
 * i of it has min(cell_len, max(0, L - i*cell_len)) bytes.  As
 * CellBuffer::encode (block_writer.rs:817-851) every cell of that row is
 * zero-padded to n0 = min(cell_len, L) and its m parity cells are n0 bytes
 * long; the engine writes them at their [row][m][cell_len] slots and zeroes
 * the slot bytes past n0.  Full rows run exactly as hec_encode_host_batch /
 * hec_encode_device. */
int hec_encode_rows_host(hec_coder_t *coder, const uint8_t *h_data, size_t data_len, uint8_t *h_parity,
                         size_t cell_len, size_t chunk_stripes);

/* The same on device memory (asynchronous on hip_stream): d_parity holds
 * ceil(data_len / (k*cell_len)) rows.  The short row's short cells are
 * zero-padded into d_workspace (hec_encode_rows_workspace_size bytes, untouched
 * until the stream reaches the work), so nothing is read past d_data +
 * data_len.  The workspace is checked before anything is queued, and is
 * needed (may be NULL otherwise) only when some cell of the short row holds
 * fewer than n0 bytes. */
size_t hec_encode_rows_workspace_size(const hec_coder_t *coder, size_t cell_len);
int hec_encode_rows_device(hec_coder_t *coder, const uint8_t *d_data, size_t data_len, uint8_t *d_parity,
                           size_t cell_len, void *d_workspace, size_t workspace_bytes, void *hip_stream);

/* hec_decode_host_batch over a whole file: h_vertical[i] holds vertical_len[i]
 * bytes of shard i (its block: max_offset(i), ec/mod.rs:40-60; NULL =
 * missing), and the file is file_len bytes.  Every cell shorter than cell_len
 * (or absent past the end of its shard) reads as zeros, as
 * CellReader::next_cell pads it (block_reader.rs:343-378); the short last row
 * is decoded like the others and trimmed to file_len (block_reader.rs:
 * 524-549).  HEC_ERR_INVALID_ARG if a present shard holds fewer than
 * full_rows * cell_len bytes. */
int hec_decode_rows_host(hec_coder_t *coder, const uint8_t *const *h_vertical, const size_t *vertical_len,
                         size_t cell_len, uint8_t *h_file, size_t file_len, size_t chunk_rows);

/* ---- Multi-GPU coder group --------------------------------- *
 * Stripes are independent, so a batch is split into contiguous stripe ranges,
 * one per device, and each range runs on its own device's coder from its own
 * host thread (own streams and 3-slot pipeline), with no collective and no
 * device-to-device traffic.  This is the in-process form of the stripe
 * sharding the bench does with one process per GPU.  Range of device slot i
 * for `total` stripes: sizes differ by at most one and tile [0, total) in slot
 * order (hec_group_range).  A device may appear more than once (several
 * coders on one GPU).  The group calls are synchronous; on failure they
 * return the status of the lowest failing slot (hec_last_error() of the
 * calling thread carries its detail) after every slot has finished. */
typedef struct hec_group hec_group_t;

/* codec "rs" or "xor" as hec_coder_create_codec; n_devices in 1..64. */
int hec_group_create(const char *codec, size_t data_units, size_t parity_units, const int *devices,
                     size_t n_devices, hec_group_t **out);
void hec_group_destroy(hec_group_t *group);
size_t hec_group_size(const hec_group_t *group);
/* Slot i's coder (owned by the group), for device-resident calls on that GPU. */
hec_coder_t *hec_group_coder(hec_group_t *group, size_t slot);
/* Slot i's contiguous share [*first, *first + *count) of `total` stripes. */
int hec_group_range(const hec_group_t *group, size_t total, size_t slot, size_t *first, size_t *count);

/* hec_encode_host_batch over the group: slot i encodes its stripe range of
 * the [stripe][k][cell] host batch into the same rows of h_parity. */
int hec_group_encode_host_batch(hec_group_t *group, const uint8_t *h_data, uint8_t *h_parity, size_t cell_len,
                                size_t stripes, size_t chunk_stripes);

/* hec_decode_host_batch over the group: slot i decodes its row range (its
 * part of every vertical buffer) into its rows of h_file. */
int hec_group_decode_host_batch(hec_group_t *group, const uint8_t *const *h_vertical, size_t cell_len,
                                size_t rows, uint8_t *h_file, size_t chunk_rows);

/* Device-resident batches over the group (the in-process form of the
 * bench's one-rank-per-GPU sharding; no host threads, no collective): slot i's
 * stripes live in ITS device's HBM.  Per-slot arrays, slot-major: d_data[i*k
 * + s] / data_strides[i*k + s] and d_parity[i*m + j] / parity_strides[i*m +
 * j] as hec_encode_device takes them; for decode d_shards[i*(k+m) + s]
 * (NULL = missing) / shard_strides[i*(k+m) + s] and d_out[i*k + s] /
 * out_strides[i*k + s] as hec_decode_device.  stripes[i] = slot i's stripe
 * count (0 = nothing), hip_streams[i] its stream on that device (NULL array =
 * default streams).  Asynchronous like the single-coder calls: every slot's
 * launch is enqueued from the calling thread, one device after another, and
 * the GPUs run concurrently; synchronise the streams before reading.
 * Returns the lowest failing slot's status; the other slots are still
 * enqueued.  Replaces the per-writer join_all fan-out of block_writer.rs:954
 * for device-resident stripes. */
int hec_group_encode_device(hec_group_t *group, const uint8_t *const *d_data, const size_t *data_strides,
                            uint8_t *const *d_parity, const size_t *parity_strides, size_t cell_len,
                            const size_t *stripes, void *const *hip_streams);
int hec_group_decode_device(hec_group_t *group, const uint8_t *const *d_shards, const size_t *shard_strides,
                            uint8_t *const *d_out, const size_t *out_strides, size_t cell_len,
                            const size_t *stripes, void *const *hip_streams);

/* ---- HBM buffers for the batched API ------------------------------------ *
 * Device memory for stripe batches on `device` (hipExtMallocWithFlags).
 * Checksum sum / flag buffers passed to the checksum calls must be 4-byte
 * aligned (they are read and written as u32).
 * HEC_ALLOC_CONTIGUOUS asks for physically contiguous HBM, which the GPU
 * maps with large page fragments: a batch of tens of GiB then needs far
 * fewer translation entries.  hec_device_free releases it
 * (synchronous, like hipFree). */
#define HEC_ALLOC_DEFAULT 0
#define HEC_ALLOC_CONTIGUOUS 1
int hec_device_alloc(int device, size_t bytes, unsigned flags, void **out);
int hec_device_free(int device, void *ptr);
/* hec_device_copy: `bytes` from src to dst, host or device memory either
 * side (unified addressing), synchronous; for callers without a HIP binding
 * of their own (the Rust shim's DeviceBuffer).  hec_device_synchronize: wait
 * for `hip_stream` on `device` (NULL = the device's default stream) -- the
 * device calls above only enqueue. */
int hec_device_copy(int device, void *dst, const void *src, size_t bytes);
int hec_device_synchronize(int device, void *hip_stream);

/* ---- NUMA-placed pinned host buffers (host-batch / group calls) -------- *
 * hec_host_alloc: `bytes` of page-locked host memory whose pages live on
 * NUMA node `numa_node` (-1 = the node of `device`'s PCIe root, read from
 * sysfs), registered with HIP for full-rate DMA: the buffers one group slot
 * streams to its GPU should sit next to that GPU's root complex.  Free with
 * hec_host_free.  hec_device_numa_node: that node, -1 if unknown. */
int hec_device_numa_node(int device);
int hec_host_alloc(int device, size_t bytes, int numa_node, void **out);
int hec_host_free(void *ptr);


#ifdef __cplusplus
}
#endif

#endif /* HDFS_EC_AMD_H */
