/* shim_replay.c -- replays, call for call, what rust/src/ec/mi355x.rs (the
 * Rust shim a maintainer adds to hdfs-native; not compilable in this image)
 * does through the C ABI, and checks the results against the CPU oracle
 * (oracle/ec_oracle.c, test infrastructure):
 *   GpuCoder::new     -> hec_abi_version, hec_coder_create_codec("rs")
 *   GpuCoder::encode  -> hec_encode (the shim asserts n > 0 first; the C side
 *                        rejects n == 0 with HEC_ERR_INVALID_ARG as well)
 *   GpuCoder::decode  -> hec_decode with null out slots for present shards
 *                        and parity (here: sentinel buffers, which must stay
 *                        untouched); HEC_ERR_NOT_ENOUGH_SHARDS -> the shim's
 *                        ErasureCodingError("Not enough valid shards")
 *   encode_rows / decode_rows / GpuGroup -> the batched calls
 *   Coder::new per row (rust/patches/ec_mi355x.patch: PooledCoder) ->
 *                        hec_coder_acquire / hec_coder_release: 10,000
 *                        acquire / encode / release cycles, timed against
 *                        create / destroy and against one device-routed call
 *   the reference's striped writer and reader (unchanged by the patch:
 *                        CellBuffer::encode per row, the short last row
 *                        zero-padded; read_slice per row with failed readers
 *                        replaced) -- byte streams == the oracle's; and
 *                        ec_decode's vertical stripes of several rows
 *   Coder::new without a GPU -> hec_coder_acquire(-1) = a host-only coder
 *                        (HEC_DEVICE_HOST); decode reads only the first k
 *                        present shards (a shorter shard past them is fine,
 *                        matrix.rs:212-216)
 *   the patch's device group of rust/benches/ec.rs (bench_mi355x) ->
 *                        hec_device_alloc / hec_device_copy, hec_encode_device
 *                        / hec_decode_device + hec_device_synchronize
 * The host-only part runs first and needs no GPU (exit 2 after it when no
 * device is visible).  Built by __graft_entry__.build(); run by
 * tests/test_shim_replay.py. */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/hdfs_ec_amd.h"

/* oracle/ec_oracle.c */
int orc_encode(size_t k, size_t m, const uint8_t *const *data, size_t n, uint8_t *const *parity);

static int failures = 0;
#define CHECK(cond, ...)                                  \
    do {                                                  \
        if (!(cond)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fprintf(stderr, "\n");                        \
            failures++;                                   \
        }                                                 \
    } while (0)

static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static uint64_t rng = 0x5EEDEC00u;
static uint8_t next_byte(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint8_t)(rng >> 24);
}

/* rows per Coder call in the reference's writer / reader: one (round 4's
 * patch batched 4; measured and dropped) */
enum { K = 6, M = 3, ROWS_PER_CALL = 1 };

/* CellBuffer::write + encode (block_writer.rs:791-851) over a file of `len`
 * bytes: every batch of up to ROWS_PER_CALL rows is one encode of the
 * vertical stripes (whole rows) plus one of the zero-padded short row; the
 * k + m shard streams are compared with the oracle's row-by-row CellBuffer
 * encode (block_writer.rs:817-851). */
static void replay_batched_writer(hec_coder_t *c, size_t cell, size_t len) {
    uint8_t *file = malloc(len);
    for (size_t b = 0; b < len; b++) file[b] = next_byte();
    const size_t row = K * cell;
    const size_t nrows = (len + row - 1) / row;
    /* expected streams: shard i = its cells row by row (data at their own
     * lengths, parity at len(cell 0) of the row) */
    uint8_t *want[K + M], *got[K + M];
    size_t want_len[K + M], got_len[K + M];
    for (int i = 0; i < K + M; i++) {
        want[i] = malloc(nrows * cell + 1);
        got[i] = malloc(nrows * cell + 1);
        want_len[i] = got_len[i] = 0;
    }
    uint8_t *pad = calloc(K, cell), *rp[M];
    for (int j = 0; j < M; j++) rp[j] = malloc(cell);
    for (size_t r = 0; r < nrows; r++) {
        const size_t base = r * row, L = len - base < row ? len - base : row;
        const size_t n0 = L < cell ? L : cell;
        const uint8_t *in[K];
        for (int i = 0; i < K; i++) {
            const size_t have = L > i * cell ? (L - i * cell < cell ? L - i * cell : cell) : 0;
            memset(pad + i * cell, 0, n0);
            memcpy(pad + i * cell, file + base + i * cell, have);
            in[i] = pad + i * cell;
            memcpy(want[i] + want_len[i], file + base + i * cell, have);
            want_len[i] += have;
        }
        orc_encode(K, M, in, n0, rp);
        for (int j = 0; j < M; j++) {
            memcpy(want[K + j] + want_len[K + j], rp[j], n0);
            want_len[K + j] += n0;
        }
    }
    /* the writer, ROWS_PER_CALL rows per encode */
    size_t pos = 0;
    while (pos < len) {
        const size_t take = len - pos < ROWS_PER_CALL * row ? len - pos : ROWS_PER_CALL * row;
        const size_t whole = take / row, L = take - whole * row;
        const size_t slice = whole * cell + (L < cell ? L : cell); /* shard 0's bytes */
        uint8_t *vd[K], *vp[M];
        size_t orig[K];
        for (int i = 0; i < K; i++) {
            vd[i] = calloc(slice ? slice : 1, 1);
            orig[i] = 0;
            for (size_t r = 0; r <= whole; r++) {
                const size_t rb = r * row + i * cell;
                if (rb >= take) break;
                const size_t have = take - rb < cell ? take - rb : cell;
                memcpy(vd[i] + r * cell, file + pos + rb, have);
                orig[i] = r * cell + have;
            }
        }
        for (int j = 0; j < M; j++) vp[j] = malloc(slice ? slice : 1);
        if (whole) {
            int rc = hec_encode(c, (const uint8_t *const *)vd, whole * cell, vp);
            CHECK(rc == HEC_OK, "batched encode %s", hec_strerror(rc));
        }
        if (slice > whole * cell) {
            const uint8_t *tin[K];
            uint8_t *tout[M];
            for (int i = 0; i < K; i++) tin[i] = vd[i] + whole * cell;
            for (int j = 0; j < M; j++) tout[j] = vp[j] + whole * cell;
            int rc = hec_encode(c, tin, slice - whole * cell, tout);
            CHECK(rc == HEC_OK, "short-row encode %s", hec_strerror(rc));
        }
        for (int i = 0; i < K; i++) {
            memcpy(got[i] + got_len[i], vd[i], orig[i]);
            got_len[i] += orig[i];
            free(vd[i]);
        }
        for (int j = 0; j < M; j++) {
            memcpy(got[K + j] + got_len[K + j], vp[j], slice);
            got_len[K + j] += slice;
            free(vp[j]);
        }
        pos += take;
    }
    for (int i = 0; i < K + M; i++) {
        CHECK(got_len[i] == want_len[i] && memcmp(got[i], want[i], want_len[i]) == 0,
              "writer stream %d (len %zu vs %zu, file %zu)", i, got_len[i], want_len[i], len);
        free(want[i]);
        free(got[i]);
    }
    for (int j = 0; j < M; j++) free(rp[j]);
    free(pad);
    free(file);
}

/* EcSchema::ec_decode of vertical stripes (ec/mod.rs:62-89): R rows whose
 * survivors are the same, every present shard's R cells back to back -> one
 * hec_decode of R * cell bytes; each rebuilt cell == the original. */
static void replay_batched_reader(hec_coder_t *c, size_t cell, size_t R, int lost_a, int lost_b) {
    uint8_t *vert[K + M];
    for (int i = 0; i < K; i++) {
        vert[i] = malloc(R * cell);
        for (size_t b = 0; b < R * cell; b++) vert[i][b] = next_byte();
    }
    for (int j = 0; j < M; j++) vert[K + j] = malloc(R * cell);
    for (size_t r = 0; r < R; r++) { /* parity row by row with the oracle */
        const uint8_t *in[K];
        uint8_t *out[M];
        for (int i = 0; i < K; i++) in[i] = vert[i] + r * cell;
        for (int j = 0; j < M; j++) out[j] = vert[K + j] + r * cell;
        orc_encode(K, M, in, cell, out);
    }
    const uint8_t *sh[K + M];
    uint8_t *out[K + M];
    for (int i = 0; i < K + M; i++) {
        sh[i] = (i == lost_a || i == lost_b) ? NULL : vert[i];
        out[i] = (i < K && !sh[i]) ? malloc(R * cell) : NULL;
    }
    int rc = hec_decode(c, sh, R * cell, out);
    CHECK(rc == HEC_OK, "batched decode %s", hec_strerror(rc));
    for (int i = 0; i < K; i++)
        if (out[i]) {
            CHECK(memcmp(out[i], vert[i], R * cell) == 0, "vertical-stripe decode shard %d", i);
            free(out[i]);
        }
    for (int i = 0; i < K + M; i++) free(vert[i]);
}

/* block_reader.rs StripedBlockStream::read_slice (:480-554), modelled call
 * for call over in-memory shard streams: cell_readers[] in shard order,
 * start_next_reader() opens the next shard at current_block_start (or, for
 * a shard in fail_open, records a failed reader), read_row() takes the first
 * k good cells of a row -- a reader whose DataNode dies at row `die_row`
 * errors there and is dropped ("trying next replica") -- and advances
 * current_block_start past the row; ROWS_PER_CALL rows with equal survivors
 * go to one hec_decode (1: the reference's per-row ec_decode).  The file read
 * back must equal the written one; m + 1 lost shards must end in "Not enough
 * valid shards".  `bug` = 1 advances current_block_start once per call
 * instead of per row (round 4's batched patch): with more than
 * one row per call a reader opened mid-call starts rows behind. */
typedef struct {
    int open;     /* a live reader */
    size_t pos;   /* next cell's byte offset in its shard */
} cell_reader;

typedef struct {
    const uint8_t *shard[K + M];
    size_t rows;
    int fail_open[K + M]; /* start_next_reader records a failed reader */
    long die_row[K + M];  /* next_cell errors when asked for this row (-1: never) */
    cell_reader rd[K + M];
    size_t n_readers, current_block_start, cell;
    int bug;
} stripe_stream;

static int start_next_reader(stripe_stream *st) {
    if (st->n_readers >= K + M) return -1; /* "Not enough valid shards" */
    const size_t i = st->n_readers++;
    st->rd[i].open = !st->fail_open[i];
    st->rd[i].pos = st->current_block_start;
    return st->rd[i].open;
}

/* -> 0 and the row's first k good cells (pointers into the shards), or -1 */
static int read_row(stripe_stream *st, const uint8_t **slice) {
    size_t good = 0;
    for (size_t i = 0; i < st->n_readers; i++) good += st->rd[i].open;
    while (good < K) {
        int r = start_next_reader(st);
        if (r < 0) return -1;
        good += (size_t)r;
    }
    for (int i = 0; i < K + M; i++) slice[i] = NULL;
    size_t cells = 0, b = 0;
    while (cells < K) {
        if (b >= st->n_readers) {
            int r = start_next_reader(st);
            if (r < 0) return -1;
            if (!r) {
                b++;
                continue;
            }
        }
        cell_reader *rd = &st->rd[b];
        if (rd->open) {
            const size_t row = rd->pos / st->cell;
            if (st->die_row[b] >= 0 && row >= (size_t)st->die_row[b]) {
                rd->open = 0; /* "trying next replica" */
            } else {
                slice[b] = st->shard[b] + rd->pos;
                rd->pos += st->cell;
                cells++;
            }
        }
        b++;
    }
    if (!st->bug) st->current_block_start += st->cell;
    return 0;
}

/* the whole block group through read_slice: 1 = the file read back equals
 * the written one, 0 = it differs, -1 = the read failed (not enough shards) */
static int replay_reader_faults(hec_coder_t *c, size_t cell, size_t rows, const int *fail_open,
                                const long *die_row, int bug) {
    uint8_t *sh[K + M];
    for (int i = 0; i < K + M; i++) sh[i] = malloc(rows * cell);
    for (int i = 0; i < K; i++)
        for (size_t b = 0; b < rows * cell; b++) sh[i][b] = next_byte();
    for (size_t r = 0; r < rows; r++) {
        const uint8_t *in[K];
        uint8_t *out[M];
        for (int i = 0; i < K; i++) in[i] = sh[i] + r * cell;
        for (int j = 0; j < M; j++) out[j] = sh[K + j] + r * cell;
        orc_encode(K, M, in, cell, out);
    }
    stripe_stream st;
    memset(&st, 0, sizeof st);
    for (int i = 0; i < K + M; i++) {
        st.shard[i] = sh[i];
        st.fail_open[i] = fail_open ? fail_open[i] : 0;
        st.die_row[i] = die_row ? die_row[i] : -1;
    }
    st.rows = rows;
    st.cell = cell;
    st.bug = bug;
    uint8_t *file = malloc(rows * K * cell), *vert[K + M];
    for (int i = 0; i < K + M; i++) vert[i] = malloc(ROWS_PER_CALL * cell);
    const uint8_t *pending[K + M];
    int have_pending = 0;
    size_t done = 0;
    int ok = 1, failed = 0;
    while (done < rows && ok) {
        const size_t left = rows - (st.current_block_start / cell) + (size_t)have_pending;
        size_t want = left < 1 ? 1 : left > ROWS_PER_CALL ? ROWS_PER_CALL : left;
        if (st.bug) want = rows - done < ROWS_PER_CALL ? rows - done : ROWS_PER_CALL;
        int present[K + M], got = 0;
        size_t n = 0;
        while (n < want) {
            const uint8_t *slice[K + M];
            if (have_pending) {
                memcpy(slice, pending, sizeof slice);
                have_pending = 0;
            } else if (read_row(&st, slice) != 0) {
                ok = 0;
                failed = 1;
                break;
            }
            int same = 1;
            for (int i = 0; i < K + M; i++) same &= !got || present[i] == (slice[i] != NULL);
            if (!same) {
                memcpy(pending, slice, sizeof slice);
                have_pending = 1;
                break;
            }
            for (int i = 0; i < K + M; i++) {
                present[i] = slice[i] != NULL;
                if (slice[i]) memcpy(vert[i] + n * cell, slice[i], cell);
            }
            got = 1;
            n++;
        }
        if (!ok || !n) break;
        if (st.bug) st.current_block_start += n * cell;
        /* ec_decode of the vertical stripes: rebuild missing data, split into rows */
        const uint8_t *in[K + M];
        uint8_t *out[K + M];
        for (int i = 0; i < K + M; i++) {
            in[i] = present[i] ? vert[i] : NULL;
            out[i] = (i < K && !present[i]) ? vert[i] : NULL;
        }
        if (hec_decode(c, in, n * cell, out) != HEC_OK) {
            ok = 0;
            failed = 1;
            break;
        }
        for (size_t r = 0; r < n; r++)
            for (int i = 0; i < K; i++) memcpy(file + ((done + r) * K + i) * cell, vert[i] + r * cell, cell);
        done += n;
    }
    for (size_t r = 0; ok && r < rows; r++)
        for (int i = 0; i < K; i++) ok &= memcmp(file + (r * K + i) * cell, sh[i] + r * cell, cell) == 0;
    for (int i = 0; i < K + M; i++) {
        free(sh[i]);
        free(vert[i]);
    }
    free(file);
    return failed ? -1 : ok;
}

static void replay_reader_fault_cases(hec_coder_t *c) {
    const size_t cell = 4096, rows = 9;
    const long none[K + M] = {-1, -1, -1, -1, -1, -1, -1, -1, -1};
    long die[K + M];
    int fopen_[K + M] = {0};
    CHECK(replay_reader_faults(c, cell, rows, NULL, none, 0) == 1, "striped reader, no faults");
    /* shard 1's DataNode dies at row 2: rows 0-1 from shards 0..5, rows 2..
     * from 0,2..6 (parity 0 opened at row 2) -- the ADVICE r04 case */
    memcpy(die, none, sizeof die);
    die[1] = 2;
    CHECK(replay_reader_faults(c, cell, rows, NULL, die, 0) == 1, "shard 1 dies at row 2");
    if (ROWS_PER_CALL > 1)
        CHECK(replay_reader_faults(c, cell, rows, NULL, die, 1) == 0, "per-call advance misreads a mid-call death");
    /* two deaths in different batches, and one at the batch boundary */
    die[1] = 2;
    die[4] = 5;
    CHECK(replay_reader_faults(c, cell, rows, NULL, die, 0) == 1, "shards 1 and 4 die at rows 2 and 5");
    memcpy(die, none, sizeof die);
    die[0] = 4;
    CHECK(replay_reader_faults(c, cell, rows, NULL, die, 0) == 1, "shard 0 dies at row 4 (a batch boundary)");
    /* fault-injected open failures (EC_FAULT_INJECTOR fail_blocks) plus a death */
    fopen_[2] = 1;
    memcpy(die, none, sizeof die);
    die[3] = 1;
    CHECK(replay_reader_faults(c, cell, rows, fopen_, die, 0) == 1, "shard 2 never opens, shard 3 dies at row 1");
    /* m + 1 lost: Not enough valid shards, never a wrong file */
    die[4] = 6;
    die[5] = 7;
    CHECK(replay_reader_faults(c, cell, rows, fopen_, die, 0) == -1, "m + 1 lost shards: Not enough valid shards");
}

/* What needs no GPU: Coder::new's host-only fallback, decode over the first
 * k present shards only, and the writer / reader sequences on it. */
static void host_only_replay(void) {
    hec_coder_t *h = NULL;
    int rc = hec_coder_acquire("rs", K, M, HEC_DEVICE_HOST, &h);
    CHECK(rc == HEC_OK && hec_coder_device(h) == HEC_DEVICE_HOST, "host-only acquire %s", hec_strerror(rc));
    if (rc != HEC_OK) return;
    /* a present shard past the first k may differ in length (never read):
     * survivors 0,2,3,4,5,6 (n bytes); shard 7 is 1 byte long */
    const size_t n = 3000;
    uint8_t *d[K], *p[M], *rec = malloc(n), *stub = malloc(1);
    for (int i = 0; i < K; i++) {
        d[i] = malloc(n);
        for (size_t b = 0; b < n; b++) d[i][b] = next_byte();
    }
    for (int j = 0; j < M; j++) p[j] = malloc(n);
    CHECK(hec_encode(h, (const uint8_t *const *)d, n, p) == HEC_OK, "host-only encode");
    const uint8_t *sh[K + M] = {d[0], NULL, d[2], d[3], d[4], d[5], p[0], stub, NULL};
    uint8_t *out[K + M] = {NULL, rec, NULL, NULL, NULL, NULL, NULL, NULL, NULL};
    CHECK(hec_decode(h, sh, n, out) == HEC_OK && memcmp(rec, d[1], n) == 0, "decode over the first k present");
    for (int i = 0; i < K; i++) free(d[i]);
    for (int j = 0; j < M; j++) free(p[j]);
    free(rec);
    free(stub);
    /* the reference's writer / reader sequences on the host-only coder */
    const size_t cell = 4096;
    const size_t lens[] = {1, 100, cell - 1, cell, K * cell - 4, K * cell, 3 * K * cell + 7, 4 * K * cell,
                           4 * K * cell + 1, 9 * K * cell + 2 * cell + 5};
    for (size_t t = 0; t < sizeof lens / sizeof lens[0]; t++) replay_batched_writer(h, cell, lens[t]);
    replay_batched_reader(h, cell, ROWS_PER_CALL, 0, 4);
    replay_batched_reader(h, cell, 3, 1, 2);
    replay_reader_fault_cases(h);
    hec_coder_release(h);
    (void)hec_coder_pool_trim();
    printf("host-only replay %s\n", failures ? "FAILED" : "ok");
}

/* The patch's `mi355x` Criterion group of rust/benches/ec.rs (bench_mi355x),
 * call for call: GpuCoder::new -> hec_coder_create_codec; DeviceBuffer::upload
 * / new -> hec_device_alloc + hec_device_copy; the reference bench's six
 * 16 MiB slices (big-endian i32 counters, v + i * slice_size) in one HBM
 * image; encode_device + synchronize -> hec_encode_device (1 stripe, default
 * stream) + hec_device_synchronize; decode with 1, 2, 3 data slices missing
 * -> hec_decode_device + hec_device_synchronize; DeviceBuffer::download ->
 * hec_device_copy.  Parity against the oracle, rebuilt slices against the
 * originals; each leg timed over its iterations (Criterion's Throughput::
 * Bytes(slice_size * 6)). */
static void replay_bench_device(void) {
    enum { SLICE = 16 << 20, ENC_IT = 30, DEC_IT = 10 };
    hec_coder_t *c = NULL;
    int rc = hec_coder_create_codec("rs", K, M, 0, &c);
    CHECK(rc == HEC_OK, "bench coder %s", hec_strerror(rc));
    if (rc != HEC_OK) return;
    uint8_t *host = malloc((size_t)K * SLICE), *hpar = malloc((size_t)M * SLICE), *want[M];
    for (int i = 0; i < K; i++)
        for (uint32_t v = 0; v < SLICE / 4; v++) {
            const uint32_t x = v + (uint32_t)i * SLICE; /* put_i32: big-endian */
            uint8_t *q = host + (size_t)i * SLICE + 4 * (size_t)v;
            q[0] = (uint8_t)(x >> 24), q[1] = (uint8_t)(x >> 16), q[2] = (uint8_t)(x >> 8), q[3] = (uint8_t)x;
        }
    const uint8_t *hin[K];
    for (int i = 0; i < K; i++) hin[i] = host + (size_t)i * SLICE;
    for (int j = 0; j < M; j++) want[j] = malloc(SLICE);
    CHECK(orc_encode(K, M, hin, SLICE, want) == 0, "oracle encode of the bench slices");
    void *data = NULL, *parity = NULL, *rebuilt = NULL;
    CHECK(hec_device_alloc(0, (size_t)K * SLICE, 0, &data) == HEC_OK, "alloc data");
    CHECK(hec_device_alloc(0, (size_t)M * SLICE, 0, &parity) == HEC_OK, "alloc parity");
    CHECK(hec_device_alloc(0, (size_t)M * SLICE, 0, &rebuilt) == HEC_OK, "alloc rebuilt");
    if (data && parity && rebuilt) {
        CHECK(hec_device_copy(0, data, host, (size_t)K * SLICE) == HEC_OK, "upload");
        const uint8_t *d[K];
        uint8_t *p[M];
        size_t strides[K + M];
        for (int i = 0; i < K; i++) d[i] = (const uint8_t *)data + (size_t)i * SLICE;
        for (int j = 0; j < M; j++) p[j] = (uint8_t *)parity + (size_t)j * SLICE;
        for (int i = 0; i < K + M; i++) strides[i] = (size_t)(K + M) * SLICE; /* one stripe: any stride */
        double t0 = now_us();
        for (int it = 0; it < ENC_IT; it++) {
            rc = hec_encode_device(c, d, strides, p, strides, SLICE, 1, NULL);
            if (rc == HEC_OK) rc = hec_device_synchronize(0, NULL);
            if (rc != HEC_OK) break;
        }
        const double enc_us = (now_us() - t0) / ENC_IT;
        CHECK(rc == HEC_OK, "encode_device %s", hec_strerror(rc));
        CHECK(hec_device_copy(0, hpar, parity, (size_t)M * SLICE) == HEC_OK, "download parity");
        for (int j = 0; j < M; j++) CHECK(memcmp(hpar + (size_t)j * SLICE, want[j], SLICE) == 0, "bench parity %d", j);
        double dec_us[4] = {0};
        for (int lost = 1; lost <= 3; lost++) {
            const uint8_t *sh[K + M];
            uint8_t *out[K];
            for (int i = 0; i < K + M; i++) sh[i] = i < lost ? NULL : (i < K ? d[i] : p[i - K]);
            for (int i = 0; i < K; i++) out[i] = i < lost ? (uint8_t *)rebuilt + (size_t)i * SLICE : NULL;
            t0 = now_us();
            for (int it = 0; it < DEC_IT; it++) {
                rc = hec_decode_device(c, sh, strides, out, strides, SLICE, 1, NULL);
                if (rc == HEC_OK) rc = hec_device_synchronize(0, NULL);
                if (rc != HEC_OK) break;
            }
            dec_us[lost] = (now_us() - t0) / DEC_IT;
            CHECK(rc == HEC_OK, "decode_device (%d lost) %s", lost, hec_strerror(rc));
            CHECK(hec_device_copy(0, hpar, rebuilt, (size_t)lost * SLICE) == HEC_OK, "download rebuilt");
            CHECK(memcmp(hpar, host, (size_t)lost * SLICE) == 0, "decode-%d-slice: rebuilt != originals", lost);
        }
        const double gib = (double)K * SLICE / (1024.0 * 1024.0 * 1024.0);
        printf("bench ec.rs mi355x group (6 x 16 MiB, device-resident, per iteration incl. sync): "
               "encode %.1f us = %.1f GiB/s; decode-1/2/3-slice %.1f / %.1f / %.1f us = %.1f / %.1f / %.1f GiB/s\n",
               enc_us, gib / (enc_us * 1e-6), dec_us[1], dec_us[2], dec_us[3], gib / (dec_us[1] * 1e-6),
               gib / (dec_us[2] * 1e-6), gib / (dec_us[3] * 1e-6));
    }
    hec_device_free(0, data);
    hec_device_free(0, parity);
    hec_device_free(0, rebuilt);
    hec_coder_destroy(c);
    free(host);
    free(hpar);
    for (int j = 0; j < M; j++) free(want[j]);
}

int main(void) {
    CHECK(hec_abi_version() == 5, "ABI %d", hec_abi_version());
    host_only_replay();
    hec_coder_t *c = NULL;
    int rc = hec_coder_create_codec("rs", K, M, 0, &c);
    if (rc != HEC_OK) {
        fprintf(stderr, "coder create: %s (%s)\n", hec_strerror(rc), hec_last_error());
        return failures ? 1 : 2;
    }
    hec_coder_t *bad = NULL;
    CHECK(hec_coder_create_codec("lrc", K, M, 0, &bad) == HEC_ERR_UNSUPPORTED_CODEC && bad == NULL,
          "an unknown codec must be UnsupportedErasureCodingPolicy");

    const size_t n = (1u << 20) + 5; /* a full cell plus a tail the 16-B kernels do not cover */
    uint8_t *data[K], *par[M], *want[M];
    for (int i = 0; i < K; i++) {
        data[i] = malloc(n);
        for (size_t b = 0; b < n; b++) data[i][b] = next_byte();
    }
    for (int j = 0; j < M; j++) {
        par[j] = malloc(n);
        want[j] = malloc(n);
    }
    CHECK(orc_encode(K, M, (const uint8_t *const *)data, n, want) == 0, "oracle encode");

    /* GpuCoder::encode: zero length is the reference's panic, a status here */
    CHECK(hec_encode(c, (const uint8_t *const *)data, 0, par) == HEC_ERR_INVALID_ARG, "n == 0");
    rc = hec_encode(c, (const uint8_t *const *)data, n, par);
    CHECK(rc == HEC_OK, "encode %s", hec_strerror(rc));
    for (int j = 0; j < M; j++) CHECK(memcmp(par[j], want[j], n) == 0, "parity %d != oracle", j);

    /* GpuCoder::decode: data 0..2 missing; out slots of present shards and of
     * parity hold sentinels that must not change */
    uint8_t *shards[K + M], *out[K + M];
    uint8_t *sentinel = malloc(n);
    memset(sentinel, 0xCC, n);
    for (int i = 0; i < K + M; i++) {
        shards[i] = i < 3 ? NULL : (i < K ? data[i] : par[i - K]);
        out[i] = malloc(n);
        memcpy(out[i], sentinel, n);
    }
    rc = hec_decode(c, (const uint8_t *const *)shards, n, out);
    CHECK(rc == HEC_OK, "decode %s", hec_strerror(rc));
    for (int i = 0; i < K + M; i++) {
        if (i < 3)
            CHECK(memcmp(out[i], data[i], n) == 0, "rebuilt data %d", i);
        else
            CHECK(memcmp(out[i], sentinel, n) == 0, "slot %d written (must be untouched)", i);
    }

    /* data 0,1 and parity 0 missing: parity is never regenerated
     * (gf256.rs:96-97); survivors 2,3,4,5,7,8 */
    shards[2] = data[2];
    shards[K] = NULL;
    for (int i = 0; i < K + M; i++) memcpy(out[i], sentinel, n);
    rc = hec_decode(c, (const uint8_t *const *)shards, n, out);
    CHECK(rc == HEC_OK, "decode with a parity missing %s", hec_strerror(rc));
    CHECK(memcmp(out[K], sentinel, n) == 0, "missing parity slot written");
    CHECK(memcmp(out[2], sentinel, n) == 0, "present data slot written");
    for (int i = 0; i < 2; i++) CHECK(memcmp(out[i], data[i], n) == 0, "rebuilt data %d (parity missing)", i);

    /* 4 missing of RS(6,3): the shim's ErasureCodingError("Not enough valid shards") */
    shards[3] = NULL;
    rc = hec_decode(c, (const uint8_t *const *)shards, n, out);
    CHECK(rc == HEC_ERR_NOT_ENOUGH_SHARDS, "4 missing -> %d", rc);
    CHECK(strstr(hec_strerror(rc), "Not enough valid shards") != NULL, "message");

    /* nothing missing: Ok, no write (gf256.rs:102-105) */
    for (int i = 0; i < K; i++) shards[i] = data[i];
    for (int j = 0; j < M; j++) shards[K + j] = NULL;
    memcpy(out[0], sentinel, n);
    CHECK(hec_decode(c, (const uint8_t *const *)shards, n, out) == HEC_OK, "no-op decode");
    CHECK(memcmp(out[0], sentinel, n) == 0, "no-op decode wrote");

    /* encode_rows / decode_rows: R rows of 64 KiB cells in file order */
    enum { R = 5 };
    const size_t cell = 65536;
    uint8_t *rows = malloc(R * K * cell), *rpar = malloc(R * M * cell), *file = malloc(R * K * cell);
    for (size_t b = 0; b < R * K * cell; b++) rows[b] = next_byte();
    rc = hec_encode_host_batch(c, rows, rpar, cell, R, 2);
    CHECK(rc == HEC_OK, "encode_rows %s", hec_strerror(rc));
    for (int r = 0; r < R; r++) {
        const uint8_t *rin[K];
        uint8_t *rout[M];
        for (int i = 0; i < K; i++) rin[i] = rows + (r * K + i) * cell;
        for (int j = 0; j < M; j++) rout[j] = want[j];
        orc_encode(K, M, rin, cell, rout);
        for (int j = 0; j < M; j++) CHECK(memcmp(rpar + (r * M + j) * cell, want[j], cell) == 0, "row %d parity %d", r, j);
    }
    uint8_t *vert[K + M];
    for (int i = 0; i < K + M; i++) {
        vert[i] = malloc(R * cell);
        for (int r = 0; r < R; r++)
            memcpy(vert[i] + r * cell, i < K ? rows + (r * K + i) * cell : rpar + (r * M + i - K) * cell, cell);
    }
    const uint8_t *vin[K + M];
    for (int i = 0; i < K + M; i++) vin[i] = (i == 1 || i == 4) ? NULL : vert[i];
    rc = hec_decode_host_batch(c, vin, cell, R, file, 2);
    CHECK(rc == HEC_OK, "decode_rows %s", hec_strerror(rc));
    CHECK(memcmp(file, rows, R * K * cell) == 0, "decode_rows file order");

    /* GpuGroup over device 0 twice: same rows, same parity */
    hec_group_t *g = NULL;
    const int devs[2] = {0, 0};
    rc = hec_group_create("rs", K, M, devs, 2, &g);
    CHECK(rc == HEC_OK, "group %s", hec_strerror(rc));
    if (rc == HEC_OK) {
        uint8_t *gpar = malloc(R * M * cell);
        CHECK(hec_group_encode_host_batch(g, rows, gpar, cell, R, 2) == HEC_OK, "group encode_rows");
        CHECK(memcmp(gpar, rpar, R * M * cell) == 0, "group parity");
        memset(file, 0, R * K * cell);
        CHECK(hec_group_decode_host_batch(g, vin, cell, R, file, 2) == HEC_OK, "group decode_rows");
        CHECK(memcmp(file, rows, R * K * cell) == 0, "group file order");
        free(gpar);
        hec_group_destroy(g);
    }

    /* Coder::new per row (ec/mod.rs:71, block_writer.rs:787) through the pool:
     * 10,000 acquire / encode / release cycles of a 4 KiB row (the host
     * small-row path), each checked against the oracle every 1000th cycle;
     * then the same cost with create / destroy instead, and one
     * device-routed call of the same row (host limit 0) for scale */
    {
        enum { CYCLES = 10000, SMALL = 4096 };
        const uint8_t *sin[K];
        uint8_t *sout[M], *swant[M];
        for (int i = 0; i < K; i++) sin[i] = data[i];
        for (int j = 0; j < M; j++) {
            sout[j] = malloc(SMALL);
            swant[j] = malloc(SMALL);
        }
        orc_encode(K, M, sin, SMALL, swant);
        hec_coder_t *first = NULL;
        double t0 = now_us();
        for (int it = 0; it < CYCLES; it++) {
            hec_coder_t *pc = NULL;
            rc = hec_coder_acquire("rs", K, M, 0, &pc);
            if (rc != HEC_OK) {
                CHECK(0, "acquire %s", hec_strerror(rc));
                break;
            }
            if (it == 0) first = pc;
            rc = hec_encode(pc, sin, SMALL, sout);
            if (rc != HEC_OK || it % 1000 == 0)
                for (int j = 0; j < M; j++) CHECK(rc == HEC_OK && memcmp(sout[j], swant[j], SMALL) == 0, "pooled encode %d", it);
            hec_coder_release(pc);
        }
        const double pooled_us = (now_us() - t0) / CYCLES;
        hec_coder_t *again = NULL;
        CHECK(hec_coder_acquire("rs", K, M, 0, &again) == HEC_OK && again == first, "the pool hands the idle coder back");
        hec_coder_release(again);
        t0 = now_us();
        for (int it = 0; it < CYCLES; it++) {
            hec_coder_t *pc = NULL;
            hec_coder_acquire("rs", K, M, 0, &pc);
            hec_coder_release(pc);
        }
        const double cycle_us = (now_us() - t0) / CYCLES;
        enum { FRESH = 50 };
        t0 = now_us();
        for (int it = 0; it < FRESH; it++) {
            hec_coder_t *fc = NULL;
            CHECK(hec_coder_create_codec("rs", K, M, 0, &fc) == HEC_OK, "create");
            hec_encode(fc, sin, SMALL, sout);
            hec_coder_destroy(fc);
        }
        const double fresh_us = (now_us() - t0) / FRESH;
        hec_coder_set_host_limit(c, 0); /* this row through the device, for scale */
        hec_encode(c, sin, SMALL, sout);
        t0 = now_us();
        for (int it = 0; it < 100; it++) hec_encode(c, sin, SMALL, sout);
        const double device_us = (now_us() - t0) / 100;
        for (int j = 0; j < M; j++) CHECK(memcmp(sout[j], swant[j], SMALL) == 0, "device-routed encode");
        printf("pool: acquire+encode(4 KiB)+release %.2f us/cycle, acquire+release %.3f us, "
               "create+encode+destroy %.1f us, device-routed encode %.1f us, host isa %s\n",
               pooled_us, cycle_us, fresh_us, device_us, hec_host_isa());
        CHECK(pooled_us <= device_us, "a pooled cycle must cost less than one device-routed call");
        CHECK(hec_coder_pool_trim() >= 1, "trim");
        for (int j = 0; j < M; j++) {
            free(sout[j]);
            free(swant[j]);
        }
    }

    /* the writer / reader sequences through the device (1 MiB cells, host
     * limit 256 KiB: every row takes the device route) */
    hec_coder_set_host_limit(c, 256 << 10);
    replay_batched_writer(c, 1 << 20, 4 * K * (1 << 20) + 3 * (1 << 20) + 11);
    replay_batched_reader(c, 1 << 20, ROWS_PER_CALL, 0, 1);

    replay_bench_device();

    hec_coder_destroy(c);
    for (int i = 0; i < K; i++) free(data[i]);
    for (int j = 0; j < M; j++) {
        free(par[j]);
        free(want[j]);
    }
    for (int i = 0; i < K + M; i++) {
        free(out[i]);
        free(vert[i]);
    }
    free(sentinel);
    free(rows);
    free(rpar);
    free(file);
    if (failures) {
        fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    printf("shim replay ok\n");
    return 0;
}
