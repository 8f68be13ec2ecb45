/* asan_capi.c -- host-side AddressSanitizer + LeakSanitizer run over the C
 * ABI paths that need no GPU: every coding matrix up to RS(32,16), the
 * inversion, the decode plan of all 2^14 presence masks of RS(10,4), and the
 * coder / group creation failure paths (no device in the container: each
 * must return a status and leak nothing), and a host-only coder
 * (HEC_DEVICE_HOST) through every host call.  Built and run by
 * scripts/asan_host.sh (tests/test_capi.py).  Device code is not sanitized
 * (no GPU ASan on this pool). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "hdfs_ec_amd.h"
int main(void) {
    uint8_t m[14 * 10];
    int bad = 0;
    for (size_t k = 1; k <= 32; k++)
        for (size_t p = 1; p <= 16; p++) {
            uint8_t buf[48 * 32];
            if (hec_gen_rs_matrix(k, p, buf) != HEC_OK) bad++;
        }
    if (hec_gen_rs_matrix(10, 4, m) != HEC_OK) bad++;
    uint8_t sub[100];
    memcpy(sub, m + 40, 60);      /* rows 4..9 (identity part) */
    memcpy(sub + 60, m + 100, 40); /* + parity rows 10..13: a decodable 10 x 10 submatrix */
    int rc = hec_matrix_invert(sub, 10);
    uint8_t present[14]; size_t e, surv[10], miss[10]; uint8_t mat[100];
    for (unsigned mask = 0; mask < (1u << 14); mask++) {
        for (int i = 0; i < 14; i++) present[i] = (mask >> i) & 1;
        int r = hec_decode_plan(10, 4, present, &e, surv, miss, mat);
        if (r != HEC_OK && r != HEC_ERR_NOT_ENOUGH_SHARDS) bad++;
    }
    hec_group_t* g = 0; int devs[2] = {0, 0};
    if (hec_group_create("rs", 6, 3, devs, 0, &g) != HEC_ERR_INVALID_ARG) bad++;
    (void)hec_group_create("rs", 6, 3, devs, 2, &g);  /* no GPU here: a status, never a crash */
    hec_group_destroy(g);
    hec_coder_t* c = 0;
    (void)hec_coder_create(6, 3, 0, &c);
    hec_coder_destroy(c);
    /* pool: no device -> acquire(-1) hands out a host-only coder; a double
     * release is ignored; trim frees it */
    c = 0;
    if (hec_coder_acquire("rs", 6, 3, -1, &c) != HEC_OK || hec_coder_device(c) != HEC_DEVICE_HOST) bad++;
    hec_coder_release(c);
    hec_coder_release(c);
    if (hec_coder_pool_trim() != 1) bad++;
    /* a host-only coder end to end: rows, host batches (file-order decode),
     * the short-row file calls, and the device calls as statuses */
    {
        enum { K = 6, P = 3, CELL = 4099, S = 3 };
        hec_coder_t* h = 0;
        if (hec_coder_create_codec("rs", K, P, HEC_DEVICE_HOST, &h) != HEC_OK) bad++;
        uint8_t* data = (uint8_t*)malloc(S * K * CELL);
        uint8_t* par = (uint8_t*)malloc(S * P * CELL);
        uint8_t* file = (uint8_t*)malloc(S * K * CELL);
        for (size_t b = 0; b < (size_t)S * K * CELL; b++) data[b] = (uint8_t)(b * 131 + 7);
        if (hec_encode_host_batch(h, data, par, CELL, S, 2) != HEC_OK) bad++;
        uint8_t* vert[K + P];
        for (int i = 0; i < K + P; i++) {
            vert[i] = (uint8_t*)malloc(S * CELL);
            for (int s = 0; s < S; s++)
                memcpy(vert[i] + s * CELL, i < K ? data + (s * K + i) * CELL : par + (s * P + i - K) * CELL, CELL);
        }
        const uint8_t* vin[K + P];
        size_t vlen[K + P];
        for (int i = 0; i < K + P; i++) {
            vin[i] = (i == 1 || i == 5) ? 0 : vert[i];
            vlen[i] = S * CELL;
        }
        if (hec_decode_host_batch(h, vin, CELL, S, file, 2) != HEC_OK || memcmp(file, data, S * K * CELL)) bad++;
        memset(file, 0, S * K * CELL);
        if (hec_decode_rows_host(h, vin, vlen, CELL, file, S * K * CELL - 5, 2) != HEC_OK ||
            memcmp(file, data, S * K * CELL - 5)) bad++;
        if (hec_encode_rows_host(h, data, S * K * CELL - 4000, par, CELL, 2) != HEC_OK) bad++;
        const uint8_t* rin[K];
        uint8_t* rout[P];
        for (int i = 0; i < K; i++) rin[i] = data + i * CELL;
        for (int j = 0; j < P; j++) rout[j] = par + j * CELL;
        if (hec_encode(h, rin, CELL, rout) != HEC_OK) bad++;
        /* decode reads only the first k present shards (matrix.rs:212-216):
         * a present shard past them may be shorter -- here a 1-byte heap
         * block, which ASan would flag if the engine touched its row */
        {
            uint8_t *stub = (uint8_t *)malloc(1), *rec = (uint8_t *)malloc(CELL);
            const uint8_t *sh[K + P];
            uint8_t *out[K + P];
            for (int i = 0; i < K + P; i++) {
                sh[i] = i == 1 ? 0 : (i < K ? data + i * CELL : par + (i - K) * CELL);
                out[i] = 0;
            }
            sh[K + 1] = stub;
            out[1] = rec;
            if (hec_decode(h, sh, CELL, out) != HEC_OK || memcmp(rec, data + CELL, CELL)) bad++;
            free(stub);
            free(rec);
        }
        size_t st[K + P] = {0};
        if (hec_encode_device(h, rin, st, rout, st, CELL, 1, 0) != HEC_ERR_DEVICE) bad++;
        for (int i = 0; i < K + P; i++) free(vert[i]);
        free(data);
        free(par);
        free(file);
        hec_coder_destroy(h);
    }
    /* the host small-row routine over exact-size heap buffers (every tail
     * length up to 200 and a 64 KiB + 5 row): no access past the shards */
    for (size_t n = 1; n < 200 || n == 65541; n = n < 199 ? n + 1 : (n == 199 ? 65541 : 0)) {
        const uint8_t* in[10];
        uint8_t* out[4];
        for (int i = 0; i < 10; i++) {
            uint8_t* p = (uint8_t*)malloc(n);
            for (size_t b = 0; b < n; b++) p[b] = (uint8_t)(b * 7 + i);
            in[i] = p;
        }
        for (int j = 0; j < 4; j++) out[j] = (uint8_t*)malloc(n);
        if (hec_gf_matmul_host(m + 100, 4, 10, in, out, n) != HEC_OK) bad++;
        for (int i = 0; i < 10; i++) free((void*)in[i]);
        for (int j = 0; j < 4; j++) free(out[j]);
        if (n == 65541) break;
    }
    printf("invert rc=%d bad=%d host_isa=%s last_error=%s\n", rc, bad, hec_host_isa(), hec_last_error());
    return bad != 0;
}
