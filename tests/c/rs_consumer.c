/* A plain C99 consumer of include/rs_amd.h — what a cgo / FFI caller sees.
 *
 * Built by tests/test_c_consumer.py with `gcc -std=c99 -pedantic -Werror`
 * (and as C++ with g++) against librsamd.so.
 *
 *   rs_consumer host   checks that need no GPU: error text, KATs of the
 *                      reference (rs_test.go:26-49 via the generator matrix,
 *                      matrix_test.go:45-134, rs_test.go:139-163), argument
 *                      checks in the reference's order (rs.go)
 *   rs_consumer gpu    the Go-API shaped calls on host memory: Encode vs a
 *                      naive product built from rs_gen_matrix + rs_gf_mul,
 *                      Reconst of every 1..4-erasure pattern of 10+4, Update
 *                      and Replace against re-encoding (rs_test.go:165-331)
 *
 * Exit status 0 = all checks passed; otherwise the first failure is printed.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rs_amd.h"

static int g_fail = 0;
#define CHECK(cond)                                                                 \
    do {                                                                            \
        if (!(cond)) {                                                              \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond); \
            g_fail = 1;                                                             \
            return 1;                                                               \
        }                                                                           \
    } while (0)

static uint64_t g_state = 0x5EEDull;
static uint8_t next_byte(void) {
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint8_t)(z ^ (z >> 31));
}
static void fill(uint8_t* p, size_t n) {
    size_t i;
    for (i = 0; i < n; ++i) p[i] = next_byte();
}

static int host_checks(void) {
    static const uint8_t row0_10_4[10] = {221, 152, 173, 157, 93, 150, 61, 170, 142, 244}; /* SURVEY 8a a1 */
    static const uint8_t kat_in[5] = {0, 4, 2, 6, 8}, kat_out[5] = {97, 173, 218, 107, 110}; /* rs_test.go:26-49 */
    /* TestMatrixInvert KATs, matrix_test.go:45-134 */
    static const uint8_t m3[9] = {56, 23, 98, 3, 100, 200, 45, 201, 123};
    static const uint8_t m3_inv[9] = {175, 133, 33, 130, 13, 245, 112, 35, 126};
    static const uint8_t singular[4] = {4, 2, 12, 6}, not_square[3] = {7, 8, 9};
    uint8_t gen[25], inv[9];
    int surv[3] = {0, 1, 2}, code, i, j;
    rs_t* rs = NULL;
    size_t lens[14];
    uint8_t* vects[14];

    CHECK(rs_version() >= 100);
    CHECK(strcmp(rs_strerror(RS_OK), "") == 0 || rs_strerror(RS_OK) != NULL);
    CHECK(strcmp(rs_strerror(RS_ERR_TOO_MANY_LOST), "too many lost") == 0);
    CHECK(strcmp(rs_strerror(RS_ERR_SINGULAR_MATRIX), "matrix is singular") == 0);
    for (code = 0; code <= 15; ++code) CHECK(rs_strerror(code) != NULL);

    CHECK(rs_new(0, 4, -1, &rs) == RS_ERR_ILLEGAL_VECTS && rs == NULL);
    CHECK(rs_new(200, 57, -1, &rs) == RS_ERR_ILLEGAL_VECTS);
    CHECK(rs_new(10, 4, -1, &rs) == RS_OK && rs != NULL);
    CHECK(rs_data_num(rs) == 10 && rs_parity_num(rs) == 4);
    {
        uint8_t g[40];
        CHECK(rs_gen_matrix(rs, g) == RS_OK);
        CHECK(memcmp(g, row0_10_4, 10) == 0);
    }
    rs_free(rs);

    /* TestRS_mul: 5+5, one byte per vector, via the generator matrix and rs_gf_mul */
    CHECK(rs_new(5, 5, -1, &rs) == RS_OK);
    CHECK(rs_gen_matrix(rs, gen) == RS_OK);
    for (j = 0; j < 5; ++j) {
        uint8_t acc = 0;
        for (i = 0; i < 5; ++i) acc ^= rs_gf_mul(gen[j * 5 + i], kat_in[i]);
        CHECK(acc == kat_out[j]);
    }
    rs_free(rs);

    CHECK(rs_matrix_invert(m3, 9, 3, inv) == RS_OK && memcmp(inv, m3_inv, 9) == 0);
    CHECK(rs_matrix_invert(singular, 4, 2, inv) == RS_ERR_SINGULAR_MATRIX);
    CHECK(rs_matrix_invert(not_square, 3, 2, inv) == RS_ERR_NOT_SQUARE);
    CHECK(rs_inverse_cache_key(surv, 3) == 7u); /* rs_test.go:139-163 */

    /* argument checks run before any device work, in the reference's order */
    CHECK(rs_new(10, 4, -1, &rs) == RS_OK);
    for (i = 0; i < 14; ++i) {
        lens[i] = 64;
        vects[i] = NULL;
    }
    CHECK(rs_encode(rs, vects, lens, 13) == RS_ERR_MISMATCH_VECTS);  /* rs.go:113-117 */
    lens[3] = 0; /* only vects[0] is tested for zero size (rs.go:124-127) */
    CHECK(rs_encode(rs, vects, lens, 14) == RS_ERR_MISMATCH_VECT_SIZE);
    lens[0] = 0;
    CHECK(rs_encode(rs, vects, lens, 14) == RS_ERR_ZERO_VECT_SIZE);
    lens[0] = lens[3] = 64;
    {
        int need5[5] = {0, 1, 2, 3, 4};
        CHECK(rs_reconst(rs, vects, lens, 14, NULL, 0, need5, 5) == RS_ERR_TOO_MANY_LOST);
    }
    CHECK(rs_update(rs, vects[0], 64, vects[1], 64, 10, vects + 10, lens + 10, 4) == RS_ERR_ILLEGAL_VECT_INDEX);
    rs_free(rs);
    return 0;
}

static int gpu_checks(void) {
    enum { D = 10, P = 4, N = D + P, L = 8192 + 3 };
    uint8_t* buf = (uint8_t*)malloc((size_t)N * L * 3);
    uint8_t *ref = buf, *work = buf + (size_t)N * L, *exp = buf + (size_t)2 * N * L;
    uint8_t gen[P * D];
    uint8_t* v[N];
    size_t lens[N];
    rs_t* rs = NULL;
    int i, j, k, npat = 0;
    size_t b;

    CHECK(buf != NULL);
    CHECK(rs_device_count() >= 1);
    CHECK(rs_new(D, P, -1, &rs) == RS_OK);
    CHECK(rs_gen_matrix(rs, gen) == RS_OK);
    fill(ref, (size_t)D * L);
    memset(ref + (size_t)D * L, 0xA5, (size_t)P * L);
    for (i = 0; i < N; ++i) {
        v[i] = ref + (size_t)i * L;
        lens[i] = L;
    }
    CHECK(rs_encode(rs, v, lens, N) == RS_OK);
    for (j = 0; j < P; ++j)
        for (b = 0; b < L; ++b) {
            uint8_t acc = 0;
            for (i = 0; i < D; ++i) acc ^= rs_gf_mul(gen[j * D + i], ref[(size_t)i * L + b]);
            CHECK(ref[(size_t)(D + j) * L + b] == acc);
        }

    /* every 1..4-erasure pattern, garbage in the lost vectors */
    for (k = 1; k <= P; ++k) {
        int idx[P];
        for (i = 0; i < k; ++i) idx[i] = i;
        for (;;) {
            memcpy(work, ref, (size_t)N * L);
            for (i = 0; i < k; ++i) memset(work + (size_t)idx[i] * L, 0x3C + i, L);
            for (i = 0; i < N; ++i) v[i] = work + (size_t)i * L;
            CHECK(rs_reconst(rs, v, lens, N, NULL, 0, idx, k) == RS_OK);
            CHECK(memcmp(work, ref, (size_t)N * L) == 0);
            ++npat;
            for (i = k - 1; i >= 0 && idx[i] == N - k + i; --i) {}
            if (i < 0) break;
            ++idx[i];
            for (j = i + 1; j < k; ++j) idx[j] = idx[j - 1] + 1;
        }
    }
    CHECK(npat == 14 + 91 + 364 + 1001);

    /* Update row 3 == re-encode with the new data (rs_test.go:219-266) */
    memcpy(work, ref, (size_t)N * L);
    memcpy(exp, ref, (size_t)N * L);
    fill(exp + (size_t)3 * L, L);
    for (i = 0; i < N; ++i) v[i] = exp + (size_t)i * L;
    CHECK(rs_encode(rs, v, lens, N) == RS_OK);
    for (i = 0; i < N; ++i) v[i] = work + (size_t)i * L;
    CHECK(rs_update(rs, work + (size_t)3 * L, L, exp + (size_t)3 * L, L, 3, v + D, lens + D, P) == RS_OK);
    CHECK(memcmp(work + (size_t)D * L, exp + (size_t)D * L, (size_t)P * L) == 0);

    /* Replace rows {1,4} to zero == encode with those rows zeroed (rs_test.go:268-331) */
    {
        int rows[2] = {1, 4};
        const uint8_t* data[2];
        size_t dl[2] = {L, L};
        memcpy(work, ref, (size_t)N * L);
        memcpy(exp, ref, (size_t)N * L);
        memset(exp + (size_t)1 * L, 0, L);
        memset(exp + (size_t)4 * L, 0, L);
        for (i = 0; i < N; ++i) v[i] = exp + (size_t)i * L;
        CHECK(rs_encode(rs, v, lens, N) == RS_OK);
        data[0] = ref + (size_t)1 * L;
        data[1] = ref + (size_t)4 * L;
        for (i = 0; i < N; ++i) v[i] = work + (size_t)i * L;
        CHECK(rs_replace(rs, data, dl, 2, rows, 2, v + D, lens + D, P) == RS_OK);
        CHECK(memcmp(work + (size_t)D * L, exp + (size_t)D * L, (size_t)P * L) == 0);
    }
    CHECK(rs_inverse_cache_size(rs) > 0);
    rs_free(rs);
    free(buf);
    return 0;
}

int main(int argc, char** argv) {
    int rc;
    if (argc != 2 || (strcmp(argv[1], "host") != 0 && strcmp(argv[1], "gpu") != 0)) {
        fprintf(stderr, "usage: %s host|gpu\n", argv[0]);
        return 2;
    }
    rc = strcmp(argv[1], "host") == 0 ? host_checks() : gpu_checks();
    if (rc == 0 && !g_fail) printf("rs_consumer %s: ok\n", argv[1]);
    return rc || g_fail;
}
