/* Randomised host-side exercise of the C ABI for AddressSanitizer builds
 * (tools/asan_host.sh): argument checks, reconst planning, matrix inverse,
 * inverse cache, groups, knobs — everything that runs without a GPU, with
 * malformed inputs mixed in.  No call may crash, leak or touch memory it
 * does not own; return codes must stay within the documented set.
 *
 *   tools/asan_host.sh            (builds librsamd + this with -fsanitize=address)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rs_amd.h"

static uint64_t st = 0x5EEDull;
static uint32_t rnd(void) {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (uint32_t)st;
}
static int rr(int lo, int hi) { return lo + (int)(rnd() % (uint32_t)(hi - lo + 1)); }

#define CHECK_RC(rc)                                                      \
    do {                                                                  \
        int r_ = (rc);                                                    \
        if (r_ < 0 || r_ > 15) {                                          \
            fprintf(stderr, "%s:%d: rc %d out of range\n", __FILE__, __LINE__, r_); \
            return 1;                                                     \
        }                                                                 \
    } while (0)

int main(int argc, char** argv) {
    int iters = argc > 1 ? atoi(argv[1]) : 20000, it;
    static uint8_t buf[256 * 256], out[256 * 256];
    for (it = 0; it < iters; ++it) {
        const int d = rr(-2, 40), p = rr(-2, 30);
        rs_t* rs = NULL;
        int rc = rs_new(d, p, -1, &rs), i;
        CHECK_RC(rc);
        if (rc) continue;
        {
            int surv[80], need[80], vs[256], nr[256], nvs, nnr, dn;
            const int ns = rr(0, d + p + 2), nn = rr(0, p + 3);
            for (i = 0; i < ns; ++i) surv[i] = rr(-1, d + p);
            for (i = 0; i < nn; ++i) need[i] = rr(-1, d + p);
            rc = rs_plan_reconst(rs, surv, ns, need, nn, vs, &nvs, nr, &nnr, &dn);
            CHECK_RC(rc);
            if (rc == RS_OK && dn > 0 && nvs >= d) {
                int nd[256], k = 0;
                for (i = 0; i < nnr && k < dn; ++i)
                    if (nr[i] < d) nd[k++] = nr[i];
                CHECK_RC(rs_reconst_matrix(rs, vs, nd, k, out));
            }
            (void)rs_inverse_cache_key(surv, ns < 64 ? ns : 64);
            if (d > 0 && d <= 80) {
                /* any survivor list (repeats, parity only, out of order): the
                 * full inverse (d + p <= 64) or the reduced system beyond */
                int sd[80], nd2[80], k2 = rr(0, d < 8 ? d : 8);
                for (i = 0; i < d; ++i) sd[i] = rr(0, 3) ? i : rr(0, d + p - 1);
                for (i = 0; i < k2; ++i) nd2[i] = rr(0, d - 1);
                CHECK_RC(rs_reconst_matrix(rs, sd, nd2, k2, out));
            }
        }
        {
            uint8_t* v[80];
            size_t lens[80];
            const int n = rr(0, d + p + 1);
            for (i = 0; i < n; ++i) {
                v[i] = buf;
                lens[i] = (size_t)rr(0, 3) * 16;
            }
            /* malformed shapes return errors before any device work; a
             * well-formed one reaches the device and fails with RS_ERR_DEVICE
             * here (no GPU), never anything else */
            rc = rs_encode(rs, v, lens, n);
            CHECK_RC(rc);
            {
                int surv[4] = {0, 1, 2, 3}, need[3] = {0, rr(0, d + p), rr(-1, 300)};
                rc = rs_reconst(rs, v, lens, n, surv, rr(0, 4), need, rr(0, 3));
                CHECK_RC(rc);
            }
            rc = rs_update(rs, buf, (size_t)rr(0, 32), buf, (size_t)rr(0, 32), rr(-1, d), v, lens, n < p ? n : p);
            CHECK_RC(rc);
            {
                int rows[8];
                const int nd = rr(0, 8);
                for (i = 0; i < nd; ++i) rows[i] = rr(-1, d);
                rc = rs_replace(rs, (const uint8_t* const*)v, lens, n < nd ? n : nd, rows, nd, v, lens,
                                n < p ? n : p);
                CHECK_RC(rc);
            }
        }
        {
            const int n = rr(0, 12);
            for (i = 0; i < n * n; ++i) buf[i] = (uint8_t)rnd();
            CHECK_RC(rs_matrix_invert(buf, (size_t)(n * n - rr(0, 1) * (n > 0)), n, out));
        }
        (void)rs_inverse_cache_size(rs);
        rs_free(rs);
        if (it % 97 == 0) {
            int devs[3] = {0, rr(-1, 2), 1};
            rs_group_t* g = NULL;
            rc = rs_group_new(rr(1, 12), rr(1, 4), devs, rr(0, 3), &g);
            CHECK_RC(rc);
            if (!rc) {
                (void)rs_group_codec(g, rr(-1, 3));
                (void)rs_group_size(g);
                rs_group_free(g);
            }
        }
    }
    CHECK_RC(rs_tune("no_such_knob", 1));
    (void)rs_strerror(-5);
    (void)rs_strerror(99);
    printf("host_fuzz: %d iterations ok\n", iters);
    return 0;
}
