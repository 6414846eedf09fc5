/*
 * rs_oracle.c — CPU restatement of templexxx/reedsolomon (TEST INFRASTRUCTURE).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * this file (through oracle/_build/liborc.so).  It is the checker, never the
 * thing measured or shipped: the product library does not link it.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to /root/reference).  Parity of this restatement with the reference is
 * pinned by tests/test_oracle.py: tables vs gftbl.go and ISA-L's table
 * (gftbl_test.go:56), and the KATs of matrix_test.go / rs_test.go.
 */
#include "rs_oracle.h"

#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ---------------------------------------------------------------------- */
/* GF(2^8) tables — mathtool/gentbls/gentbls.go                            */
/* ---------------------------------------------------------------------- */

static uint8_t g_exp[255], g_log[256], g_mul[256 * 256], g_lowhigh[256 * 32], g_inv[256];
static int g_ready = 0;

/* genExpTable gentbls.go:145-156 with primitive polynomial x^8+x^4+x^3+x^2+1
 * (gentbls.go:44-49).  Each step multiplies the running polynomial by x and
 * reduces by the primitive polynomial (expGrowPolynomial :158-178). */
static void gen_exp(uint8_t* t) {
    const unsigned poly_low = 0x1d; /* coefficients of x^4+x^3+x^2+1 */
    unsigned v = 1;
    t[0] = 1;
    for (int i = 1; i < 255; i++) {
        v <<= 1;
        if (v & 0x100) v = (v & 0xff) ^ poly_low;
        t[i] = (uint8_t)v;
    }
}

static void build_tables(void) {
    if (g_ready) return;
    gen_exp(g_exp);
    /* genLogTable gentbls.go:191-198 */
    memset(g_log, 0, sizeof g_log);
    for (int i = 0; i < 255; i++) g_log[g_exp[i]] = (uint8_t)i;
    /* genMulTable gentbls.go:200-218 */
    for (int a = 0; a < 256; a++)
        for (int b = 0; b < 256; b++) {
            if (a == 0 || b == 0) { g_mul[a * 256 + b] = 0; continue; }
            int s = g_log[a] + g_log[b];
            while (s >= 255) s -= 255;
            g_mul[a * 256 + b] = g_exp[s];
        }
    /* genMulTableHalf gentbls.go:220-247 + packing gentbls.go:70-74:
     * lowHighTbl[c*32 + j] = c*j (j<16), lowHighTbl[c*32+16+j] = c*(j<<4). */
    for (int c = 0; c < 256; c++)
        for (int j = 0; j < 16; j++) {
            g_lowhigh[c * 32 + j] = g_mul[c * 256 + j];
            g_lowhigh[c * 32 + 16 + j] = g_mul[c * 256 + (j << 4)];
        }
    /* genInverseTable gentbls.go:249-260 (inv(0) stays 0) */
    memset(g_inv, 0, sizeof g_inv);
    for (int i = 0; i < 256; i++)
        for (int j = 0; j < 256; j++)
            if (g_mul[i * 256 + j] == 1) g_inv[i] = (uint8_t)j;
    g_ready = 1;
}

void orc_tables(uint8_t exp_tbl[255], uint8_t log_tbl[256], uint8_t mul_tbl[65536],
                uint8_t low_high_tbl[8192], uint8_t inverse_tbl[256]) {
    build_tables();
    if (exp_tbl) memcpy(exp_tbl, g_exp, 255);
    if (log_tbl) memcpy(log_tbl, g_log, 256);
    if (mul_tbl) memcpy(mul_tbl, g_mul, 65536);
    if (low_high_tbl) memcpy(low_high_tbl, g_lowhigh, 8192);
    if (inverse_tbl) memcpy(inverse_tbl, g_inv, 256);
}

/* gfMul gmu.go:26-28 */
uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
    build_tables();
    return g_mul[a * 256 + b];
}

/* ---------------------------------------------------------------------- */
/* gmu no-SIMD kernels — gmu.go:11-23                                       */
/* ---------------------------------------------------------------------- */

void orc_mul_vect(uint8_t c, const uint8_t* in, uint8_t* out, size_t n) {
    build_tables();
    const uint8_t* t = &g_mul[c * 256];
    for (size_t i = 0; i < n; i++) out[i] = t[in[i]];
}

void orc_mul_vect_xor(uint8_t c, const uint8_t* in, uint8_t* out, size_t n) {
    build_tables();
    const uint8_t* t = &g_mul[c * 256];
    for (size_t i = 0; i < n; i++) out[i] ^= t[in[i]];
}

/* ---------------------------------------------------------------------- */
/* matrix.go                                                                */
/* ---------------------------------------------------------------------- */

/* makeEncodeMatrix matrix.go:37-54: identity on top, Cauchy inverseTbl[i^j]
 * for i in [d, d+p), j in [0, d) below. */
void orc_make_encode_matrix(int d, int p, uint8_t* m) {
    build_tables();
    int r = d + p;
    memset(m, 0, (size_t)r * d);
    for (int i = 0; i < d; i++) m[i * d + i] = 1;
    int off = d * d;
    for (int i = d; i < r; i++)
        for (int j = 0; j < d; j++) m[off++] = g_inv[i ^ j];
}

static void swap_rows(uint8_t* m, int i, int j, int n) { /* swap matrix.go:150-154 */
    for (int k = 0; k < n; k++) {
        uint8_t t = m[i * n + k];
        m[i * n + k] = m[j * n + k];
        m[j * n + k] = t;
    }
}

/* invert matrix.go:85-147: Gauss-Jordan with a swap against the first
 * lower row holding a non-zero pivot, pivot scaling by inverseTbl, and
 * elimination of every other row. */
int orc_invert(const uint8_t* src, size_t m_len, int n, uint8_t* out) {
    build_tables();
    if ((size_t)n * n != m_len) return ORC_ERR_NOT_SQUARE;
    uint8_t* left = (uint8_t*)malloc((size_t)n * n);
    uint8_t* inv = (uint8_t*)calloc((size_t)n * n, 1);
    memcpy(left, src, (size_t)n * n);
    for (int i = 0; i < n; i++) inv[i * n + i] = 1;
    int rc = ORC_OK;
    for (int i = 0; i < n; i++) {
        if (left[i * n + i] == 0) {
            int j;
            for (j = i + 1; j < n; j++)
                if (left[j * n + i] != 0) break;
            if (j == n) { rc = ORC_ERR_SINGULAR_MATRIX; goto done; }
            swap_rows(left, i, j, n);
            swap_rows(inv, i, j, n);
        }
        if (left[i * n + i] != 1) {
            uint8_t v = g_inv[left[i * n + i]];
            for (int j = 0; j < n; j++) {
                left[i * n + j] = g_mul[left[i * n + j] * 256 + v];
                inv[i * n + j] = g_mul[inv[i * n + j] * 256 + v];
            }
        }
        for (int j = 0; j < n; j++) {
            if (j == i) continue;
            uint8_t v = left[j * n + i];
            if (v != 0) {
                for (int k = 0; k < n; k++) {
                    left[j * n + k] ^= g_mul[v * 256 + left[i * n + k]];
                    inv[j * n + k] ^= g_mul[v * 256 + inv[i * n + k]];
                }
            }
        }
    }
    memcpy(out, inv, (size_t)n * n);
done:
    free(left);
    free(inv);
    return rc;
}

/* ---------------------------------------------------------------------- */
/* rs.go                                                                    */
/* ---------------------------------------------------------------------- */

/* newWithFeature rs.go:59-63 */
int orc_new_check(int d, int p) {
    if (d <= 0 || p <= 0 || d + p > 256) return ORC_ERR_ILLEGAL_VECTS;
    return ORC_OK;
}

/* makeInverseCacheKey rs.go:414-420 (Go: 1<<uint8(i) is 0 for i>=64). */
uint64_t orc_inverse_cache_key(const int* survived, int ns) {
    uint64_t key = 0;
    for (int k = 0; k < ns; k++) {
        unsigned s = (uint8_t)survived[k];
        key += (s < 64) ? ((uint64_t)1 << s) : 0;
    }
    return key;
}

/* getSplitSize rs.go:158-173 with the default L1D of 32 KiB (cpu.X86.Cache.L1D
 * unknown, rs.go:160-162; orc_set_l1d sets another). For Encode the chunking changes no output byte;
 * for Update / Replace (updateOnly) it does, see encode_part. */
static size_t g_l1d = 32 * 1024;
/* cpu.X86.Cache.L1D as the reference would read it on another host (tests of
 * librsamd's rs_set_ref_l1d compat mode); 0 restores 32 KiB. */
void orc_set_l1d(size_t l1d) { g_l1d = l1d ? l1d : 32 * 1024; }

static size_t split_size(size_t n) {
    const size_t l1d = g_l1d;
    if (n < 16) return 16;
    if (n < l1d / 2) return (n >> 4) << 4;
    return l1d / 2;
}

/* encodePart rs.go:175-203 on the no-SIMD feature (gmu_generic.go:6-9): the
 * first data row overwrites unless updateOnly, every other term XORs.
 *
 * Restated as written, including a reference defect: the sub-16-byte tail
 * pass (rs.go:190-200) runs over the WHOLE chunk [start, end), not just
 * [start + done, end).  For Encode that is harmless (its i == 0 term
 * overwrites the chunk again).  For updateOnly (Update rs.go:447, Replace
 * rs.go:527) the chunk's 16-byte-multiple body is XORed twice, so it keeps
 * its old parity: whenever the last chunk has >= 16 bytes and a length that
 * is not a multiple of 16 (vectors >= L1D/2 whose size mod L1D/2 is such a
 * length), the reference's Update / Replace differ from re-encoding there.
 * The region depends on the host's L1D size (cpu.X86.Cache.L1D).  The
 * reference's own tests define Update / Replace as equal to re-encoding
 * (rs_test.go:225-331, at 1 KiB, outside this case); librsamd computes that
 * definition for every size (DESIGN.md §4 "Reference defect"). */
static void encode_part(size_t start, size_t end, int d, int p, const uint8_t* g,
                        uint8_t* const* dv, uint8_t* const* pv, int update_only) {
    size_t undone = end - start;
    size_t done = (undone >> 4) << 4;
    if (done >= 16) {
        size_t end2 = start + done;
        for (int i = 0; i < d; i++)
            for (int j = 0; j < p; j++) {
                if (i != 0 || update_only)
                    orc_mul_vect_xor(g[j * d + i], dv[i] + start, pv[j] + start, end2 - start);
                else
                    orc_mul_vect(g[j * d + i], dv[0] + start, pv[j] + start, end2 - start);
            }
    }
    if (undone > done) {
        for (int i = 0; i < d; i++)
            for (int j = 0; j < p; j++) {
                if (i != 0 || update_only)
                    orc_mul_vect_xor(g[j * d + i], dv[i] + start, pv[j] + start, end - start);
                else
                    orc_mul_vect(g[j * d], dv[0] + start, pv[j] + start, end - start);
            }
    }
}

/* encode rs.go:141-154 (chunk loop) */
static void encode_raw(int d, int p, const uint8_t* g, uint8_t* const* vects, size_t size,
                       int update_only) {
    size_t split = split_size(size);
    for (size_t start = 0; start < size;) {
        size_t end = start + split;
        if (end > size) end = size;
        encode_part(start, end, d, p, g, vects, vects + d, update_only);
        start = end;
    }
}

/* checkEncode rs.go:119-134 */
static int check_encode(int d, int p, const size_t* lens, int n) {
    if (d + p != n) return ORC_ERR_MISMATCH_VECTS;
    size_t size = lens[0];
    if (size == 0) return ORC_ERR_ZERO_VECT_SIZE;
    for (int i = 1; i < n; i++)
        if (lens[i] != size) return ORC_ERR_MISMATCH_VECT_SIZE;
    return ORC_OK;
}

/* Encode rs.go:104-111 with an explicit generator (the temporary-RS trick of
 * reconst rs.go:375-380, Update rs.go:446 and Replace rs.go:525 all reduce to
 * this). */
int orc_encode_gen(int d, int p, const uint8_t* gen, uint8_t* const* vects,
                   const size_t* lens, int n, int update_only) {
    int rc = check_encode(d, p, lens, n);
    if (rc) return rc;
    encode_raw(d, p, gen, vects, lens[0], update_only);
    return ORC_OK;
}

int orc_encode(int d, int p, uint8_t* const* vects, const size_t* lens, int n) {
    if (orc_new_check(d, p)) return ORC_ERR_ILLEGAL_VECTS;
    uint8_t* e = (uint8_t*)malloc((size_t)(d + p) * d);
    orc_make_encode_matrix(d, p, e);
    int rc = orc_encode_gen(d, p, e + d * d, vects, lens, n, 0);
    free(e);
    return rc;
}

/* naive mul rs_test.go:58-70 */
void orc_naive_mul(const uint8_t* m, int input, int output, uint8_t* const* vects, size_t n) {
    build_tables();
    for (int i = 0; i < output; i++)
        for (size_t j = 0; j < n; j++) {
            uint8_t s = 0;
            for (int k = 0; k < input; k++) s ^= g_mul[vects[k][j] * 256 + m[i * input + k]];
            vects[input + i][j] = s;
        }
}

/* checkVectIdx rs.go:250-258 */
static int check_vect_idx(const int* idx, int cnt, int d, int p) {
    for (int k = 0; k < cnt; k++)
        if (idx[k] < 0 || idx[k] >= d + p) return ORC_ERR_ILLEGAL_VECTS;
    return ORC_OK;
}

/* checkReconst rs.go:264-325 */
int orc_check_reconst(int d, int p, const int* survived, int ns, const int* need, int nn,
                      int* vs, int* nvs, int* nr, int* nnr, int* dn) {
    *nvs = *nnr = *dn = 0;
    if (nn == 0) return ORC_ERR_NO_NEED_RECONST;
    int rc = check_vect_idx(survived, ns, d, p);
    if (rc) return rc;
    rc = check_vect_idx(need, nn, d, p);
    if (rc) return rc;
    enum { UNKNOWN = 0, SURVIVED = 1, NEED = 2 };
    uint8_t status[256];
    memset(status, UNKNOWN, sizeof status);
    if (ns == 0)
        for (int i = 0; i < d + p; i++) status[i] = SURVIVED;
    for (int k = 0; k < ns; k++) status[survived[k]] = SURVIVED;
    int full_data = 0;
    for (int k = 0; k < nn; k++) {
        status[need[k]] = NEED;
        if (need[k] >= d) full_data = 1;
    }
    if (full_data)
        for (int i = 0; i < d; i++)
            if (status[i] == UNKNOWN) status[i] = NEED;
    for (int i = 0; i < d + p; i++) {
        if (status[i] == SURVIVED) vs[(*nvs)++] = i;
        else if (status[i] == NEED) {
            if (i < d) (*dn)++;
            nr[(*nnr)++] = i;
        }
    }
    if (*nvs < d || *nnr > p) return ORC_ERR_TOO_MANY_LOST;
    return ORC_OK;
}

/* reconst rs.go:375-380: Encode with a temporary RS (DataNum d, ParityNum
 * nn, GenMatrix gm) over the d+nn vectors vs. */
static int reconst_gm(int d, int nn, const uint8_t* gm, uint8_t* const* vs, const size_t* lens) {
    return orc_encode_gen(d, nn, gm, vs, lens, d + nn, 0);
}

/* Reconst rs.go:221-237, reconstData :327-349, reconstParity :351-373,
 * getReconstMatrix :382-392 (no cache: the cache changes no output byte),
 * makeEncMatrixForReconst matrix.go:68-79, makeReconstMatrix matrix.go:56-64. */
int orc_reconst(int d, int p, uint8_t* const* vects, const size_t* lens, int n,
                const int* survived, int ns, const int* need, int nn) {
    int vs[256], nr[256], nvs, nnr, dn;
    int rc = orc_check_reconst(d, p, survived, ns, need, nn, vs, &nvs, nr, &nnr, &dn);
    if (rc == ORC_ERR_NO_NEED_RECONST) return ORC_OK;
    if (rc) return rc;
    uint8_t* e = (uint8_t*)malloc((size_t)(d + p) * d);
    orc_make_encode_matrix(d, p, e);
    uint8_t* bufv[512];
    size_t bufl[512];
    /* reconstData */
    if (dn > 0) {
        for (int i = 0; i < d; i++) if (vs[i] >= n) { free(e); return ORC_ERR_INVAL; }
        for (int i = 0; i < dn; i++) if (nr[i] >= n) { free(e); return ORC_ERR_INVAL; }
        uint8_t* sub = (uint8_t*)malloc((size_t)d * d);
        uint8_t* inv = (uint8_t*)malloc((size_t)d * d);
        for (int i = 0; i < d; i++) memcpy(sub + i * d, e + vs[i] * d, d);
        rc = orc_invert(sub, (size_t)d * d, d, inv);
        if (rc) { free(sub); free(inv); free(e); return rc; }
        uint8_t* gm = (uint8_t*)malloc((size_t)dn * d);
        for (int i = 0; i < dn; i++) memcpy(gm + i * d, inv + nr[i] * d, d);
        for (int i = 0; i < d; i++) { bufv[i] = vects[vs[i]]; bufl[i] = lens[vs[i]]; }
        for (int i = 0; i < dn; i++) { bufv[d + i] = vects[nr[i]]; bufl[d + i] = lens[nr[i]]; }
        rc = reconst_gm(d, dn, gm, bufv, bufl);
        free(gm); free(sub); free(inv);
        if (rc) { free(e); return rc; }
    }
    /* reconstParity */
    int pn = nnr - dn;
    if (pn > 0) {
        for (int i = 0; i < d; i++) if (i >= n) { free(e); return ORC_ERR_INVAL; }
        for (int i = dn; i < nnr; i++) if (nr[i] >= n) { free(e); return ORC_ERR_INVAL; }
        uint8_t* gm = (uint8_t*)malloc((size_t)pn * d);
        for (int i = 0; i < pn; i++) memcpy(gm + i * d, e + nr[dn + i] * d, d);
        for (int i = 0; i < d; i++) { bufv[i] = vects[i]; bufl[i] = lens[i]; }
        for (int i = 0; i < pn; i++) { bufv[d + i] = vects[nr[dn + i]]; bufl[d + i] = lens[nr[dn + i]]; }
        rc = reconst_gm(d, pn, gm, bufv, bufl);
        free(gm);
    }
    free(e);
    return rc;
}

/* Update rs.go:424-449 with checkUpdate rs.go:456-477.  Step 1 is
 * xorsimd's xor.Encode(buf, [old, new]) = byte XOR (templexxx/xorsimd
 * v0.1.1, go.mod:5; pinned at API level by rs_test.go:225-266). */
int orc_update(int d, int p, const uint8_t* old_data, size_t old_len,
               const uint8_t* new_data, size_t new_len, int row,
               uint8_t* const* parity, const size_t* parity_lens, int np) {
    if (np != p) return ORC_ERR_MISMATCH_PARITY_NUM;
    size_t size = new_len;
    if (size == 0) return ORC_ERR_ZERO_VECT_SIZE;
    if (size != old_len) return ORC_ERR_MISMATCH_VECT_SIZE;
    for (int i = 0; i < np; i++)
        if (parity_lens[i] != size) return ORC_ERR_MISMATCH_VECT_SIZE;
    if (row >= d || row < 0) return ORC_ERR_ILLEGAL_VECT_INDEX;
    uint8_t* buf = (uint8_t*)malloc(size);
    for (size_t i = 0; i < size; i++) buf[i] = old_data[i] ^ new_data[i];
    uint8_t* e = (uint8_t*)malloc((size_t)(d + p) * d);
    orc_make_encode_matrix(d, p, e);
    const uint8_t* g = e + d * d;
    uint8_t gm[256];
    uint8_t* vv[257];
    vv[0] = buf;
    for (int i = 0; i < p; i++) {
        gm[i] = g[i * d + row];
        vv[i + 1] = parity[i];
    }
    encode_raw(1, p, gm, vv, size, 1);
    free(e);
    free(buf);
    return ORC_OK;
}

/* Replace rs.go:492-529 with checkReplace rs.go:536-570. */
int orc_replace(int d, int p, const uint8_t* const* data, const size_t* data_lens, int nd,
                const int* rows, int nr, uint8_t* const* parity,
                const size_t* parity_lens, int np) {
    if (nd > d) return ORC_ERR_TOO_MANY_REPLACE;
    if (nr != nd) return ORC_ERR_MISMATCH_REPLACE;
    if (np != p) return ORC_ERR_MISMATCH_PARITY_NUM;
    if (nd == 0) return ORC_ERR_INVAL; /* data[0] index panic, rs.go:549 */
    size_t size = data_lens[0];
    if (size == 0) return ORC_ERR_ZERO_VECT_SIZE;
    for (int i = 0; i < nd; i++)
        if (data_lens[i] != size) return ORC_ERR_MISMATCH_VECT_SIZE;
    for (int i = 0; i < np; i++)
        if (parity_lens[i] != size) return ORC_ERR_MISMATCH_VECT_SIZE;
    for (int i = 0; i < nr; i++)
        if (rows[i] >= d || rows[i] < 0) return ORC_ERR_ILLEGAL_VECT_INDEX;
    uint8_t* e = (uint8_t*)malloc((size_t)(d + p) * d);
    orc_make_encode_matrix(d, p, e);
    const uint8_t* g = e + d * d;
    uint8_t* gm = (uint8_t*)malloc((size_t)p * nr);
    int off = 0;
    for (int i = 0; i < p; i++)
        for (int j = 0; j < nr; j++) gm[off++] = g[i * d + rows[j]];
    uint8_t* vv[512];
    for (int i = 0; i < nr; i++) vv[i] = (uint8_t*)data[i];
    for (int i = 0; i < p; i++) vv[nr + i] = parity[i];
    encode_raw(nr, p, gm, vv, size, 1);
    free(gm);
    free(e);
    return ORC_OK;
}

/* ---------------------------------------------------------------------- */
/* AVX2 split-nibble restatement of gmu_amd64.s:40-329 — CPU baseline only. */
/* ---------------------------------------------------------------------- */

#if defined(__x86_64__)
int orc_has_avx2(void) { return __builtin_cpu_supports("avx2"); }

/* One (coefficient, chunk) pass: out (=|^=) lowTbl[x&15] ^ highTbl[x>>4]
 * 32 bytes at a time (VPSRLQ/VPAND/VPSHUFB/VPXOR, gmu_amd64.s:66-77),
 * requires n % 32 == 0 here; the 16-byte and table tails are handled by the
 * caller like encodePart. */
__attribute__((target("avx2"))) static void mul_vect_avx2(const uint8_t* tbl, const uint8_t* in,
                                                          uint8_t* out, size_t n, int xor_out) {
    __m128i lo128 = _mm_loadu_si128((const __m128i*)tbl);
    __m128i hi128 = _mm_loadu_si128((const __m128i*)(tbl + 16));
    __m256i lo = _mm256_broadcastsi128_si256(lo128);
    __m256i hi = _mm256_broadcastsi128_si256(hi128);
    __m256i mask = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    /* 256 B per iteration, as the reference's unrolled loop (gmu_amd64.s:64-144) */
    for (; i + 256 <= n; i += 256) {
        __m256i r[8];
        for (int u = 0; u < 8; u++) {
            __m256i x = _mm256_loadu_si256((const __m256i*)(in + i + 32 * u));
            __m256i xl = _mm256_and_si256(x, mask);
            __m256i xh = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
            r[u] = _mm256_xor_si256(_mm256_shuffle_epi8(lo, xl), _mm256_shuffle_epi8(hi, xh));
        }
        if (xor_out)
            for (int u = 0; u < 8; u++)
                r[u] = _mm256_xor_si256(r[u], _mm256_loadu_si256((const __m256i*)(out + i + 32 * u)));
        for (int u = 0; u < 8; u++) _mm256_storeu_si256((__m256i*)(out + i + 32 * u), r[u]);
    }
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i*)(in + i));
        __m256i xl = _mm256_and_si256(x, mask);
        __m256i xh = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(lo, xl), _mm256_shuffle_epi8(hi, xh));
        if (xor_out) r = _mm256_xor_si256(r, _mm256_loadu_si256((const __m256i*)(out + i)));
        _mm256_storeu_si256((__m256i*)(out + i), r);
    }
    for (; i + 16 <= n; i += 16) { /* one16b gmu_amd64.s:169-181 */
        __m128i x = _mm_loadu_si128((const __m128i*)(in + i));
        __m128i m4 = _mm_set1_epi8(0x0f);
        __m128i xl = _mm_and_si128(x, m4);
        __m128i xh = _mm_and_si128(_mm_srli_epi64(x, 4), m4);
        __m128i r = _mm_xor_si128(_mm_shuffle_epi8(lo128, xl), _mm_shuffle_epi8(hi128, xh));
        if (xor_out) r = _mm_xor_si128(r, _mm_loadu_si128((const __m128i*)(out + i)));
        _mm_storeu_si128((__m128i*)(out + i), r);
    }
}

/* encode rs.go:141-154 + encodePart rs.go:175-203 on the AVX2 feature. */
int orc_encode_avx2(int d, int p, uint8_t* const* vects, size_t size) {
    build_tables();
    if (!orc_has_avx2()) {
        size_t lens[512];
        for (int i = 0; i < d + p; i++) lens[i] = size;
        orc_encode(d, p, vects, lens, d + p);
        return 0;
    }
    uint8_t* e = (uint8_t*)malloc((size_t)(d + p) * d);
    orc_make_encode_matrix(d, p, e);
    const uint8_t* g = e + d * d;
    size_t split = split_size(size);
    for (size_t start = 0; start < size;) {
        size_t end = start + split;
        if (end > size) end = size;
        size_t undone = end - start, done = (undone >> 4) << 4;
        if (done >= 16)
            for (int i = 0; i < d; i++)
                for (int j = 0; j < p; j++) {
                    uint8_t c = g[j * d + i];
                    mul_vect_avx2(&g_lowhigh[c * 32], vects[i] + start, vects[d + j] + start, done,
                                  i != 0);
                }
        if (undone > done)
            for (int i = 0; i < d; i++)
                for (int j = 0; j < p; j++) {
                    if (i != 0) orc_mul_vect_xor(g[j * d + i], vects[i] + start + done,
                                                 vects[d + j] + start + done, undone - done);
                    else orc_mul_vect(g[j * d], vects[0] + start + done,
                                      vects[d + j] + start + done, undone - done);
                }
        start = end;
    }
    free(e);
    return 1;
}
#else
int orc_has_avx2(void) { return 0; }
int orc_encode_avx2(int d, int p, uint8_t* const* vects, size_t size) {
    size_t lens[512];
    for (int i = 0; i < d + p; i++) lens[i] = size;
    orc_encode(d, p, vects, lens, d + p);
    return 0;
}
#endif
