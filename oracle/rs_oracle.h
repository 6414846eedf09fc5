/*
 * rs_oracle.h — CPU restatement of templexxx/reedsolomon (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle: tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg are the only users.  The product (reedsolomon_amd/,
 * librsamd.so) never links, loads or calls it.
 *
 * Parity is pinned: the GF tables this file generates are checked against
 * the reference's gftbl.go (byte-for-byte, via fixtures extracted by
 * tools/extract_reference_fixtures.py) and ISA-L's table from
 * gftbl_test.go:56; the matrix / codec functions reproduce every KAT in
 * matrix_test.go and rs_test.go (tests/test_oracle.py).
 *
 * Error codes are numerically identical to include/rs_amd.h (checked by a
 * test) but declared independently so the oracle shares no code with the
 * product.
 */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

enum {
    ORC_OK = 0,
    ORC_ERR_ILLEGAL_VECTS = 1,
    ORC_ERR_MISMATCH_VECTS = 2,
    ORC_ERR_ZERO_VECT_SIZE = 3,
    ORC_ERR_MISMATCH_VECT_SIZE = 4,
    ORC_ERR_NO_NEED_RECONST = 5,
    ORC_ERR_TOO_MANY_LOST = 6,
    ORC_ERR_MISMATCH_PARITY_NUM = 7,
    ORC_ERR_ILLEGAL_VECT_INDEX = 8,
    ORC_ERR_TOO_MANY_REPLACE = 9,
    ORC_ERR_MISMATCH_REPLACE = 10,
    ORC_ERR_NOT_SQUARE = 11,
    ORC_ERR_SINGULAR_MATRIX = 12,
    ORC_ERR_INVAL = 13
};

/* GF(2^8) tables, generated like mathtool/gentbls/gentbls.go. */
void orc_tables(uint8_t exp_tbl[255], uint8_t log_tbl[256], uint8_t mul_tbl[65536],
                uint8_t low_high_tbl[8192], uint8_t inverse_tbl[256]);
uint8_t orc_gf_mul(uint8_t a, uint8_t b);

/* gmu.go:11-23 */
void orc_mul_vect(uint8_t c, const uint8_t* in, uint8_t* out, size_t n);
void orc_mul_vect_xor(uint8_t c, const uint8_t* in, uint8_t* out, size_t n);

/* matrix.go */
void orc_make_encode_matrix(int d, int p, uint8_t* out);
int  orc_invert(const uint8_t* m, size_t m_len, int n, uint8_t* out);

/* rs.go */
int  orc_new_check(int d, int p);
uint64_t orc_inverse_cache_key(const int* survived, int ns);
int  orc_check_reconst(int d, int p, const int* survived, int ns, const int* need, int nn,
                       int* vs, int* nvs, int* nr, int* nnr, int* dn);
int  orc_encode(int d, int p, uint8_t* const* vects, const size_t* lens, int n);
int  orc_encode_gen(int d, int p, const uint8_t* gen, uint8_t* const* vects,
                    const size_t* lens, int n, int update_only);
int  orc_reconst(int d, int p, uint8_t* const* vects, const size_t* lens, int n,
                 const int* survived, int ns, const int* need, int nn);
int  orc_update(int d, int p, const uint8_t* old_data, size_t old_len,
                const uint8_t* new_data, size_t new_len, int row,
                uint8_t* const* parity, const size_t* parity_lens, int np);
int  orc_replace(int d, int p, const uint8_t* const* data, const size_t* data_lens, int nd,
                 const int* rows, int nr, uint8_t* const* parity,
                 const size_t* parity_lens, int np);

/* Naive matrix multiply used by rs_test.go:53-70 to check Encode. */
void orc_naive_mul(const uint8_t* gen, int input, int output, uint8_t* const* vects, size_t n);

/* AVX2 split-nibble restatement of gmu_amd64.s (the reference's timed
 * path); the CPU baseline in bench.py.  Falls back to the table path when
 * the host lacks AVX2.  Returns 1 if AVX2 was used. */
int  orc_has_avx2(void);
int  orc_encode_avx2(int d, int p, uint8_t* const* vects, size_t size);

/* L1D size the restated getSplitSize uses (rs.go:158-173; default 32 KiB). */
void orc_set_l1d(size_t l1d);

#endif
