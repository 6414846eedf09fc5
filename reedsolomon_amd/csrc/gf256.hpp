// gf256.hpp — GF(2^8) arithmetic for the host side of librsamd.
//
// Field: GF(2^8) with primitive polynomial x^8+x^4+x^3+x^2+1 (0x11d), the
// reference's field (rs.go:6-8, mathtool/gentbls/gentbls.go:44-49).  The
// tables are built once at first use from the exp/log representation; a
// test checks them byte-for-byte against the reference's gftbl.go fixtures.
//
// The device never sees these tables: the HIP kernels use per-coefficient
// "perm tables" (see perm_table()) that let one v_perm_b32 multiply four
// packed bytes by a constant.
#pragma once
#include <cstdint>
#include <cstring>

namespace rsamd {

struct GfTables {
    uint8_t exp[512];   // exp[i] = alpha^i, doubled so exp[log a + log b] needs no mod
    uint8_t log[256];
    uint8_t mul[256][256];
    uint8_t inv[256];   // inv[0] = 0, like inverseTbl (gftbl.go:12)
    GfTables() {
        unsigned v = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = static_cast<uint8_t>(v);
            log[v] = static_cast<uint8_t>(i);
            v <<= 1;
            if (v & 0x100) v ^= 0x11d;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
        for (int a = 0; a < 256; ++a)
            for (int b = 0; b < 256; ++b)
                mul[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
        inv[0] = 0;
        for (int a = 1; a < 256; ++a) inv[a] = exp[255 - log[a]];
    }
};

inline const GfTables& gf() {
    static const GfTables t;
    return t;
}

inline uint8_t gf_mul(uint8_t a, uint8_t b) { return gf().mul[a][b]; }
inline uint8_t gf_inv(uint8_t a) { return gf().inv[a]; }

// Device "perm table" of coefficient c: five dwords such that for a byte x
//   c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]
// with T0/T1 eight-entry byte tables (two dwords each: entries 0-3 in the low
// dword, 4-7 in the high one) and T2 a four-entry table (one dword).  This is
// the GF(2)-linear split of multiplication by c over the bit groups
// {0,1,2}, {3,4,5}, {6,7} of x; the kernel evaluates each group for four
// packed bytes with one v_perm_b32.  (Analogue of the reference's
// split-nibble lowHighTbl, gftbl.go:16 / gmu_amd64.go:19-27, reshaped for the
// 8-byte pool of v_perm_b32.)
inline void perm_table(uint8_t c, uint32_t out[5]) {
    uint8_t t0[8], t1[8], t2[4];
    for (int e = 0; e < 8; ++e) {
        t0[e] = gf_mul(c, static_cast<uint8_t>(e));
        t1[e] = gf_mul(c, static_cast<uint8_t>(e << 3));
    }
    for (int e = 0; e < 4; ++e) t2[e] = gf_mul(c, static_cast<uint8_t>(e << 6));
    std::memcpy(&out[0], t0, 4);
    std::memcpy(&out[1], t0 + 4, 4);
    std::memcpy(&out[2], t1, 4);
    std::memcpy(&out[3], t1 + 4, 4);
    std::memcpy(&out[4], t2, 4);
}

}  // namespace rsamd
