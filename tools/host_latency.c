/* Per-call latency of the synchronous host-memory C ABI (the calls a cgo
 * binding of the Go API makes), timed from C so no binding overhead is
 * included.  10+4, pageable malloc'd vectors, median of N calls.
 *
 *   gcc -O2 -std=c99 -Iinclude tools/host_latency.c -Lreedsolomon_amd/_lib -lrsamd \
 *       -Wl,-rpath,$PWD/reedsolomon_amd/_lib -o tools/_build/host_latency
 *   tools/_build/host_latency [host_zc_max host_pinned_max [host_chunk]]
 *   (host_zc_max -1 = default chunked zero-copy for every size, 0 = staged paths)
 *   HL_REGISTER=1: page-aligned vectors registered with rs_host_register (the
 *   calls then run zero-copy over the caller's memory)
 *   HL_ENGINE=0/1: the resident host-call engine off / on (default on);
 *   HL_ENGINE_IDLE / HL_ENGINE_LIFE=us: its idle exit and lifetime;
 *   HL_ENGINE_WAVES=n: its workgroups
 *   HL_ZC_MAX / HL_PINNED_MAX / HL_CHUNK=bytes: rs_tune host_zc_max /
 *   host_pinned_max / host_chunk (as the positional arguments);
 *   HL_GAP_US=us: idle time between calls (outside the timed region), so the
 *   engine's idle exit is exercised as a sporadic caller would;
 *   HL_SIZES=a,b,...: these vector sizes instead of 4 KiB..4 MiB;
 *   HL_VEC=bytes: only this vector size; HL_OPS=mask: only these ops (bit 0
 *   Encode, 1 Reconst lost=1, 2 Reconst lost=4, 3 Update, 4 Replace)
 *   HL_VRAM=0/1: engine call slots and input staging in host-writable device
 *   memory (default 0); HL_SPLIT_ROWS=0/1: a lone call's rows on separate
 *   waves (default 1)
 *
 * Every call's result is checked outside the timed region: Encode's parity
 * and Update / Replace's new parity against a plain GF(2^8)/0x11d product
 * over the library's generator matrix (rs_gen_matrix), Reconst's rebuilt
 * vectors (overwritten with junk before each call) against their bytes.
 * Prints one JSON object per (op, size); "checked" counts verified calls.
 */
#define _POSIX_C_SOURCE 200112L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rs_amd.h"

enum { D = 10, P = 4, N = D + P, REPS = 400 };

static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

static int cmp(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

static double t[REPS];
static double g_gap_us;

static void gap(void) {  /* idle the caller between calls (HL_GAP_US) */
    if (g_gap_us > 0) {
        const double end = now_us() + g_gap_us;
        while (now_us() < end) {
        }
    }
}
static uint8_t gexp[512], glog[256], gen[P * D];
static long checked;

static void gf_init(void) {
    int x = 1, i;
    for (i = 0; i < 255; ++i) {
        gexp[i] = gexp[i + 255] = (uint8_t)x;
        glog[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11d;
    }
}
static uint8_t gmul(uint8_t a, uint8_t b) { return a && b ? gexp[glog[a] + glog[b]] : 0; }

/* parity row j of data vectors v[0..D) at byte k */
static uint8_t par_byte(uint8_t* const* v, int j, size_t k) {
    uint8_t x = 0;
    int c;
    for (c = 0; c < D; ++c) x ^= gmul(gen[j * D + c], v[c][k]);
    return x;
}
static int check_parity(uint8_t* const* v, size_t vec) {
    size_t k;
    int j;
    for (j = 0; j < P; ++j)
        for (k = 0; k < vec; ++k)
            if (v[D + j][k] != par_byte(v, j, k)) return 0;
    ++checked;
    return 1;
}

static void report(const char* op, size_t vec, double bytes, int reps) {
    double med;
    qsort(t, (size_t)reps, sizeof(double), cmp);
    med = t[reps / 2];
    printf("{\"op\": \"%s\", \"vec\": %zu, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, "
           "\"GiBps\": %.3f}\n",
           op, vec, med, t[reps / 10], t[reps * 9 / 10], bytes / (med * 1e-6) / 1073741824.0);
    fflush(stdout);
}

/* HL_TUNE="name=value,name=value": any rs_tune knobs (applied after the
 * HL_* shorthands). */
static void apply_tune_env(void) {
    const char* e = getenv("HL_TUNE");
    char buf[512], *tok, *save = NULL;
    if (!e) return;
    strncpy(buf, e, sizeof buf - 1);
    buf[sizeof buf - 1] = 0;
    for (tok = strtok_r(buf, ",", &save); tok; tok = strtok_r(NULL, ",", &save)) {
        char* eq = strchr(tok, '=');
        if (!eq) continue;
        *eq = 0;
        if (rs_tune(tok, atoi(eq + 1)) != RS_OK) fprintf(stderr, "HL_TUNE: unknown knob %s\n", tok);
    }
}

int main(int argc, char** argv) {
    size_t sizes[16] = {4096, 8192, 65536, 262144, 1048576, 4194304};
    size_t nsizes = 6;
    rs_t* rs = NULL;
    size_t si;
    if (getenv("HL_SIZES")) {
        char buf[256], *tok;
        strncpy(buf, getenv("HL_SIZES"), sizeof buf - 1);
        buf[sizeof buf - 1] = 0;
        nsizes = 0;
        for (tok = strtok(buf, ","); tok && nsizes < 16; tok = strtok(NULL, ",")) sizes[nsizes++] = (size_t)atol(tok);
    }
    if (argc >= 3) {
        rs_tune("host_zc_max", atoi(argv[1]));
        rs_tune("host_pinned_max", atoi(argv[2]));
    }
    if (argc >= 4) rs_tune("host_chunk", atoi(argv[3]));
    if (getenv("HL_ZC_MAX")) rs_tune("host_zc_max", atoi(getenv("HL_ZC_MAX")));
    if (getenv("HL_PINNED_MAX")) rs_tune("host_pinned_max", atoi(getenv("HL_PINNED_MAX")));
    if (getenv("HL_CHUNK")) rs_tune("host_chunk", atoi(getenv("HL_CHUNK")));
    if (getenv("HL_ENGINE")) rs_tune("host_engine", atoi(getenv("HL_ENGINE")));
    if (getenv("HL_ENGINE_MAX")) rs_tune("host_engine_max_bytes", atoi(getenv("HL_ENGINE_MAX")));  /* resident host-call engine on / off */
    if (getenv("HL_ENGINE_WAVES")) rs_tune("host_engine_waves", atoi(getenv("HL_ENGINE_WAVES")));
    if (getenv("HL_ENGINE_WG_UNITS")) rs_tune("host_engine_wg_units", atoi(getenv("HL_ENGINE_WG_UNITS")));
    if (getenv("HL_ENGINE_DIRECT")) rs_tune("host_engine_direct", atoi(getenv("HL_ENGINE_DIRECT")));
    if (getenv("HL_ENGINE_POLL_GAP")) rs_tune("host_engine_poll_gap", atoi(getenv("HL_ENGINE_POLL_GAP")));
    if (getenv("HL_ENGINE_GROUP_WAVES")) rs_tune("host_engine_group_waves", atoi(getenv("HL_ENGINE_GROUP_WAVES")));
    if (getenv("HL_VRAM")) rs_tune("host_engine_vram", atoi(getenv("HL_VRAM")));
    if (getenv("HL_ENGINE_IDLE")) rs_tune("host_engine_idle_us", atoi(getenv("HL_ENGINE_IDLE")));
    if (getenv("HL_ENGINE_LIFE")) rs_tune("host_engine_life_us", atoi(getenv("HL_ENGINE_LIFE")));
    if (getenv("HL_SPLIT_ROWS")) rs_tune("host_engine_split_rows", atoi(getenv("HL_SPLIT_ROWS")));
    apply_tune_env();
    if (rs_device_count() < 1 || rs_new(D, P, -1, &rs) != RS_OK) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    gf_init();
    if (rs_gen_matrix(rs, gen) != RS_OK) return 11;
    const long only_vec = getenv("HL_VEC") ? atol(getenv("HL_VEC")) : 0;
    g_gap_us = getenv("HL_GAP_US") ? atof(getenv("HL_GAP_US")) : 0;
    const int ops = getenv("HL_OPS") ? atoi(getenv("HL_OPS")) : 31;
    for (si = 0; si < nsizes; ++si) {
        const size_t vec = sizes[si];
        if (only_vec && (size_t)only_vec != vec) continue;
        const int reps = vec >= 4194304 ? REPS / 8 : (vec >= 262144 ? REPS / 4 : REPS);
        uint8_t* v[N];
        uint8_t* saved[N];
        size_t lens[N];
        int i, k;
        const char* reg = getenv("HL_REGISTER");
        for (i = 0; i < N; ++i) {
            void* mem = NULL;
            if (posix_memalign(&mem, 4096, vec)) return 7;
            v[i] = (uint8_t*)mem;
            lens[i] = vec;
            for (k = 0; k < (int)vec; ++k) v[i][k] = (uint8_t)(k * 31 + i * 7);
            if (reg && atoi(reg) && rs_host_register(v[i], vec) != RS_OK) return 8;
            if (!(saved[i] = (uint8_t*)malloc(vec))) return 7;
        }
        for (k = 0; k < 10; ++k) rs_encode(rs, v, lens, N);
        if (!check_parity(v, vec)) return 12;
        if (ops & 1) {
            for (k = 0; k < reps; ++k) {
                double a;
                for (i = D; i < N; ++i) memset(v[i], 0x5a, vec);
                gap();
                a = now_us();
                if (rs_encode(rs, v, lens, N) != RS_OK) return 2;
                t[k] = now_us() - a;
                if (!check_parity(v, vec)) return 13;
            }
            report("Encode", vec, (double)N * vec, reps);
        }
        for (i = 0; i < N; ++i) memcpy(saved[i], v[i], vec);
        if (ops & 2) {
            int need[1] = {0};
            for (k = 0; k < reps; ++k) {
                double a;
                memset(v[0], 0x77, vec);
                gap();
                a = now_us();
                if (rs_reconst(rs, v, lens, N, NULL, 0, need, 1) != RS_OK) return 3;
                t[k] = now_us() - a;
                if (memcmp(v[0], saved[0], vec)) return 14;
                ++checked;
            }
            report("Reconst lost=1", vec, (double)(D + 1) * vec, reps);
        }
        if (ops & 4) {
            int need[4] = {0, 3, 5, 9};
            for (k = 0; k < reps; ++k) {
                double a;
                for (i = 0; i < 4; ++i) memset(v[need[i]], 0x77, vec);
                gap();
                a = now_us();
                if (rs_reconst(rs, v, lens, N, NULL, 0, need, 4) != RS_OK) return 4;
                t[k] = now_us() - a;
                for (i = 0; i < 4; ++i)
                    if (memcmp(v[need[i]], saved[need[i]], vec)) return 15;
                ++checked;
            }
            report("Reconst lost=4", vec, (double)(D + 4) * vec, reps);
        }
        if (ops & 8) {
            /* data row 2 alternates between its bytes and row 3's: the
             * parity after each Update is that of the data as it now is */
            for (k = 0; k < reps; ++k) {
                double a;
                uint8_t* nw = (k & 1) ? saved[2] : saved[3];
                gap();
                a = now_us();
                if (rs_update(rs, v[2], vec, nw, vec, 2, v + D, lens + D, P) != RS_OK) return 5;
                t[k] = now_us() - a;
                memcpy(v[2], nw, vec);
                if (!check_parity(v, vec)) return 16;
            }
            report("Update", vec, (double)(2 + 2 * P) * vec, reps);
            memcpy(v[2], saved[2], vec);
            for (i = D; i < N; ++i) memcpy(v[i], saved[i], vec);
        }
        if (ops & 16) {
            /* parity ^= G[:, 1] x data (rs.go:492-529): from the parity before */
            int rows[1] = {1};
            for (k = 0; k < reps; ++k) {
                double a;
                size_t b;
                int j;
                for (j = 0; j < P; ++j) memcpy(saved[D + j], v[D + j], vec);
                gap();
                a = now_us();
                if (rs_replace(rs, (const uint8_t* const*)v, lens, 1, rows, 1, v + D, lens + D, P) != RS_OK)
                    return 6;
                t[k] = now_us() - a;
                for (j = 0; j < P; ++j)
                    for (b = 0; b < vec; ++b)
                        if (v[D + j][b] != (uint8_t)(saved[D + j][b] ^ gmul(gen[j * D + 1], v[0][b]))) return 17;
                ++checked;
            }
            report("Replace rn=1", vec, (double)(1 + 2 * P) * vec, reps);
        }
        for (i = 0; i < N; ++i) {
            if (reg && atoi(reg)) rs_host_unregister(v[i]);
            free(v[i]);
            free(saved[i]);
        }
    }
    {
        uint64_t calls = 0, launches = 0;
        rs_host_engine_stats(rs, &calls, &launches);
        printf("{\"engine_calls\": %llu, \"engine_launches\": %llu, \"checked\": %ld}\n",
               (unsigned long long)calls, (unsigned long long)launches, checked);
    }
    fprintf(stderr, "host_latency: rs_free\n");
    rs_free(rs);
    fprintf(stderr, "host_latency: exit\n");
    return 0;
}
