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
 *   HL_ENGINE_WAVES=n: its workgroups
 *   HL_VEC=bytes: only this vector size; HL_OPS=mask: only these ops (bit 0
 *   Encode, 1 Reconst lost=1, 2 Reconst lost=4, 3 Update, 4 Replace)
 *
 * Prints one JSON object per (op, size).
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

static void report(const char* op, size_t vec, double bytes, int reps) {
    double med;
    qsort(t, (size_t)reps, sizeof(double), cmp);
    med = t[reps / 2];
    printf("{\"op\": \"%s\", \"vec\": %zu, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, "
           "\"GiBps\": %.3f}\n",
           op, vec, med, t[reps / 10], t[reps * 9 / 10], bytes / (med * 1e-6) / 1073741824.0);
    fflush(stdout);
}

int main(int argc, char** argv) {
    static const size_t sizes[] = {4096, 8192, 65536, 262144, 1048576, 4194304};
    rs_t* rs = NULL;
    size_t si;
    if (argc >= 3) {
        rs_tune("host_zc_max", atoi(argv[1]));
        rs_tune("host_pinned_max", atoi(argv[2]));
    }
    if (argc >= 4) rs_tune("host_chunk", atoi(argv[3]));
    if (getenv("HL_ENGINE")) rs_tune("host_engine", atoi(getenv("HL_ENGINE")));
    if (getenv("HL_ENGINE_MAX")) rs_tune("host_engine_max_bytes", atoi(getenv("HL_ENGINE_MAX")));  /* resident host-call engine on / off */
    if (getenv("HL_ENGINE_WAVES")) rs_tune("host_engine_waves", atoi(getenv("HL_ENGINE_WAVES")));
    if (getenv("HL_ENGINE_WG_UNITS")) rs_tune("host_engine_wg_units", atoi(getenv("HL_ENGINE_WG_UNITS")));
    if (getenv("HL_ENGINE_DIRECT")) rs_tune("host_engine_direct", atoi(getenv("HL_ENGINE_DIRECT")));
    if (getenv("HL_ENGINE_POLL_GAP")) rs_tune("host_engine_poll_gap", atoi(getenv("HL_ENGINE_POLL_GAP")));
    if (getenv("HL_ENGINE_GROUP_WAVES")) rs_tune("host_engine_group_waves", atoi(getenv("HL_ENGINE_GROUP_WAVES")));
    if (rs_device_count() < 1 || rs_new(D, P, -1, &rs) != RS_OK) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    const long only_vec = getenv("HL_VEC") ? atol(getenv("HL_VEC")) : 0;
    const int ops = getenv("HL_OPS") ? atoi(getenv("HL_OPS")) : 31;
    for (si = 0; si < sizeof sizes / sizeof sizes[0]; ++si) {
        const size_t vec = sizes[si];
        if (only_vec && (size_t)only_vec != vec) continue;
        const int reps = vec >= 4194304 ? REPS / 8 : (vec >= 262144 ? REPS / 4 : REPS);
        uint8_t* v[N];
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
        }
        for (k = 0; k < 10; ++k) rs_encode(rs, v, lens, N);
        if (ops & 1) {
            for (k = 0; k < reps; ++k) {
                double a = now_us();
                if (rs_encode(rs, v, lens, N) != RS_OK) return 2;
                t[k] = now_us() - a;
            }
            report("Encode", vec, (double)N * vec, reps);
        }
        if (ops & 2) {
            int need[1] = {0};
            for (k = 0; k < reps; ++k) {
                double a = now_us();
                if (rs_reconst(rs, v, lens, N, NULL, 0, need, 1) != RS_OK) return 3;
                t[k] = now_us() - a;
            }
            report("Reconst lost=1", vec, (double)(D + 1) * vec, reps);
        }
        if (ops & 4) {
            int need[4] = {0, 3, 5, 9};
            for (k = 0; k < reps; ++k) {
                double a = now_us();
                if (rs_reconst(rs, v, lens, N, NULL, 0, need, 4) != RS_OK) return 4;
                t[k] = now_us() - a;
            }
            report("Reconst lost=4", vec, (double)(D + 4) * vec, reps);
        }
        if (ops & 8)
        for (k = 0; k < reps; ++k) {
            double a = now_us();
            if (rs_update(rs, v[2], vec, v[3], vec, 2, v + D, lens + D, P) != RS_OK) return 5;
            t[k] = now_us() - a;
        }
        if (ops & 8) report("Update", vec, (double)(2 + 2 * P) * vec, reps);
        if (ops & 16) {
            int rows[1] = {1};
            for (k = 0; k < reps; ++k) {
                double a = now_us();
                if (rs_replace(rs, (const uint8_t* const*)v, lens, 1, rows, 1, v + D, lens + D, P) != RS_OK)
                    return 6;
                t[k] = now_us() - a;
            }
            report("Replace rn=1", vec, (double)(1 + 2 * P) * vec, reps);
        }
        for (i = 0; i < N; ++i) {
            if (reg && atoi(reg)) rs_host_unregister(v[i]);
            free(v[i]);
        }
    }
    {
        uint64_t calls = 0, launches = 0;
        rs_host_engine_stats(rs, &calls, &launches);
        printf("{\"engine_calls\": %llu, \"engine_launches\": %llu}\n", (unsigned long long)calls,
               (unsigned long long)launches);
    }
    fprintf(stderr, "host_latency: rs_free\n");
    rs_free(rs);
    fprintf(stderr, "host_latency: exit\n");
    return 0;
}
