/* Concurrent synchronous host calls (what a Go storage server does: many
 * goroutines, one rs_encode / rs_reconst per stripe).  T threads share one
 * handle; each encodes (even threads) or rebuilds two lost vectors (odd
 * threads, mixed mode) of its own 10+4 stripe in a loop.  Every result is
 * checked against the same call made alone before the timed phase.
 *
 *   gcc -O2 -std=c99 -pthread -Iinclude tools/host_concurrency.c -Lreedsolomon_amd/_lib -lrsamd \
 *       -Wl,-rpath,$PWD/reedsolomon_amd/_lib -o tools/_build/host_concurrency
 *   tools/_build/host_concurrency <vec bytes> <calls per thread> <coalesce_max> <mixed 0/1> T1 T2 ...
 *
 * Prints one JSON object per thread count (after an untimed 8-thread warm-up
 * round that loads every path's kernels).
 *   HL_REGISTER=1: each thread's vectors are page-aligned and registered with
 *   rs_host_register (calls run over the caller's memory, no coalescing)
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <signal.h>
#include <execinfo.h>

#include "rs_amd.h"

enum { D = 10, P = 4, N = D + P, MAXT = 256, MAXCALLS = 4096 };

static rs_t* g_rs;
static size_t g_vec;
static int g_calls, g_mixed;

typedef struct {
    int id;
    uint8_t* v[N];      /* working stripe */
    uint8_t* want[N];   /* expected stripe after the call */
    size_t lens[N];
    double lat[MAXCALLS];
    int bad;
} Worker;

static Worker g_w[MAXT];
static pthread_barrier_t g_bar;

static double now_us(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

static int cmpd(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

static const int kLost[2] = {0, 11};

static int one_call(Worker* w) {
    if (g_mixed && (w->id & 1)) {
        memset(w->v[kLost[0]], 0, g_vec);
        memset(w->v[kLost[1]], 0, g_vec);
        return rs_reconst(g_rs, w->v, w->lens, N, NULL, 0, kLost, 2);
    }
    return rs_encode(g_rs, w->v, w->lens, N);
}

static void* run(void* arg) {
    Worker* w = (Worker*)arg;
    int i, j;
    pthread_barrier_wait(&g_bar);
    for (i = 0; i < g_calls; ++i) {
        double t0 = now_us();
        int rc = one_call(w);
        w->lat[i] = now_us() - t0;
        if (rc) w->bad++;
    }
    for (j = 0; j < N; ++j)
        if (memcmp(w->v[j], w->want[j], g_vec)) w->bad++;
    return NULL;
}

static void at_exit_last(void) { fprintf(stderr, "host_concurrency: atexit handlers done\n"); }

/* diagnostics: SIGUSR1 prints the main thread's stack (stall analysis) */
static pthread_t g_main_thread;
static void on_usr1(int sig) {
    void* frames[64];
    int n;
    (void)sig;
    n = backtrace(frames, 64);
    fprintf(stderr, "host_concurrency: %s thread stack:\n", pthread_equal(pthread_self(), g_main_thread) ? "main" : "other");
    backtrace_symbols_fd(frames, n, 2);
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
    int a, t, j, nt;
    atexit(at_exit_last);
    {
        void* warm[2];
        g_main_thread = pthread_self();
        backtrace(warm, 2); /* loads the unwinder before any signal */
        signal(SIGUSR1, on_usr1);
    }
    uint32_t seed = 12345;
    if (argc < 6) {
        fprintf(stderr, "usage: %s vec calls coalesce_max mixed T...\n", argv[0]);
        return 2;
    }
    g_vec = (size_t)atol(argv[1]);
    g_calls = atoi(argv[2]);
    if (g_calls > MAXCALLS) g_calls = MAXCALLS;
    rs_tune("host_coalesce_max", atoi(argv[3]));
    g_mixed = atoi(argv[4]);
    if (getenv("HL_ENGINE")) rs_tune("host_engine", atoi(getenv("HL_ENGINE")));
    if (getenv("HL_ENGINE_MAX")) rs_tune("host_engine_max_bytes", atoi(getenv("HL_ENGINE_MAX")));
    if (getenv("HL_ENGINE_WAVES")) rs_tune("host_engine_waves", atoi(getenv("HL_ENGINE_WAVES")));
    if (getenv("HL_CO_RUNNING")) rs_tune("host_coalesce_running", atoi(getenv("HL_CO_RUNNING")));
    if (getenv("HL_ENGINE_IDLE")) rs_tune("host_engine_idle_us", atoi(getenv("HL_ENGINE_IDLE")));
    if (getenv("HL_ENGINE_YIELD")) rs_tune("host_engine_yield_us", atoi(getenv("HL_ENGINE_YIELD")));
    if (getenv("HL_ENGINE_POLL_GAP")) rs_tune("host_engine_poll_gap", atoi(getenv("HL_ENGINE_POLL_GAP")));
    if (getenv("HL_ENGINE_WG_UNITS")) rs_tune("host_engine_wg_units", atoi(getenv("HL_ENGINE_WG_UNITS")));
    if (getenv("HL_ENGINE_DIRECT")) rs_tune("host_engine_direct", atoi(getenv("HL_ENGINE_DIRECT")));
    if (getenv("HL_ENGINE_GROUP_WAVES")) rs_tune("host_engine_group_waves", atoi(getenv("HL_ENGINE_GROUP_WAVES")));
    apply_tune_env();
    if (rs_device_count() < 1 || rs_new(D, P, -1, &g_rs) != RS_OK) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    for (t = 0; t < MAXT; ++t) {
        Worker* w = &g_w[t];
        w->id = t;
        for (j = 0; j < N; ++j) {
            size_t b;
            if (getenv("HL_REGISTER") && atoi(getenv("HL_REGISTER"))) {
                void* mem = NULL;
                if (posix_memalign(&mem, 4096, g_vec) || rs_host_register(mem, g_vec) != RS_OK) return 8;
                w->v[j] = (uint8_t*)mem;
            } else {
                w->v[j] = (uint8_t*)malloc(g_vec);
            }
            w->want[j] = (uint8_t*)malloc(g_vec);
            w->lens[j] = g_vec;
            for (b = 0; b < g_vec; ++b) {
                seed = seed * 1664525u + 1013904223u;
                w->v[j][b] = (uint8_t)(seed >> 24);
            }
        }
        /* expected result: the same call made alone (also leaves v in its final state) */
        if (rs_encode(g_rs, w->v, w->lens, N) != RS_OK) return 1;
        if (getenv("HL_PROGRESS") && (t & 31) == 31) fprintf(stderr, "host_concurrency: %d workers ready\n", t + 1);
        for (j = 0; j < N; ++j) memcpy(w->want[j], w->v[j], g_vec);
    }
    if (getenv("HL_PROGRESS")) fprintf(stderr, "host_concurrency: warm-up\n");
    {   /* untimed warm-up round at 8 threads: first launches of every path
         * (the engine, multi-stripe coalesced batches) load their kernels,
         * which costs milliseconds once per process and is not steady state */
        pthread_t th[8];
        pthread_barrier_init(&g_bar, NULL, 9u);
        for (t = 0; t < 8; ++t) pthread_create(&th[t], NULL, run, &g_w[t]);
        pthread_barrier_wait(&g_bar);
        for (t = 0; t < 8; ++t) pthread_join(th[t], NULL);
        pthread_barrier_destroy(&g_bar);
        for (t = 0; t < 8; ++t)
            if (g_w[t].bad) return 3;
    }
    for (a = 5; a < argc; ++a) {
        pthread_t th[MAXT];
        double t0, t1, all_lat[MAXT * 16], med, p90;
        int bad = 0, k = 0;
        nt = atoi(argv[a]);
        if (nt < 1 || nt > MAXT) continue;
        pthread_barrier_init(&g_bar, NULL, (unsigned)nt + 1);
        for (t = 0; t < nt; ++t) {
            g_w[t].bad = 0;
            pthread_create(&th[t], NULL, run, &g_w[t]);
        }
        pthread_barrier_wait(&g_bar);
        t0 = now_us();
        for (t = 0; t < nt; ++t) pthread_join(th[t], NULL);
        t1 = now_us();
        pthread_barrier_destroy(&g_bar);
        for (t = 0; t < nt; ++t) {
            int i;
            bad += g_w[t].bad;
            for (i = 0; i < g_calls && k < MAXT * 16; i += (g_calls + 15) / 16) all_lat[k++] = g_w[t].lat[i];
        }
        qsort(all_lat, (size_t)k, sizeof(double), cmpd);
        med = all_lat[k / 2];
        p90 = all_lat[k * 9 / 10];
        printf("{\"threads\": %d, \"vec\": %zu, \"calls\": %d, \"mixed\": %d, \"coalesce_max\": %s, "
               "\"calls_per_s\": %.0f, \"GiBps\": %.3f, \"median_us\": %.1f, \"p90_us\": %.1f, \"errors\": %d}\n",
               nt, g_vec, nt * g_calls, g_mixed, argv[3], nt * g_calls / ((t1 - t0) * 1e-6),
               (double)nt * g_calls * N * g_vec / ((t1 - t0) * 1e-6) / 1073741824.0, med, p90, bad);
        {
            uint64_t ec = 0, el = 0;
            rs_host_engine_stats(g_rs, &ec, &el);
            printf("{\"engine_calls_total\": %llu, \"engine_launches_total\": %llu}\n", (unsigned long long)ec,
                   (unsigned long long)el);
        }
        fflush(stdout);
        if (bad) return 3;
    }
    fprintf(stderr, "host_concurrency: rs_free\n");
    rs_free(g_rs);
    fprintf(stderr, "host_concurrency: exit\n");
    if (getenv("HL_FAST_EXIT") && atoi(getenv("HL_FAST_EXIT"))) _exit(0); /* diagnostics: skip atexit handlers and static destructors */
    return 0;
}
