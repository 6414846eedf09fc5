/* mprotect_toggler.c — a background thread (no Python GIL) that toggles one
 * page in every 2 MiB of a range read-only and back, `gap_us` apart, until
 * told to stop.  Each toggle is a CPU-side invalidation of that page; used by
 * tools/svm_invalidate_probe.py.  Build (CPU container):
 *   gcc -O2 -shared -fPIC -pthread tools/mprotect_toggler.c -o tools/_build/libtoggler.so */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <sys/mman.h>
#include <unistd.h>

static pthread_t g_th;
static atomic_int g_stop;
static atomic_long g_toggles, g_errors;
static uintptr_t g_base;
static size_t g_bytes;
static unsigned g_gap_us;

static void* loop(void* arg) {
    (void)arg;
    for (unsigned long k = 0; !atomic_load(&g_stop); ++k) {
        for (size_t h = 0; h < (g_bytes >> 21) && !atomic_load(&g_stop); ++h) {
            void* pg = (void*)(g_base + (h << 21) + ((k * 37 + h * 11) % 511 + 1) * 4096);
            if (mprotect(pg, 4096, PROT_READ) || mprotect(pg, 4096, PROT_READ | PROT_WRITE)) {
                atomic_fetch_add(&g_errors, 1);
                return 0;
            }
            atomic_fetch_add(&g_toggles, 1);
            if (g_gap_us) usleep(g_gap_us);
        }
    }
    return 0;
}

int toggler_start(uintptr_t base, size_t bytes, unsigned gap_us) {
    g_base = base;
    g_bytes = bytes;
    g_gap_us = gap_us;
    atomic_store(&g_stop, 0);
    atomic_store(&g_toggles, 0);
    atomic_store(&g_errors, 0);
    return pthread_create(&g_th, 0, loop, 0);
}

long toggler_stop(long* errors) {
    atomic_store(&g_stop, 1);
    pthread_join(g_th, 0);
    if (errors) *errors = atomic_load(&g_errors);
    return atomic_load(&g_toggles);
}
