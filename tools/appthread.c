/*
 * appthread.c — the application lcore of bench.py's two-thread socket runs,
 * in C (as the reference's application loop is: its app lcore reads the
 * socket rings beside the protocol lcore, netfamily.c:424-430).  A Python
 * thread in that role measured the interpreter (its lock hand-offs around
 * every call into the stack), not the stack.
 *
 * app_start(cpu, hash) starts one thread (pinned to cpu when cpu >= 0) that
 * calls nstack_drain_all (nstack_drain_all_sum when hash) until app_stop.
 * After a pass that found nothing it waits for the next delivered burst
 * (nstack_stat(12), read without a lock): it polls that one counter, as a
 * DPDK lcore polls its ring, spinning for ~50 us and then in 20-us sleeps,
 * instead of passing over every socket again (each pass looks at every
 * block's queue counters, lines the protocol thread is writing).  app_stop
 * ends it after one more pass and returns what it read.  Bench
 * infrastructure, built by tools/Makefile against libnstack.so (the loader
 * reuses the copy bench.py already loaded).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <stdatomic.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include "../include/nstack.h"

typedef struct {
    int64_t items;       /* datagrams + fragments read */
    uint64_t bytes;      /* payload bytes read */
    uint64_t sum;        /* hash sum (hash mode) */
    uint64_t passes;     /* drain_all calls */
    uint64_t empty;      /* of which found nothing */
    double drain_ms;     /* time inside drain_all */
    int64_t err;         /* first negative return, else 0 */
    uint64_t sleeps;     /* 20-us sleeps waiting for a delivery */
} app_result;

static pthread_t g_th;
static atomic_int g_stop, g_running;
static int g_cpu, g_hash;
static app_result g_res;
static unsigned char g_buf[65536];

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static int64_t pass(void) {
    uint64_t nb = 0, s = 0;
    const double a = now_ms();
    const int64_t g = g_hash ? nstack_drain_all_sum(g_buf, sizeof g_buf, &nb, &s)
                             : nstack_drain_all(g_buf, sizeof g_buf, &nb);
    g_res.drain_ms += now_ms() - a;
    g_res.passes++;
    if (g < 0) {
        if (!g_res.err) g_res.err = g;
        return 0;
    }
    g_res.items += g, g_res.bytes += nb, g_res.sum += s;
    if (!g) g_res.empty++;
    return g;
}

/* until the deliveries counter moves past `seen` (or app_stop) */
static void wait_delivery(uint64_t seen) {
    for (int i = 0; i < 1500; i++) {
        if (nstack_stat(12) != seen || atomic_load_explicit(&g_stop, memory_order_acquire)) return;
        __builtin_ia32_pause();
    }
    const struct timespec pause = {0, 20000};
    while (nstack_stat(12) == seen && !atomic_load_explicit(&g_stop, memory_order_acquire)) {
        nanosleep(&pause, NULL);
        g_res.sleeps++;
    }
}

static void *loop(void *arg) {
    (void)arg;
    if (g_cpu >= 0) {
        cpu_set_t c;
        CPU_ZERO(&c);
        CPU_SET(g_cpu, &c);
        pthread_setaffinity_np(pthread_self(), sizeof c, &c);
    }
    prctl(PR_SET_TIMERSLACK, 1000UL); /* (20-us sleeps, not the default 50-us slack) */
    while (!atomic_load_explicit(&g_stop, memory_order_acquire)) {
        const uint64_t seen = nstack_stat(12); /* before the pass: a burst that
                                                  lands during it is not waited for */
        if (!pass()) wait_delivery(seen);
    }
    pass(); /* what the last burst queued */
    return NULL;
}

int app_start(int cpu, int hash) {
    if (atomic_load(&g_running)) return -1;
    memset(&g_res, 0, sizeof g_res);
    g_cpu = cpu, g_hash = hash;
    atomic_store(&g_stop, 0);
    if (pthread_create(&g_th, NULL, loop, NULL)) return -2;
    atomic_store(&g_running, 1);
    return 0;
}

int app_stop(app_result *r) {
    if (!atomic_load(&g_running)) return -1;
    atomic_store_explicit(&g_stop, 1, memory_order_release);
    pthread_join(g_th, NULL);
    atomic_store(&g_running, 0);
    if (r) *r = g_res;
    return 0;
}
