/*
 * sock_host_bench.c — the host half of the socket path at cfg3's shape, no
 * GPU (diagnostics; test infrastructure: the verdicts come from the oracle).
 * A host-only stack (RXG_HOST_ONLY) with 4096 established connections takes
 * bursts of 16384 1500-B TCP segments through nstack_deliver (the segment
 * records are then built on the host, so the delivery time here includes a
 * qsort the GPU path does not have) and the application reads everything
 * with nstack_drain_all: sequentially, and with the application on a second
 * thread.  Copy and in-place receive.  Prints per-burst milliseconds.
 *   gcc -O2 -pthread tools/sock_host_bench.c -Iinclude -o tools/sock_host_bench \
 *       -Ldpdk-tcp-udp_protocol_stack_amd -lnstack -lrxgpu -Loracle -loracle \
 *       -Wl,-rpath,$PWD/dpdk-tcp-udp_protocol_stack_amd -Wl,-rpath,$PWD/oracle
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "../include/nstack.h"
#include "../oracle/ref_cpu.h"

enum { NCONN = 4096, B = 16384, SLOT = 1536, NSET = 4, K = 20 };

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static void put16be(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8), p[1] = (uint8_t)v; }

static uint8_t *pool;
static uint32_t off[B];
static uint16_t len[B];
static rxg_mbuf mb[NSET][B];
static rxg_mbuf *mp[NSET][B];
static rxg_verdict v[B];
static uint64_t gen;
static atomic_int stop;
static atomic_llong app_items;
static char appbuf[65536];

static void *app(void *arg) {
    (void)arg;
    while (!atomic_load(&stop)) {
        uint64_t nb;
        const uint64_t seen = nstack_stat(12); /* (as tools/appthread.c) */
        const int64_t g = nstack_drain_all(appbuf, sizeof appbuf, &nb);
        if (g > 0) atomic_fetch_add(&app_items, g);
        else
            while (nstack_stat(12) == seen && !atomic_load(&stop)) __builtin_ia32_pause();
    }
    uint64_t nb;
    const int64_t g = nstack_drain_all(appbuf, sizeof appbuf, &nb);
    if (g > 0) atomic_fetch_add(&app_items, g);
    return NULL;
}

static int set_free(int j) {
    for (int i = 0; i < B; i++)
        if (__atomic_load_n(&mb[j][i].refcnt, __ATOMIC_ACQUIRE)) return 0;
    return 1;
}

int main(int argc, char **argv) {
    const int inplace = argc > 1 && atoi(argv[1]);
    const int cpu0 = argc > 2 ? atoi(argv[2]) : -1;
    if (cpu0 >= 0) {
        cpu_set_t c;
        CPU_ZERO(&c);
        CPU_SET(cpu0, &c);
        sched_setaffinity(0, sizeof c, &c);
    }
    if (nstack_init(RXG_HOST_ONLY, B, (uint64_t)B * SLOT) != RXG_OK) return 1;
    const uint32_t L = inet_addr("192.168.100.77");
    uint32_t sip[NCONN];
    uint16_t sport[NCONN];
    for (int k = 0; k < NCONN; k++) {
        sip[k] = htonl(0x0A000000u | (uint32_t)(k + 1));
        sport[k] = htons((uint16_t)(20000 + k));
        if (nstack_tcb_add(sip[k], L, sport[k], htons(9999), 4) != 0) return 2;
    }
    /* the frames: Ether + IPv4 + TCP (PSH|ACK) + 1446 B, 1536-B slots */
    /* the frame pool: 2-MB pages when HUGE=1 (transparent huge pages by
     * madvise, as a DPDK mempool sits on hugepages), else 4-KB pages */
    const size_t pbytes = (size_t)NSET * B * SLOT;
    if (getenv("HUGE") && atoi(getenv("HUGE"))) {
        const size_t al = 2u << 20;
        uint8_t *raw = mmap(NULL, pbytes + al, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (raw == MAP_FAILED) return 3;
        pool = (uint8_t *)(((uintptr_t)raw + al - 1) & ~(uintptr_t)(al - 1));
        madvise(pool, pbytes, MADV_HUGEPAGE);
    } else {
        pool = aligned_alloc(4096, pbytes);
    }
    uint8_t *f0 = pool;
    srand(7);
    for (int i = 0; i < B; i++) {
        uint8_t *f = f0 + (size_t)i * SLOT;
        memset(f, 0, SLOT);
        const int k = rand() % NCONN;
        f[12] = 0x08, f[13] = 0x00;
        uint8_t *ip = f + 14;
        ip[0] = 0x45, ip[8] = 64, ip[9] = 6;
        put16be(ip + 2, 1486);
        memcpy(ip + 12, &sip[k], 4);
        memcpy(ip + 16, &L, 4);
        uint8_t *t = ip + 20;
        memcpy(t, &sport[k], 2);
        put16be(t + 2, 9999);
        t[12] = 5 << 4, t[13] = 0x18;
        for (int b = 0; b < 1446; b++) t[20 + b] = (uint8_t)(rand());
        off[i] = (uint32_t)i * (SLOT / 64);
        len[i] = 1500;
    }
    oracle_tx_cksum(f0, off, len, B, 6);
    for (int j = 1; j < NSET; j++) memcpy(pool + (size_t)j * B * SLOT, f0, (size_t)B * SLOT);
    for (int j = 0; j < NSET; j++)
        for (int i = 0; i < B; i++) {
            mb[j][i].buf_addr = pool + (size_t)j * B * SLOT + (size_t)i * SLOT;
            mb[j][i].data_len = len[i];
            mp[j][i] = &mb[j][i];
        }
    /* verdicts (stable ids) against the stack's lists */
    static rxg_udp_sock u[1];
    static rxg_tcb tl[NCONN + 8];
    static uint32_t tid[NCONN + 8];
    uint32_t nu = 0, nt = 0;
    nstack_flows(u, 1, &nu, tl, NCONN + 8, &nt, &gen);
    nstack_flow_ids(NULL, 0, tid, NCONN + 8);
    oracle_tables *tb = oracle_tables_new(u, nu, tl, nt);
    oracle_classify(tb, f0, off, len, B, 6, v, NULL);
    oracle_tables_free(tb);
    for (int i = 0; i < B; i++)
        if (v[i].flow_id != RXG_FLOW_NONE) v[i].flow_id = tid[v[i].flow_id];
    nstack_set_rx_inplace(inplace, NULL, NULL);

    /* sequential: deliver, then read everything */
    double td = 0, ta = 0;
    long items = 0;
    for (int k = 0; k < K + 2; k++) {
        const int j = k % NSET;
        while (!set_free(j)) nstack_reclaim();
        const double a = now_ms();
        nstack_deliver(mp[j], B, v, gen, NULL);
        const double b = now_ms();
        uint64_t nb;
        const int64_t g = nstack_drain_all(appbuf, sizeof appbuf, &nb);
        const double c = now_ms();
        if (k >= 2) td += b - a, ta += c - b, items += g;
    }
    printf("inplace=%d sequential: deliver %.3f ms, app %.3f ms per burst, %.2f Mpps (%ld items)\n",
           inplace, td / K, ta / K, (double)B * K / (td + ta) / 1e3, items);

    /* two threads: the application drains while this thread delivers */
    pthread_t th;
    atomic_store(&stop, 0);
    atomic_store(&app_items, 0);
    pthread_create(&th, NULL, app, NULL);
    if (cpu0 >= 0) {
        cpu_set_t c;
        CPU_ZERO(&c);
        CPU_SET(cpu0 + 1, &c);
        pthread_setaffinity_np(th, sizeof c, &c);
    }
    long waits = 0;
    const double t0 = now_ms();
    double tdel = 0;
    for (int k = 0; k < K; k++) {
        const int j = k % NSET;
        while (!set_free(j)) {
            nstack_reclaim();
            waits++;
            sched_yield();
        }
        const double a = now_ms();
        nstack_deliver(mp[j], B, v, gen, NULL);
        tdel += now_ms() - a;
    }
    atomic_store(&stop, 1);
    pthread_join(th, NULL);
    const double t1 = now_ms();
    nstack_reclaim();
    printf("inplace=%d two threads: %.3f ms per burst (deliver %.3f), %.2f Mpps, %lld items, "
           "lock wait %.3f ms, read-out %.3f ms per burst (all calls), set waits %ld\n",
           inplace, (t1 - t0) / K, tdel / K, (double)B * K / (t1 - t0) / 1e3,
           (long long)atomic_load(&app_items), nstack_stat(8) / 1e6 / K, nstack_stat(10) / 1e6 / K,
           waits);
    nstack_fini();
    return 0;
}
