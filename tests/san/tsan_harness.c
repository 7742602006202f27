/*
 * tsan_harness.c — the socket layer (host/nstack.c) under ThreadSanitizer with
 * its threads all running at once: the protocol thread delivering bursts of
 * UDP datagrams and TCP segments (nstack_deliver: the batch paths the GPU
 * bursts use), an application thread draining every socket
 * (nstack_drain_all_sum, waiting on the deliveries counter), a second
 * application thread reading sockets one by one (nrecvfrom / nrecv), and a
 * thread sending from the UDP sockets (nsendto) while the protocol thread's
 * TX pass frames what they queued and the ACKs (nstack_tx_burst), and a
 * thread closing and re-creating sockets meanwhile (nclose / nsocket / nbind;
 * in the second half of the bursts, so the first half takes the batch paths
 * and the second mostly the frame-by-frame path of a changed list).
 * In-place receive on: TCP fragments point into the frames and hold their
 * mbufs.  Built and run by tests/test_sanitizers.py; test infrastructure
 * only (the verdicts come from the oracle).  Prints "TSAN OK" and the counts;
 * any ThreadSanitizer report fails the run (exit code 66).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>

#include "../../include/nstack.h"
#include "../../oracle/ref_cpu.h"

#define CHECK(c)                                                                                   \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);                   \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

enum { NUDP = 48, NTCP = 48, BURST = 384, NBURST = 40, SLOT = 256, NSET = 6 };

static uint32_t g_local;
static int g_udp_fd[NUDP];
static atomic_int g_stop, g_churn; /* g_churn: the churn thread runs (the second half) */
static atomic_llong g_read_items;
static pthread_mutex_t g_fd_mx = PTHREAD_MUTEX_INITIALIZER; /* the harness's own fd table */

static void put16be(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8), p[1] = (uint8_t)v; }

static void sa_of(struct sockaddr_in *a, uint32_t ip, uint16_t port) {
    memset(a, 0, sizeof(*a));
    a->sin_family = AF_INET;
    a->sin_port = htons(port);
    a->sin_addr.s_addr = ip;
}

/* one frame into a SLOT-byte slot: UDP to local:20000+k, or TCP PSH|ACK from
 * 10.1.0.(k+1):30000+k to local:9999 with seq s (checksums filled after) */
static uint16_t frame(uint8_t *f, int udp, int k, uint32_t seq, uint32_t plen) {
    memset(f, 0, SLOT);
    f[12] = 0x08, f[13] = 0x00;
    uint8_t *ip = f + 14;
    ip[0] = 0x45, ip[8] = 64, ip[9] = udp ? 17 : 6;
    const uint32_t sip = htonl(0x0A010000u | (uint32_t)(k + 1));
    memcpy(ip + 12, &sip, 4);
    memcpy(ip + 16, &g_local, 4);
    uint8_t *l4 = ip + 20;
    const uint32_t l4h = udp ? 8 : 20;
    put16be(ip + 2, 20 + l4h + plen);
    put16be(l4, udp ? 5000 : 30000 + k);
    put16be(l4 + 2, udp ? 20000 + k : 9999);
    if (udp) {
        put16be(l4 + 4, 8 + plen);
    } else {
        l4[4] = (uint8_t)(seq >> 24), l4[5] = (uint8_t)(seq >> 16), l4[6] = (uint8_t)(seq >> 8),
        l4[7] = (uint8_t)seq;
        l4[12] = 5 << 4, l4[13] = 0x18;
    }
    for (uint32_t b = 0; b < plen; b++) l4[l4h + b] = (uint8_t)(seq * 31u + b);
    return (uint16_t)(14 + 20 + l4h + plen);
}

/* the second application thread: nrecvfrom / nrecv on sockets in turn */
static void *reader(void *arg) {
    (void)arg;
    unsigned char buf[2048];
    unsigned k = 0;
    while (!atomic_load(&g_stop)) {
        pthread_mutex_lock(&g_fd_mx);
        const int fd = g_udp_fd[k++ % NUDP];
        pthread_mutex_unlock(&g_fd_mx);
        struct sockaddr_in a;
        socklen_t al = sizeof(a);
        const ssize_t r = nrecvfrom(fd, buf, sizeof buf, MSG_DONTWAIT, (struct sockaddr *)&a, &al);
        if (r >= 0) atomic_fetch_add(&g_read_items, 1);
    }
    return NULL;
}

/* the application thread: drain_all, then wait for the next delivery */
static void *drainer(void *arg) {
    (void)arg;
    static unsigned char buf[65536];
    while (!atomic_load(&g_stop)) {
        const uint64_t seen = nstack_stat(12);
        uint64_t nb, hs;
        const int64_t g = nstack_drain_all_sum(buf, sizeof buf, &nb, &hs);
        CHECK(g >= 0);
        atomic_fetch_add(&g_read_items, g);
        if (!g)
            while (nstack_stat(12) == seen && !atomic_load(&g_stop)) sched_yield();
    }
    uint64_t nb, hs;
    const int64_t g = nstack_drain_all_sum(buf, sizeof buf, &nb, &hs);
    CHECK(g >= 0);
    atomic_fetch_add(&g_read_items, g);
    return NULL;
}

/* a thread sending datagrams from the UDP sockets (nsendto), which the
 * protocol thread's TX pass (nstack_tx_burst) frames meanwhile */
static atomic_llong g_sent;
static void *sender(void *arg) {
    (void)arg;
    unsigned k = 0;
    const char msg[] = "tsan harness datagram";
    while (!atomic_load(&g_stop)) {
        pthread_mutex_lock(&g_fd_mx);
        const int fd = g_udp_fd[k++ % NUDP];
        pthread_mutex_unlock(&g_fd_mx);
        struct sockaddr_in a;
        sa_of(&a, inet_addr("10.2.0.9"), 7777);
        if (nsendto(fd, msg, sizeof msg, 0, (struct sockaddr *)&a, sizeof(a)) >= 0)
            atomic_fetch_add(&g_sent, 1);
        sched_yield();
    }
    return NULL;
}

/* a thread closing UDP sockets and binding new ones to the same ports */
static void *churn(void *arg) {
    (void)arg;
    unsigned k = 0;
    while (!atomic_load(&g_stop)) {
        if (!atomic_load(&g_churn)) { /* (the first half: every burst keeps its snapshot) */
            sched_yield();
            continue;
        }
        const int i = (int)(k++ % NUDP);
        pthread_mutex_lock(&g_fd_mx);
        CHECK(nclose(g_udp_fd[i]) == 0);
        const int fd = nsocket(AF_INET, SOCK_DGRAM, 0);
        CHECK(fd >= 0);
        struct sockaddr_in a;
        sa_of(&a, g_local, (uint16_t)(20000 + i));
        CHECK(nbind(fd, (struct sockaddr *)&a, sizeof(a)) == 0);
        g_udp_fd[i] = fd;
        pthread_mutex_unlock(&g_fd_mx);
        struct timespec ts = {0, 1000000};
        nanosleep(&ts, NULL);
    }
    return NULL;
}

static void mb_release(rxg_mbuf *m, void *arg) {
    (void)m;
    atomic_fetch_add((atomic_llong *)arg, 1);
}

int main(void) {
    g_local = inet_addr("192.168.100.77");
    CHECK(nstack_init(RXG_HOST_ONLY, BURST, (uint64_t)BURST * SLOT) == RXG_OK);
    static atomic_llong released;
    CHECK(nstack_set_rx_inplace(1, mb_release, &released) == RXG_OK);
    for (int i = 0; i < NUDP; i++) {
        g_udp_fd[i] = nsocket(AF_INET, SOCK_DGRAM, 0);
        CHECK(g_udp_fd[i] >= 0);
        struct sockaddr_in a;
        sa_of(&a, g_local, (uint16_t)(20000 + i));
        CHECK(nbind(g_udp_fd[i], (struct sockaddr *)&a, sizeof(a)) == 0);
    }
    for (int k = 0; k < NTCP; k++)
        CHECK(nstack_tcb_add(htonl(0x0A010000u | (uint32_t)(k + 1)), g_local, htons((uint16_t)(30000 + k)),
                             htons(9999), 4) == 0);
    /* NSET frame sets in rotation; a set is rewritten only once every frame
     * reference the stack took on it is back (the NIC refilling its ring) */
    uint8_t *pool = aligned_alloc(4096, (size_t)NSET * BURST * SLOT);
    static rxg_mbuf mb[NSET][BURST];
    static rxg_mbuf *mp[NSET][BURST];
    static uint32_t off[BURST];
    static uint16_t len[BURST];
    static rxg_verdict v[BURST];
    static uint32_t tseq[NTCP];
    static const uint8_t peer_mac[6] = {2, 0, 0, 0, 0, 9}, my_mac[6] = {2, 0, 0, 0, 0, 1};
    CHECK(nstack_set_local(g_local, my_mac) == 0);
    CHECK(nstack_arp_insert(inet_addr("10.2.0.9"), peer_mac) == 1);
    uint8_t *txb = aligned_alloc(4096, 1 << 20);
    static uint32_t txo[512];
    static uint16_t txl[512];
    long long txf = 0;
    pthread_t th[4];
    CHECK(pthread_create(&th[0], NULL, drainer, NULL) == 0);
    CHECK(pthread_create(&th[1], NULL, reader, NULL) == 0);
    CHECK(pthread_create(&th[2], NULL, churn, NULL) == 0);
    CHECK(pthread_create(&th[3], NULL, sender, NULL) == 0);
    srand(5);
    long long delivered = 0;
    for (int b = 0; b < NBURST; b++) {
        const int j = b % NSET;
        if (b == NBURST / 2) atomic_store(&g_churn, 1);
        for (int i = 0; i < BURST; i++)
            while (__atomic_load_n(&mb[j][i].refcnt, __ATOMIC_ACQUIRE)) nstack_reclaim();
        uint8_t *base = pool + (size_t)j * BURST * SLOT;
        for (int i = 0; i < BURST; i++) {
            const int udp = rand() & 1;
            const int k = rand() % (udp ? NUDP : NTCP);
            const uint32_t plen = 1 + (uint32_t)(rand() % 150);
            len[i] = frame(base + (size_t)i * SLOT, udp, k, udp ? (uint32_t)i : tseq[k], plen);
            if (!udp) tseq[k] += plen;
            off[i] = (uint32_t)i * (SLOT / 64);
            mb[j][i].buf_addr = base + (size_t)i * SLOT;
            mb[j][i].data_off = 0;
            mb[j][i].data_len = len[i];
            mp[j][i] = &mb[j][i];
        }
        oracle_tx_cksum(base, off, len, BURST, 6);
        /* the verdicts against the lists as they stand (stable ids) */
        static rxg_udp_sock u[NUDP + 8];
        static rxg_tcb t[NTCP + 8];
        static uint32_t uid[NUDP + 8], tid[NTCP + 8];
        uint32_t nu = 0, nt = 0;
        uint64_t gen = 0;
        CHECK(nstack_flows(u, NUDP + 8, &nu, t, NTCP + 8, &nt, &gen) == RXG_OK);
        CHECK(nstack_flow_ids(uid, nu, tid, nt) == RXG_OK);
        oracle_tables *tb = oracle_tables_new(u, nu, t, nt);
        oracle_classify(tb, base, off, len, BURST, 6, v, NULL);
        oracle_tables_free(tb);
        for (int i = 0; i < BURST; i++)
            if (v[i].flow_id != RXG_FLOW_NONE)
                v[i].flow_id = v[i].cls == RXG_CLS_UDP ? uid[v[i].flow_id] : tid[v[i].flow_id];
        /* (a socket the churn thread closed since the snapshot: gen differs,
         * and the burst is looked up again frame by frame) */
        const int r = nstack_deliver(mp[j], BURST, v, gen, NULL);
        CHECK(r >= 0);
        delivered += r;
        uint64_t span = 0; /* the TX pass: ACKs and datagrams framed (no GPU checksum) */
        const int tx = nstack_tx_burst(txb, 1 << 20, txo, txl, 512, 0, &span);
        CHECK(tx >= 0);
        txf += tx;
    }
    atomic_store(&g_stop, 1);
    for (int i = 0; i < 4; i++) pthread_join(th[i], NULL);
    nstack_reclaim();
    printf("bursts %d, UDP datagrams delivered %lld, items read %lld, frames released %lld, "
           "datagrams sent %lld, TX frames %lld\n", NBURST, delivered,
           (long long)atomic_load(&g_read_items), (long long)atomic_load(&released),
           (long long)atomic_load(&g_sent), txf);
    CHECK(txf > 0);
    nstack_fini();
    free(pool);
    free(txb);
    printf("TSAN OK\n");
    return 0;
}
