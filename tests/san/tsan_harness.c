/*
 * tsan_harness.c — the socket layer (host/nstack.c) under ThreadSanitizer with
 * its threads all running at once: the protocol thread delivering bursts of
 * UDP datagrams and TCP segments (nstack_deliver: the batch paths the GPU
 * bursts use), an application thread draining every socket
 * (nstack_drain_all_sum, waiting on the deliveries counter), a second
 * application thread reading sockets one by one (nrecvfrom / nrecv), and a
 * thread sending from the UDP sockets (nsendto) while the protocol thread's
 * TX pass frames what they queued and the ACKs (nstack_tx_burst), and a
 * thread accepting connections that SYN / ACK / data / FIN / ACK frames open
 * and close in the bursts, one reading and closing them (at EOF, or at random
 * while open), and a thread closing and re-creating UDP sockets meanwhile
 * (nclose / nsocket / nbind;
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
/* connection lifecycles: NC client slots, each running SYN, ACK, 3 x data,
 * FIN, 4 x ACK against the listener on LPORT, then again from a new port */
enum { NC = 24, LPORT = 8080, NFR = BURST + NC, TMAX = 1024 };

static uint32_t g_local;
static int g_udp_fd[NUDP];
static atomic_int g_stop, g_churn; /* g_churn: the churn thread runs (the second half) */
static atomic_llong g_read_items;
static pthread_mutex_t g_fd_mx = PTHREAD_MUTEX_INITIALIZER; /* the harness's own fd table */
static int g_lfd; /* the listener */
static int g_acc[TMAX], g_nacc; /* accepted connections (under g_fd_mx) */
static atomic_llong g_accepted, g_closed, g_eofs;

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

/* slot c's frame at step st of generation g: from 10.3.0.(c+1), a port of
 * its own per generation, to local:LPORT */
static uint16_t lframe(uint8_t *f, int c, int g, int st) {
    static const uint8_t flags[11] = {0x02, 0x10, 0x18, 0x18, 0x18, 0x11, 0x10, 0x10, 0x10, 0x10, 0x10};
    memset(f, 0, SLOT);
    f[12] = 0x08, f[13] = 0x00;
    uint8_t *ip = f + 14;
    ip[0] = 0x45, ip[8] = 64, ip[9] = 6;
    const uint32_t sip = htonl(0x0A030000u | (uint32_t)(c + 1));
    memcpy(ip + 12, &sip, 4);
    memcpy(ip + 16, &g_local, 4);
    uint8_t *l4 = ip + 20;
    const uint32_t plen = flags[st] == 0x18 ? 40u : 0u;
    put16be(ip + 2, 40 + plen);
    put16be(l4, 41000 + c * 16 + g % 16);
    put16be(l4 + 2, LPORT);
    const uint32_t seq = 1000u + (uint32_t)st * 40u;
    l4[4] = (uint8_t)(seq >> 24), l4[5] = (uint8_t)(seq >> 16), l4[6] = (uint8_t)(seq >> 8), l4[7] = (uint8_t)seq;
    l4[12] = 5 << 4, l4[13] = flags[st];
    for (uint32_t b = 0; b < plen; b++) l4[20 + b] = (uint8_t)(c + st + b);
    return (uint16_t)(54 + plen);
}

/* accepts connections on the listener until it is closed (EBADF) */
static void *acceptor(void *arg) {
    (void)arg;
    for (;;) {
        struct sockaddr_in a;
        socklen_t al = sizeof(a);
        const int fd = naccept(g_lfd, (struct sockaddr *)&a, &al);
        if (fd < 0) break;
        atomic_fetch_add(&g_accepted, 1);
        pthread_mutex_lock(&g_fd_mx);
        if (g_nacc < TMAX)
            g_acc[g_nacc++] = fd;
        else
            CHECK(nclose(fd) == 0);
        pthread_mutex_unlock(&g_fd_mx);
    }
    return NULL;
}

/* reads the accepted connections (nrecv) and closes each at its EOF, or at
 * random while it is still open (an application closing an ESTABLISHED
 * connection while segments for it are being delivered) */
static void *closer(void *arg) {
    (void)arg;
    unsigned char buf[2048];
    unsigned seed = 11;
    while (!atomic_load(&g_stop)) {
        pthread_mutex_lock(&g_fd_mx);
        for (int i = 0; i < g_nacc; i++) {
            const ssize_t r = nrecv(g_acc[i], buf, sizeof buf, MSG_DONTWAIT);
            if (r == 0) atomic_fetch_add(&g_eofs, 1);
            if (r == 0 || (r < 0 && errno == EBADF) || rand_r(&seed) % 64 == 0) {
                CHECK(nclose(g_acc[i]) == 0 || errno == EBADF);
                atomic_fetch_add(&g_closed, 1);
                g_acc[i--] = g_acc[--g_nacc];
            }
        }
        pthread_mutex_unlock(&g_fd_mx);
        sched_yield();
    }
    return NULL;
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
    CHECK(nstack_init(RXG_HOST_ONLY, NFR, (uint64_t)NFR * SLOT) == RXG_OK);
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
    uint8_t *pool = aligned_alloc(4096, (size_t)NSET * NFR * SLOT);
    g_lfd = nsocket(AF_INET, SOCK_STREAM, 0);
    CHECK(g_lfd >= 0);
    {
        struct sockaddr_in a;
        sa_of(&a, g_local, LPORT);
        CHECK(nbind(g_lfd, (struct sockaddr *)&a, sizeof(a)) == 0);
        CHECK(nlisten(g_lfd, 16) == 0);
    }
    static rxg_mbuf mb[NSET][NFR];
    static rxg_mbuf *mp[NSET][NFR];
    static uint32_t off[NFR];
    static uint16_t len[NFR];
    static rxg_verdict v[NFR];
    static uint32_t tseq[NTCP];
    static const uint8_t peer_mac[6] = {2, 0, 0, 0, 0, 9}, my_mac[6] = {2, 0, 0, 0, 0, 1};
    CHECK(nstack_set_local(g_local, my_mac) == 0);
    CHECK(nstack_arp_insert(inet_addr("10.2.0.9"), peer_mac) == 1);
    uint8_t *txb = aligned_alloc(4096, 1 << 20);
    static uint32_t txo[512];
    static uint16_t txl[512];
    long long txf = 0;
    pthread_t th[6];
    CHECK(pthread_create(&th[0], NULL, drainer, NULL) == 0);
    CHECK(pthread_create(&th[1], NULL, reader, NULL) == 0);
    CHECK(pthread_create(&th[2], NULL, churn, NULL) == 0);
    CHECK(pthread_create(&th[3], NULL, sender, NULL) == 0);
    CHECK(pthread_create(&th[4], NULL, acceptor, NULL) == 0);
    CHECK(pthread_create(&th[5], NULL, closer, NULL) == 0);
    srand(5);
    long long delivered = 0;
    for (int b = 0; b < NBURST; b++) {
        const int j = b % NSET;
        if (b == NBURST / 2) atomic_store(&g_churn, 1);
        for (int i = 0; i < NFR; i++)
            while (__atomic_load_n(&mb[j][i].refcnt, __ATOMIC_ACQUIRE)) nstack_reclaim();
        uint8_t *base = pool + (size_t)j * NFR * SLOT;
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
        for (int c = 0; c < NC; c++) { /* the lifecycles, one frame per slot per burst */
            const int i = BURST + c, st = (b + c) % 11, g = (b + c) / 11;
            len[i] = lframe(base + (size_t)i * SLOT, c, g, st);
            off[i] = (uint32_t)i * (SLOT / 64);
            mb[j][i].buf_addr = base + (size_t)i * SLOT;
            mb[j][i].data_off = 0;
            mb[j][i].data_len = len[i];
            mp[j][i] = &mb[j][i];
        }
        oracle_tx_cksum(base, off, len, NFR, 6);
        /* the verdicts against the lists as they stand (stable ids) */
        static rxg_udp_sock u[NUDP + 8];
        static rxg_tcb t[TMAX];
        static uint32_t uid[NUDP + 8], tid[TMAX];
        uint32_t nu = 0, nt = 0;
        uint64_t gen = 0;
        CHECK(nstack_flows(u, NUDP + 8, &nu, t, TMAX, &nt, &gen) == RXG_OK);
        CHECK(nt <= TMAX);
        CHECK(nstack_flow_ids(uid, nu, tid, nt) == RXG_OK);
        oracle_tables *tb = oracle_tables_new(u, nu, t, nt);
        oracle_classify(tb, base, off, len, NFR, 6, v, NULL);
        oracle_tables_free(tb);
        for (int i = 0; i < NFR; i++)
            if (v[i].flow_id != RXG_FLOW_NONE)
                v[i].flow_id = v[i].cls == RXG_CLS_UDP ? uid[v[i].flow_id] : tid[v[i].flow_id];
        /* (a socket the churn thread closed since the snapshot: gen differs,
         * and the burst is looked up again frame by frame) */
        const int r = nstack_deliver(mp[j], NFR, v, gen, NULL);
        CHECK(r >= 0);
        delivered += r;
        uint64_t span = 0; /* the TX pass: ACKs and datagrams framed (no GPU checksum) */
        const int tx = nstack_tx_burst(txb, 1 << 20, txo, txl, 512, 0, &span);
        CHECK(tx >= 0);
        txf += tx;
    }
    atomic_store(&g_stop, 1);
    CHECK(nclose(g_lfd) == 0); /* (wakes the acceptor: EBADF) */
    for (int i = 0; i < 6; i++) pthread_join(th[i], NULL);
    nstack_reclaim();
    printf("bursts %d, UDP datagrams delivered %lld, items read %lld, frames released %lld, "
           "datagrams sent %lld, TX frames %lld, connections accepted %lld, closed %lld (%lld at EOF)\n",
           NBURST, delivered, (long long)atomic_load(&g_read_items), (long long)atomic_load(&released),
           (long long)atomic_load(&g_sent), txf, (long long)atomic_load(&g_accepted),
           (long long)atomic_load(&g_closed), (long long)atomic_load(&g_eofs));
    CHECK(txf > 0 && atomic_load(&g_accepted) > 0 && atomic_load(&g_closed) > 0);
    nstack_fini();
    free(pool);
    free(txb);
    printf("TSAN OK\n");
    return 0;
}
