/*
 * san_harness.c — host code under AddressSanitizer + UndefinedBehaviorSanitizer
 * (sanitizers on the host C/C++ and the C restatement).
 * Built and run by tests/test_sanitizers.py; test infrastructure only.
 *
 * Compiled together, with -fsanitize=address,undefined:
 *   oracle/ref_cpu.c                      the C restatement (classify, TX fill)
 *   oracle/ref_stack.c                    the delivery restatement (socket layer)
 *   dpdk-tcp-udp_protocol_stack_amd/csrc/rx_pcap.cpp   pcap ingest (g++)
 *   dpdk-tcp-udp_protocol_stack_amd/host/nstack.c      the socket layer
 * and linked against librxgpu.so for the control-plane calls nstack makes
 * (a host-only context: no GPU, no kernel launch).
 *
 * Exercised: runts, truncated captures, tl < 20 and tl > caplen, odd L4
 * lengths, IHL != 5, ARP/ICMP/non-IP frames, 9000-B frames; pcap files that
 * are truncated, oversized, empty or of the wrong link type; the socket calls
 * (UDP bind/recvfrom split reads, TCP listen/handshake/data/FIN, sendto/send
 * and TX framing) fed with oracle verdicts.
 */
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/nstack.h"
#include "../../include/rxgpu.h"
#include "../../oracle/ref_cpu.h"

#define CHECK(c)                                                                                   \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);                   \
            exit(2);                                                                               \
        }                                                                                          \
    } while (0)

static const uint8_t MAC_A[6] = {2, 0, 0, 0, 0, 1}, MAC_B[6] = {2, 0, 0, 0, 0, 2};

/* Ethernet + IPv4 (+ UDP/TCP header) + payload; checksums filled by the oracle */
static size_t frame(uint8_t *f, uint8_t proto, uint32_t sip, uint16_t sport, uint32_t dip,
                    uint16_t dport, uint8_t tcp_flags, uint32_t seq, const void *pl, size_t pn) {
    memcpy(f, MAC_B, 6);
    memcpy(f + 6, MAC_A, 6);
    f[12] = 0x08, f[13] = 0x00;
    uint8_t *ip = f + 14;
    const size_t l4h = proto == 17 ? 8 : (proto == 6 ? 20 : 8);
    const uint16_t tl = (uint16_t)(20 + l4h + pn);
    memset(ip, 0, 20);
    ip[0] = 0x45, ip[8] = 64, ip[9] = proto;
    ip[2] = (uint8_t)(tl >> 8), ip[3] = (uint8_t)tl;
    memcpy(ip + 12, &sip, 4);
    memcpy(ip + 16, &dip, 4);
    uint8_t *l4 = ip + 20;
    memset(l4, 0, l4h);
    memcpy(l4, &sport, 2);
    memcpy(l4 + 2, &dport, 2);
    if (proto == 17) {
        const uint16_t dl = htons((uint16_t)(8 + pn));
        memcpy(l4 + 4, &dl, 2);
    } else if (proto == 6) {
        const uint32_t s = htonl(seq);
        memcpy(l4 + 4, &s, 4);
        l4[12] = 5 << 4, l4[13] = tcp_flags;
        l4[14] = 0xFF, l4[15] = 0xFF;
    }
    if (pn) memcpy(l4 + l4h, pl, pn);
    return 14 + tl;
}

/* pack frames at 64-B units; caps may cut frames short */
typedef struct {
    uint8_t *buf;
    uint32_t off[64];
    uint16_t len[64];
    uint32_t n;
    size_t pos;
} burst;

static void push(burst *b, const uint8_t *f, size_t n, size_t cap) {
    memcpy(b->buf + b->pos, f, cap < n ? cap : n);
    b->off[b->n] = (uint32_t)(b->pos >> 6);
    b->len[b->n] = (uint16_t)(cap < n ? cap : n);
    b->n++;
    b->pos += (n + 63) & ~(size_t)63;
}

static void oracle_edge_cases(void) {
    burst b = {.buf = calloc(1, 1 << 20)};
    uint8_t f[9100], pl[9000];
    for (size_t i = 0; i < sizeof pl; ++i) pl[i] = (uint8_t)(i * 131u + 7u);
    const uint32_t L = inet_addr("192.168.100.77"), C = inet_addr("10.0.0.1");
    size_t n;
    n = frame(f, 17, C, htons(5555), L, htons(8889), 0, 0, "HELLO", 5);
    push(&b, f, n, n);                       /* delivered UDP */
    push(&b, f, n, 20);                      /* runt: caplen inside the IPv4 header */
    push(&b, f, n, 0);                       /* empty capture */
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x18, 1, pl, 1401);
    push(&b, f, n, n);                       /* odd L4 length */
    push(&b, f, n, 100);                     /* tl > caplen - 14 */
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x02, 1, NULL, 0);
    f[16] = 0, f[17] = 19;                   /* tl < 20 */
    push(&b, f, n, n);
    n = frame(f, 17, C, htons(1), L, htons(2), 0, 0, pl, 8972);
    push(&b, f, n, n);                       /* 9000-B jumbo */
    n = frame(f, 17, C, htons(1), L, htons(2), 0, 0, pl, 40);
    f[14] = 0x46;                            /* IHL 6: ignored, as in the reference */
    push(&b, f, n, n);
    n = frame(f, 1, C, 0, L, 0, 0, 0, pl, 20); /* ICMP-like: IPv4, neither UDP nor TCP */
    push(&b, f, n, n);
    n = frame(f, 17, C, htons(1), L, htons(2), 0, 0, pl, 30);
    f[12] = 0x08, f[13] = 0x06;              /* ARP ethertype */
    push(&b, f, n, n);
    f[12] = 0x86, f[13] = 0xDD;              /* IPv6 ethertype: non-IPv4 */
    push(&b, f, n, n);

    oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
    rxg_udp_sock u = {L, htons(8889), 17, 0};
    rxg_tcb t[2] = {{0, L, 0, htons(9999), 1}, {C, L, htons(40000), htons(9999), 4}};
    oracle_tables *tb = oracle_tables_new(&u, 1, t, 2);
    CHECK(tb);
    rxg_verdict v[64];
    uint64_t counts[3] = {0, 0, 0};
    oracle_classify(tb, b.buf, b.off, b.len, b.n, 6, v, counts);
    CHECK(v[0].rc == 0 && v[0].flow_id == 0);
    CHECK(v[3].rc == 0 && v[3].cksum_ok == 1);
    CHECK(v[5].l4_cksum == 0);
    CHECK(v[9].cls == RXG_CLS_ARP && v[10].cls == RXG_CLS_NON_IP);
    oracle_tables_free(tb);
    free(b.buf);
}

static void pcap_cases(void) {
    char path[] = "/tmp/san_pcap_XXXXXX";
    const int fd = mkstemp(path);
    CHECK(fd >= 0);
    close(fd);
    uint8_t f[2048], pl[1500];
    memset(pl, 0x5A, sizeof pl);
    burst b = {.buf = calloc(1, 1 << 16)};
    const uint32_t L = inet_addr("192.168.100.77"), C = inet_addr("10.0.0.1");
    for (int i = 0; i < 5; ++i) {
        const size_t n = frame(f, 17, C, htons(1), L, htons(2), 0, 0, pl, (size_t)(i * 300));
        push(&b, f, n, n);
    }
    CHECK(rxg_pcap_write(path, b.buf, b.off, b.len, b.n, 6) == RXG_OK);
    rxg_pcap *p = NULL;
    CHECK(rxg_pcap_open(&p, path) == RXG_OK);
    uint8_t *dst = malloc(4096);
    uint32_t off[8], n = 0;
    uint16_t len[8];
    uint64_t span = 0;
    /* a 4-KiB buffer: bursts end when the next frame does not fit */
    uint32_t total = 0;
    for (int k = 0; k < 10; ++k) {
        int rc = rxg_pcap_read_burst(p, dst, 4096, off, len, 8, 6, &n, &span);
        CHECK(rc == RXG_OK);
        if (n == 0) break;
        total += n;
    }
    CHECK(total == 5);
    CHECK(rxg_pcap_rewind(p) == RXG_OK);
    CHECK(rxg_pcap_read_burst(p, dst, 32, off, len, 8, 6, &n, &span) == RXG_ERANGE); /* first frame > buffer */
    rxg_pcap_close(p);

    /* malformed files: truncated record, oversized record, short header, wrong link type */
    FILE *w = fopen(path, "r+b");
    CHECK(w);
    fseek(w, 0, SEEK_END);
    const long size = ftell(w);
    CHECK(ftruncate(fileno(w), size - 7) == 0);
    fclose(w);
    CHECK(rxg_pcap_open(&p, path) == RXG_OK);
    int rc = RXG_OK;
    for (int k = 0; k < 10 && rc == RXG_OK; ++k) {
        rc = rxg_pcap_read_burst(p, dst, 4096, off, len, 8, 6, &n, &span);
        if (rc == RXG_OK && n == 0) break;
    }
    CHECK(rc == RXG_EINVAL); /* the cut record */
    rxg_pcap_close(p);
    w = fopen(path, "r+b");
    CHECK(w);
    const uint32_t huge = 70000;
    fseek(w, 24 + 8, SEEK_SET);
    fwrite(&huge, 4, 1, w);
    fclose(w);
    CHECK(rxg_pcap_open(&p, path) == RXG_OK);
    CHECK(rxg_pcap_read_burst(p, dst, 4096, off, len, 8, 6, &n, &span) == RXG_ERANGE);
    rxg_pcap_close(p);
    w = fopen(path, "r+b");
    CHECK(w);
    const uint32_t linktype = 101;
    fseek(w, 20, SEEK_SET);
    fwrite(&linktype, 4, 1, w);
    fclose(w);
    CHECK(rxg_pcap_open(&p, path) == RXG_EINVAL);
    CHECK(truncate(path, 10) == 0);
    CHECK(rxg_pcap_open(&p, path) == RXG_EINVAL);
    unlink(path);
    free(dst);
    free(b.buf);
}

/* classify a burst against the stack's current control blocks (oracle
 * verdicts: the GPU's are bit-identical, tests/test_gpu_parity.py) and
 * deliver, through the caller's mbufs (persistent: in-place delivery points
 * into them) or, mb NULL, through descriptors on the stack */
static void deliver_mb(burst *b, int *rc, rxg_mbuf *mbp);
static void deliver(burst *b, int *rc) { deliver_mb(b, rc, NULL); }
static void deliver_mb(burst *b, int *rc, rxg_mbuf *mbp) {
    rxg_udp_sock u[64];
    rxg_tcb t[64];
    uint32_t nu = 0, nt = 0;
    uint64_t gen = 0;
    CHECK(nstack_flows(u, 64, &nu, t, 64, &nt, &gen) == RXG_OK);
    oracle_tables *tb = oracle_tables_new(u, nu, t, nt);
    CHECK(tb);
    rxg_verdict v[64];
    oracle_classify(tb, b->buf, b->off, b->len, b->n, 6, v, NULL);
    oracle_tables_free(tb);
    uint32_t uid[64], tid[64]; /* oracle index (creation order) -> stable flow id */
    CHECK(nstack_flow_ids(uid, 64, tid, 64) == RXG_OK);
    for (uint32_t i = 0; i < b->n; ++i)
        if (v[i].flow_id != RXG_FLOW_NONE)
            v[i].flow_id = v[i].cls == RXG_CLS_TCP ? tid[v[i].flow_id] : uid[v[i].flow_id];
    rxg_mbuf mbl[64], *mp[64];
    rxg_mbuf *mb = mbp ? mbp : mbl;
    memset(mb, 0, 64 * sizeof(rxg_mbuf));
    for (uint32_t i = 0; i < b->n; ++i) {
        mb[i].buf_addr = b->buf + ((size_t)b->off[i] << 6);
        mb[i].data_len = b->len[i];
        mb[i].refcnt = 1; /* the caller's reference (rte_pktmbuf_alloc) */
        mp[i] = &mb[i];
    }
    CHECK(nstack_deliver(mp, b->n, v, gen, rc) >= 0);
    if (mbp) nstack_mbufs_put(mp, b->n); /* the caller lets go (rte_pktmbuf_free) */
}

/* ---- block lifetime under two threads, and in-place receive ------------- */
static void on_release(rxg_mbuf *m, void *arg) {
    (void)m;
    ++*(int *)arg;
}

typedef struct {
    int fd, kind; /* 0 nrecv, 1 nrecvfrom, 2 naccept */
    ssize_t r;
    int err;
    volatile int entered;
} blocker;

static void *block_call(void *p) {
    blocker *b = p;
    char out[256];
    struct sockaddr_in s;
    socklen_t sl = sizeof s;
    b->entered = 1;
    if (b->kind == 0)
        b->r = nrecv(b->fd, out, sizeof out, 0);
    else if (b->kind == 1)
        b->r = nrecvfrom(b->fd, out, sizeof out, 0, (struct sockaddr *)&s, &sl);
    else
        b->r = naccept(b->fd, (struct sockaddr *)&s, &sl);
    b->err = errno;
    return NULL;
}

static void start_blocked(blocker *b, pthread_t *th) {
    CHECK(pthread_create(th, NULL, block_call, b) == 0);
    while (!b->entered) usleep(1000);
    usleep(100000); /* in the call, waiting */
}

static void lifetime_cases(void) {
    CHECK(nstack_init(RXG_HOST_ONLY, 256, 1 << 20) == RXG_OK);
    const uint32_t L = inet_addr("192.168.100.77"), C = inet_addr("10.0.0.9");
    CHECK(nstack_set_local(L, MAC_A) == RXG_OK);
    const int us = nsocket(AF_INET, SOCK_DGRAM, 0);
    struct sockaddr_in a = {.sin_family = AF_INET, .sin_port = htons(8889), .sin_addr.s_addr = L};
    CHECK(nbind(us, (struct sockaddr *)&a, sizeof a) == 0);
    const int ls = nsocket(AF_INET, SOCK_STREAM, 0);
    a.sin_port = htons(9999);
    CHECK(nbind(ls, (struct sockaddr *)&a, sizeof a) == 0);
    CHECK(nlisten(ls, 16) == 0);
    CHECK(nstack_tcb_add(C, L, htons(40000), htons(9999), 4) == 0); /* ESTABLISHED */
    struct sockaddr_in peer;
    socklen_t pl2 = sizeof peer;
    const int cs = naccept(ls, (struct sockaddr *)&peer, &pl2);
    CHECK(cs >= 0);

    /* in place: the data segments' fragments point into their frames and hold
     * their mbufs until read; the other frames' mbufs go at the caller's put */
    int released = 0;
    CHECK(nstack_set_rx_inplace(1, on_release, &released) == RXG_OK);
    static rxg_mbuf mb[64];
    uint8_t f[2048], pl[1400], out[2048];
    for (size_t i = 0; i < sizeof pl; ++i) pl[i] = (uint8_t)(i * 13 + 1);
    burst b = {.buf = calloc(1, 1 << 20)};
    size_t n;
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x18, 1001, pl, 300); /* PSH data */
    push(&b, f, n, n);
    n = frame(f, 17, C, htons(5555), L, htons(8889), 0, 0, pl, 40); /* a datagram (copied) */
    push(&b, f, n, n);
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x18, 1301, pl + 300, 700);
    push(&b, f, n, n);
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x18, 2001, pl, 500);
    push(&b, f, n, 300); /* captured short: copied, zero filled */
    oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
    int rc[64];
    deliver_mb(&b, rc, mb);
    CHECK(rc[0] == 0 && rc[1] == 0 && rc[2] == 0);
    CHECK(mb[0].refcnt == 1 && mb[2].refcnt == 1); /* held by their fragments */
    CHECK(mb[1].refcnt == 0 && mb[3].refcnt == 0 && released == 2);
    CHECK(nrecv(cs, out, sizeof out, MSG_DONTWAIT) == 300 && memcmp(out, pl, 300) == 0);
    CHECK(nrecv(cs, out, sizeof out, MSG_DONTWAIT) == 700 && memcmp(out, pl + 300, 700) == 0);
    CHECK(nrecv(cs, out, sizeof out, MSG_DONTWAIT) == 500);
    CHECK(mb[0].refcnt == 0 && mb[2].refcnt == 0 && released == 4); /* the batch is freed */
    CHECK(nrecvfrom(us, out, sizeof out, MSG_DONTWAIT, NULL, NULL) == 48);

    /* an application thread blocked in nrecv while another closes the
     * connection and the peer's last ACK frees the tcb (tcp.c:312-331): the
     * call wakes and returns -1 (EBADF); the tcb's memory goes with its put */
    blocker br = {.fd = cs, .kind = 0};
    pthread_t th;
    start_blocked(&br, &th);
    CHECK(nclose(cs) == 0); /* FIN queued, LAST_ACK */
    b.n = 0, b.pos = 0;
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x10, 2501, NULL, 0); /* the last ACK */
    push(&b, f, n, n);
    oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
    deliver(&b, rc);
    CHECK(rc[0] == 0);
    pthread_join(th, NULL);
    CHECK(br.r == -1 && br.err == EBADF);
    CHECK(nstack_tcb_count() == 1); /* the listener */

    /* nrecvfrom blocked on a socket another thread closes */
    blocker bu = {.fd = us, .kind = 1};
    start_blocked(&bu, &th);
    CHECK(nclose(us) == 0);
    pthread_join(th, NULL);
    CHECK(bu.r == -1 && bu.err == EBADF);

    /* naccept blocked on a listener another thread closes */
    blocker ba = {.fd = ls, .kind = 2};
    start_blocked(&ba, &th);
    CHECK(nclose(ls) == 0);
    pthread_join(th, NULL);
    CHECK(ba.r == -1 && ba.err == EBADF);
    CHECK(nstack_set_rx_inplace(0, NULL, NULL) == RXG_OK);
    free(b.buf);
    nstack_fini();
}

static void socket_cases(void) {
    CHECK(nstack_init(RXG_HOST_ONLY, 256, 1 << 20) == RXG_OK);
    const uint32_t L = inet_addr("192.168.100.77"), C = inet_addr("10.0.0.9");
    CHECK(nstack_set_local(L, MAC_A) == RXG_OK);
    CHECK(nstack_arp_insert(C, MAC_B) == 1); /* inserted (ng_arp_entry_insert) */
    const int us = nsocket(AF_INET, SOCK_DGRAM, 0);
    struct sockaddr_in a = {.sin_family = AF_INET, .sin_port = htons(8889), .sin_addr.s_addr = L};
    CHECK(nbind(us, (struct sockaddr *)&a, sizeof a) == 0);
    const int ls = nsocket(AF_INET, SOCK_STREAM, 0);
    a.sin_port = htons(9999);
    CHECK(nbind(ls, (struct sockaddr *)&a, sizeof a) == 0);
    CHECK(nlisten(ls, 16) == 0);

    uint8_t f[2048], pl[1400];
    memset(pl, 'q', sizeof pl);
    burst b = {.buf = calloc(1, 1 << 20)};
    size_t n;
    n = frame(f, 17, C, htons(5555), L, htons(8889), 0, 0, pl, 700);
    push(&b, f, n, n);
    n = frame(f, 17, C, htons(5555), L, htons(8889), 0, 0, NULL, 0); /* dgram_len 8: rc -2 */
    push(&b, f, n, n);
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x02, 1000, NULL, 0); /* SYN */
    push(&b, f, n, n);
    oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
    int rc[64];
    deliver(&b, rc);
    CHECK(rc[0] == 0 && rc[1] == -2 && rc[2] == 0);

    char out[4096];
    struct sockaddr_in src;
    socklen_t sl = sizeof src;
    CHECK(nrecvfrom(us, out, 100, 0, (struct sockaddr *)&src, &sl) == 100); /* split read */
    sl = sizeof src;
    CHECK(nrecvfrom(us, out, sizeof out, 0, (struct sockaddr *)&src, &sl) > 0);
    CHECK(nsendto(us, "reply", 5, 0, (struct sockaddr *)&src, sizeof src) == 5);

    uint8_t tx[1 << 16];
    uint32_t toff[64];
    uint16_t tlen[64];
    uint64_t tspan = 0;
    const int ntx = nstack_tx_burst(tx, sizeof tx, toff, tlen, 64, 0, &tspan);
    CHECK(ntx >= 1); /* the datagram and the SYN-ACK */
    uint32_t ack = 0; /* our ISN + 1, from the SYN-ACK */
    for (int i = 0; i < ntx; ++i) {
        const uint8_t *g = tx + ((size_t)toff[i] << 6);
        if (tlen[i] >= 54 && g[23] == 6 && (g[47] & 0x12) == 0x12) {
            uint32_t s;
            memcpy(&s, g + 38, 4);
            ack = ntohl(s) + 1;
        }
    }
    b.n = 0, b.pos = 0;
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x10, 1001, NULL, 0); /* ACK */
    {
        const uint32_t a32 = htonl(ack);
        memcpy(f + 42, &a32, 4);
    }
    push(&b, f, n, n);
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x18, 1001, pl, 300); /* PSH data */
    push(&b, f, n, n);
    oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
    deliver(&b, rc);
    CHECK(rc[0] == 0 && rc[1] == 0);
    /* the handshake completed: an ESTABLISHED (4) tcb for the client exists,
     * so naccept (which blocks, like the reference's) returns at once */
    rxg_udp_sock fu[64];
    rxg_tcb ft[64];
    uint32_t nu = 0, nt = 0, est = 0;
    CHECK(nstack_flows(fu, 64, &nu, ft, 64, &nt, NULL) == RXG_OK);
    for (uint32_t i = 0; i < nt; ++i) est += ft[i].sip == C && ft[i].status == 4;
    CHECK(est == 1);
    struct sockaddr_in peer;
    socklen_t pl2 = sizeof peer;
    const int cs = naccept(ls, (struct sockaddr *)&peer, &pl2);
    CHECK(cs >= 0);
    CHECK(nrecv(cs, out, 128, MSG_DONTWAIT) > 0); /* split read: the rest stays queued */
    CHECK(nrecv(cs, out, sizeof out, MSG_DONTWAIT) > 0);
    CHECK(nrecv(cs, out, sizeof out, MSG_DONTWAIT) == -1); /* drained */
    CHECK(nsend(cs, "bye", 3, 0) == 3);
    (void)nstack_tx_burst(tx, sizeof tx, toff, tlen, 64, 0, &tspan);
    b.n = 0, b.pos = 0;
    n = frame(f, 6, C, htons(40000), L, htons(9999), 0x11, 1301, NULL, 0); /* FIN */
    push(&b, f, n, n);
    oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
    deliver(&b, rc);
    CHECK(nrecv(cs, out, 128, MSG_DONTWAIT) == 0); /* EOF */
    (void)nstack_tx_burst(tx, sizeof tx, toff, tlen, 64, 0, &tspan);
    nclose(cs);
    CHECK(nclose(us) == 0);
    CHECK(nclose(ls) == 0);
    CHECK(nclose(us) == -1);
    free(b.buf);
    nstack_fini();
}

/* the delivery oracle (ref_stack.c) through a UDP + TCP session, truncated
 * frames included */
static void oracle_stack_cases(void) {
    oracle_stack *st = oracle_stack_new();
    CHECK(st);
    const uint32_t L = inet_addr("192.168.100.77"), C = inet_addr("10.0.0.9");
    const int us = oracle_nsocket(st, 2), ls = oracle_nsocket(st, 1);
    CHECK(oracle_nbind(st, us, L, htons(8889)) == 0 && oracle_nbind(st, ls, L, htons(9999)) == 0);
    CHECK(oracle_nlisten(st, ls) == 0);
    uint8_t f[2048], out[2048], pl[600];
    for (size_t i = 0; i < sizeof pl; ++i) pl[i] = (uint8_t)(i * 7);
    burst b = {malloc(1 << 16), {0}, {0}, 0, 0};
    const struct {
        uint8_t proto, flags;
        uint32_t seq;
        size_t pn, cap;
    } seg[] = {{17, 0, 0, 100, 4000}, {17, 0, 0, 0, 4000}, {17, 0, 0, 50, 40},
               {6, 0x02, 1000, 0, 4000}, {6, 0x10, 1001, 0, 4000}, {6, 0x18, 1001, 300, 4000},
               {6, 0x18, 1301, 200, 90}, {6, 0x11, 1501, 0, 4000}};
    for (size_t k = 0; k < sizeof seg / sizeof seg[0]; ++k) {
        const size_t n = frame(f, seg[k].proto, C, htons(40000), L,
                               htons(seg[k].proto == 17 ? 8889 : 9999), seg[k].flags, seg[k].seq,
                               pl, seg[k].pn);
        b.n = 0, b.pos = 0;
        push(&b, f, n, seg[k].cap);
        oracle_tx_cksum(b.buf, b.off, b.len, b.n, 6);
        (void)oracle_rx(st, b.buf, b.len[0]);
    }
    uint32_t sip = 0;
    uint16_t sport = 0;
    CHECK(oracle_nrecvfrom(st, us, out, 30, &sip, &sport) == 30); /* split */
    while (oracle_nrecvfrom(st, us, out, sizeof out, &sip, &sport) > 0) {
    }
    const int cs = oracle_naccept(st, ls, &sip, &sport);
    CHECK(cs >= 0);
    while (oracle_nrecv(st, cs, out, 77) > 0) {
    }
    int32_t status = 0;
    CHECK(oracle_tcb_state(st, C, L, htons(40000), htons(9999), &status, NULL, NULL, NULL) >= 0);
    CHECK(oracle_nclose(st, cs) == 0 && oracle_nclose(st, us) == 0 && oracle_nclose(st, ls) == 0);
    free(b.buf);
    oracle_stack_free(st);
}

int main(void) {
    oracle_edge_cases();
    pcap_cases();
    socket_cases();
    lifetime_cases();
    oracle_stack_cases();
    printf("SAN OK\n");
    return 0;
}
