/*
 * udp_tcp_app.c — a C application on the drop-in socket API (include/nstack.h),
 * written the way the reference's own servers are (netfamily.c:211-383: a UDP
 * server on nsocket/nbind/nrecvfrom, a TCP server on nsocket/nbind/nlisten/
 * naccept/nrecv), with the protocol loop's receive burst (netfamily.c:147-200)
 * replaced by nstack_rx_burst and its udp_out/tcp_out pass by nstack_tx_burst.
 *
 * The frames a NIC would deliver are built here (Ethernet/IPv4/UDP|TCP with
 * the checksums a sender computes, RFC 1071), in rte_mbuf-shaped descriptors.
 * It checks, in C and without Python, that:
 *   - every datagram of a burst reaches the UDP socket with its payload and
 *     source (offload.length = dgram_len, udp.c:37);
 *   - a SYN, its handshake ACK and PSH data in later bursts establish a
 *     connection that naccept returns and whose nrecv reads the data;
 *   - a frame with a corrupted TCP checksum is dropped (rc -1, RXG_RC_TCP_BAD_CKSUM: tcp.c:349-357);
 *   - the TX pass encodes the SYN|ACK and the data ACK with GPU checksums.
 * Exit 0 and "udp_tcp_app ok" on success.  Needs a GPU (device 0).
 */
#include <arpa/inet.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/nstack.h"

#define LOCAL_IP "192.168.100.77"
#define FAIL(...)                                                                                  \
    do {                                                                                           \
        fprintf(stderr, "udp_tcp_app: " __VA_ARGS__);                                              \
        fprintf(stderr, "\n");                                                                     \
        exit(1);                                                                                   \
    } while (0)

static uint32_t sum16(const uint8_t *p, size_t n, uint32_t acc) { /* RFC 1071 words */
    for (size_t i = 0; i + 1 < n; i += 2) acc += (uint32_t)p[i] << 8 | p[i + 1];
    if (n & 1) acc += (uint32_t)p[n - 1] << 8;
    return acc;
}
static uint16_t fold(uint32_t acc) {
    while (acc >> 16) acc = (acc & 0xFFFF) + (acc >> 16);
    return (uint16_t)~acc;
}

/* one Ethernet/IPv4 frame with a UDP (proto 17) or TCP (6) segment */
static size_t frame(uint8_t *f, const char *src, uint16_t sport, const char *dst, uint16_t dport,
                    int proto, uint8_t tcp_flags, uint32_t seq, uint32_t ack, const void *pl,
                    size_t plen) {
    const size_t l4h = proto == 17 ? 8 : 20, l4 = l4h + plen, tl = 20 + l4;
    memset(f, 0, 14 + tl);
    memcpy(f, "\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02\x08\x00", 14);
    uint8_t *ip = f + 14, *l4p = ip + 20;
    ip[0] = 0x45;
    ip[2] = (uint8_t)(tl >> 8), ip[3] = (uint8_t)tl;
    ip[8] = 64;
    ip[9] = (uint8_t)proto;
    inet_pton(AF_INET, src, ip + 12);
    inet_pton(AF_INET, dst, ip + 16);
    const uint16_t ic = fold(sum16(ip, 20, 0));
    ip[10] = (uint8_t)(ic >> 8), ip[11] = (uint8_t)ic;
    l4p[0] = (uint8_t)(sport >> 8), l4p[1] = (uint8_t)sport;
    l4p[2] = (uint8_t)(dport >> 8), l4p[3] = (uint8_t)dport;
    if (proto == 17) {
        l4p[4] = (uint8_t)(l4 >> 8), l4p[5] = (uint8_t)l4;
    } else {
        for (int k = 0; k < 4; k++) l4p[4 + k] = (uint8_t)(seq >> (24 - 8 * k));
        for (int k = 0; k < 4; k++) l4p[8 + k] = (uint8_t)(ack >> (24 - 8 * k));
        l4p[12] = 0x50;
        l4p[13] = tcp_flags;
        l4p[14] = 0xFF, l4p[15] = 0xFF;
    }
    memcpy(l4p + l4h, pl, plen);
    uint32_t acc = sum16(ip + 12, 8, 0) + proto + (uint32_t)l4; /* pseudo header */
    uint16_t c = fold(sum16(l4p, l4, acc));
    if (proto == 17 && c == 0) c = 0xFFFF;
    uint8_t *cf = l4p + (proto == 17 ? 6 : 16);
    cf[0] = (uint8_t)(c >> 8), cf[1] = (uint8_t)c;
    return 14 + tl;
}

#define MAXF 256
static uint8_t g_pool[MAXF][2048] __attribute__((aligned(64)));
static rxg_mbuf g_mb[MAXF];
static rxg_mbuf *g_mp[MAXF];
static uint32_t g_n;

static void add(size_t len) {
    g_mb[g_n].buf_addr = g_pool[g_n];
    g_mb[g_n].data_off = 0;
    g_mb[g_n].data_len = (uint16_t)len;
    g_mp[g_n] = &g_mb[g_n];
    g_n++;
}

static void burst(int *rcs) {
    const int r = nstack_rx_burst(g_mp, g_n, rcs, NULL);
    if (r < 0) FAIL("nstack_rx_burst: %d", r);
    g_n = 0;
}

int main(void) {
    if (nstack_init(0, 4096, 4096u * 1536u) != RXG_OK) FAIL("nstack_init (needs a GPU)");
    struct sockaddr_in la = {0};
    la.sin_family = AF_INET;
    inet_pton(AF_INET, LOCAL_IP, &la.sin_addr);
    uint8_t mac[6] = {2, 0, 0, 0, 0, 1};
    nstack_set_local(la.sin_addr.s_addr, mac);

    /* UDP server (netfamily.c:211-262) */
    const int ufd = nsocket(AF_INET, SOCK_DGRAM, 0);
    la.sin_port = htons(8889);
    if (ufd < 0 || nbind(ufd, (struct sockaddr *)&la, sizeof(la))) FAIL("udp socket");
    /* TCP server (netfamily.c:284-383) */
    const int lfd = nsocket(AF_INET, SOCK_STREAM, 0);
    la.sin_port = htons(9999);
    if (lfd < 0 || nbind(lfd, (struct sockaddr *)&la, sizeof(la)) || nlisten(lfd, 10))
        FAIL("tcp listener");

    /* burst 1: 100 datagrams from 10.0.0.1:5555, one SYN from 10.0.0.9:40000 */
    char msg[64];
    for (int i = 0; i < 100; i++) {
        const int l = snprintf(msg, sizeof(msg), "datagram %03d", i);
        add(frame(g_pool[g_n], "10.0.0.1", 5555, LOCAL_IP, 8889, 17, 0, 0, 0, msg, (size_t)l));
    }
    add(frame(g_pool[g_n], "10.0.0.9", 40000, LOCAL_IP, 9999, 6, 0x02, 1000, 0, "", 0));
    int rcs[MAXF];
    burst(rcs);
    for (int i = 0; i <= 100; i++)
        if (rcs[i] != 0) FAIL("burst 1 frame %d: rc %d", i, rcs[i]);
    for (int i = 0; i < 100; i++) {
        char buf[128];
        struct sockaddr_in src;
        socklen_t sl = sizeof(src);
        const ssize_t r = nrecvfrom(ufd, buf, sizeof(buf), MSG_DONTWAIT, (struct sockaddr *)&src, &sl);
        const int l = snprintf(msg, sizeof(msg), "datagram %03d", i);
        if (r != l + 8 || memcmp(buf, msg, (size_t)l) || src.sin_port != htons(5555))
            FAIL("datagram %d: r %zd", i, r);
    }

    /* the SYN|ACK goes out through the TX pass (GPU checksums); the client
     * then ACKs it and sends data, one segment with a broken checksum */
    uint8_t tx[4 * 2048];
    uint32_t toff[4];
    uint16_t tlen[4];
    uint64_t span = 0;
    nstack_arp_insert(inet_addr("10.0.0.9"), (uint8_t[6]){2, 0, 0, 0, 0, 9});
    const int ntx = nstack_tx_burst(tx, sizeof(tx), toff, tlen, 4, 1, &span);
    if (ntx < 1) FAIL("tx pass: %d frames", ntx);
    const uint8_t *sa = tx + ((size_t)toff[0] << 6); /* the SYN|ACK */
    if (sa[23] != 6 || (sa[47] & 0x12) != 0x12) FAIL("tx frame is not the SYN|ACK");
    const uint32_t isn = (uint32_t)sa[38] << 24 | sa[39] << 16 | sa[40] << 8 | sa[41];
    add(frame(g_pool[g_n], "10.0.0.9", 40000, LOCAL_IP, 9999, 6, 0x10, 1001, isn + 1, "", 0));
    add(frame(g_pool[g_n], "10.0.0.9", 40000, LOCAL_IP, 9999, 6, 0x18, 1001, isn + 1, "hello, stack", 12));
    const size_t bl = frame(g_pool[g_n], "10.0.0.9", 40000, LOCAL_IP, 9999, 6, 0x18, 1013, isn + 1,
                            "corrupted!", 10);
    g_pool[g_n][bl - 1] ^= 0x5A; /* payload byte: the TCP checksum no longer holds */
    add(bl);
    burst(rcs);
    if (rcs[0] != 0 || rcs[1] != 0 || rcs[2] != RXG_RC_TCP_BAD_CKSUM)
        FAIL("burst 2 rcs %d %d %d", rcs[0], rcs[1], rcs[2]);
    struct sockaddr_in ca;
    socklen_t cl = sizeof(ca);
    const int cfd = naccept(lfd, (struct sockaddr *)&ca, &cl); /* the handshake completed */
    if (cfd < 0 || ca.sin_port != htons(40000)) FAIL("naccept: %d", cfd);
    char data[64];
    const ssize_t r = nrecv(cfd, data, sizeof(data), MSG_DONTWAIT);
    if (r != 12 || memcmp(data, "hello, stack", 12)) FAIL("nrecv: %zd", r);
    if (nrecv(cfd, data, sizeof(data), MSG_DONTWAIT) != -1) FAIL("the corrupted segment was queued");
    const int ntx2 = nstack_tx_burst(tx, sizeof(tx), toff, tlen, 4, 1, &span); /* the data ACK */
    if (ntx2 < 1) FAIL("second tx pass: %d", ntx2);

    /* the pipelined receive: burst B goes to the GPU while burst A is
     * delivered (nstack_rx_submit / nstack_rx_complete); each burst carries
     * 60 datagrams and one segment of the open connection */
    uint32_t first[2];
    int prc[2][MAXF];
    for (int b = 0; b < 2; b++) {
        first[b] = g_n;
        for (int i = 0; i < 60; i++) {
            const int l = snprintf(msg, sizeof(msg), "pipe %d/%02d", b, i);
            add(frame(g_pool[g_n], "10.0.0.1", 5555, LOCAL_IP, 8889, 17, 0, 0, 0, msg, (size_t)l));
        }
        add(frame(g_pool[g_n], "10.0.0.9", 40000, LOCAL_IP, 9999, 6, 0x18, 1013 + 11 * b, isn + 1,
                  b ? "pipelined-2" : "pipelined-1", 11));
    }
    const uint32_t na = first[1] - first[0], nb = g_n - first[1];
    if (nstack_rx_submit(g_mp + first[0], na, prc[0], NULL) != RXG_OK) FAIL("submit A");
    if (nstack_rx_submit(g_mp + first[1], nb, prc[1], NULL) != RXG_OK) FAIL("submit B");
    if (nstack_rx_submit(g_mp + first[1], nb, prc[1], NULL) != RXG_EINVAL) FAIL("a third submit");
    if (nstack_rx_pending() != 2) FAIL("pending %d", nstack_rx_pending());
    if (nstack_rx_complete() != 60 || nstack_rx_complete() != 60) FAIL("completes");
    if (nstack_rx_complete() != RXG_EINVAL) FAIL("a complete with nothing pending");
    g_n = 0;
    for (int b = 0; b < 2; b++)
        for (uint32_t i = 0; i < 61; i++)
            if (prc[b][i] != 0) FAIL("pipelined burst %d frame %u: rc %d", b, i, prc[b][i]);
    for (int b = 0; b < 2; b++)
        for (int i = 0; i < 60; i++) {
            char buf[128];
            const ssize_t r2 = nrecvfrom(ufd, buf, sizeof(buf), MSG_DONTWAIT, NULL, NULL);
            const int l = snprintf(msg, sizeof(msg), "pipe %d/%02d", b, i);
            if (r2 != l + 8 || memcmp(buf, msg, (size_t)l)) FAIL("pipelined datagram %d/%d: %zd", b, i, r2);
        }
    for (int b = 0; b < 2; b++) {
        const ssize_t r2 = nrecv(cfd, data, sizeof(data), MSG_DONTWAIT);
        if (r2 != 11 || memcmp(data, b ? "pipelined-2" : "pipelined-1", 11)) FAIL("pipelined nrecv %d: %zd", b, r2);
    }
    nclose(cfd);
    nclose(lfd);
    nclose(ufd);
    nstack_fini();
    printf("udp_tcp_app ok: 100 + 120 pipelined datagrams, 1 connection, %d + %d frames sent\n", ntx, ntx2);
    return 0;
}
