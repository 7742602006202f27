/*
 * ref_cpu.c — CPU restatement of the reference receive front end.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + bench.py cpu_baseline leg).
 * Not part of the product: librxgpu.so neither links nor calls this code.
 *
 * What it restates (reference = hjlogzw/DPDK-TCP-UDP_Protocol_Stack @ v2):
 *   pkt_process loop body ............ netfamily.c:152-200
 *   udp_process front ................ udp.c:4-57
 *   tcp_process front ................ tcp.c:333-371
 *   get_hostinfo_fromip_port ......... common.c:97-108
 *   tcp_stream_search ................ common.c:31-55
 *   LL_ADD head insert ............... common.h:43-49
 *   checksum (third-party, DPDK 19.11.12 lib/librte_net/rte_ip.h, inlined
 *   into the reference; not vendored in /root/reference — pinned by the
 *   include paths in build/.tcp.o.cmd and .vscode/c_cpp_properties.json:7-8):
 *     __rte_raw_cksum       rte_ip.h:121-138
 *     __rte_raw_cksum_reduce rte_ip.h:151-155
 *     rte_raw_cksum          rte_ip.h:169-174
 *     rte_ipv4_cksum         rte_ip.h:255-265
 *     rte_ipv4_phdr_cksum    rte_ip.h:288-309
 *     rte_ipv4_udptcp_cksum  rte_ip.h:325-349
 *
 * Parity pin: the reference cannot be built here (tcp.c holds unresolved
 * merge-conflict hunks and DPDK headers are absent) and its prebuilt
 * objects (build/ *.o files) are vendored machine code that this project never
 * runs or loads.  The reference ships no tests or fixtures.  This
 * restatement is therefore pinned by (1) the known-answer values SURVEY.md
 * §8(a) records from the reference's compiled code, (2) RFC 1071 §3's
 * published example, (3) the published Microsoft RSS verification vectors
 * (for the RSS hash only).  See tests/golden/ and DESIGN.md §Oracle.
 *
 * Frames shorter than what the reference would read (caplen < bytes it
 * touches) are evaluated on a zero-extended copy and flagged RXG_F_TRUNC:
 * the reference reads adjacent memory there, so parity is defined, not
 * inherited, for those bytes.
 */
#include "ref_cpu.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* byte access helpers (native little-endian words, like the reference) */

static inline uint16_t ld16(const uint8_t *p) {
    uint16_t v;
    memcpy(&v, p, 2);
    return v;
}
static inline uint32_t ld32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

/* ------------------------------------------------------------------ */
/* DPDK 19.11.12 checksum arithmetic                                    */

/* __rte_raw_cksum, rte_ip.h:121-138: 16-bit native words, 4 per step,
 * then single words, then an odd trailing byte placed in the low byte. */
uint32_t oracle_raw_cksum_acc(const void *buf, uint32_t len, uint32_t sum) {
    const uint8_t *u = (const uint8_t *)buf;
    while (len >= 8) {
        sum += ld16(u + 0);
        sum += ld16(u + 2);
        sum += ld16(u + 4);
        sum += ld16(u + 6);
        len -= 8;
        u += 8;
    }
    while (len >= 2) {
        sum += ld16(u);
        len -= 2;
        u += 2;
    }
    if (len == 1) {
        uint16_t left = 0;
        *(uint8_t *)&left = *u;
        sum += left;
    }
    return sum;
}

/* __rte_raw_cksum_reduce, rte_ip.h:151-155: two folds */
static inline uint16_t raw_cksum_reduce(uint32_t sum) {
    sum = ((sum & 0xffff0000u) >> 16) + (sum & 0xffffu);
    sum = ((sum & 0xffff0000u) >> 16) + (sum & 0xffffu);
    return (uint16_t)sum;
}

/* rte_raw_cksum, rte_ip.h:169-174 */
uint16_t oracle_raw_cksum(const void *buf, uint32_t len) {
    return raw_cksum_reduce(oracle_raw_cksum_acc(buf, len, 0));
}

/* rte_ipv4_cksum, rte_ip.h:255-265 (TX only in the reference; used by the
 * tests to build well-formed frames) */
uint16_t oracle_ipv4_cksum(const uint8_t *ipv4_hdr) {
    uint16_t c = oracle_raw_cksum(ipv4_hdr, 20);
    return (uint16_t)((c == 0xffff) ? c : ~c);
}

/* rte_ipv4_phdr_cksum, rte_ip.h:288-309 with ol_flags = 0:
 * psd {src, dst, zero, proto, be16(total_length - 20)}.  The length is a
 * 16-bit subtraction (uint16_t cast in the header), so tl < 20 wraps. */
uint16_t oracle_ipv4_phdr_cksum(const uint8_t *ip) {
    uint8_t psd[12];
    uint16_t l4 = (uint16_t)(be16(ip + 2) - 20);
    memcpy(psd + 0, ip + 12, 4);
    memcpy(psd + 4, ip + 16, 4);
    psd[8] = 0;
    psd[9] = ip[9];
    psd[10] = (uint8_t)(l4 >> 8);
    psd[11] = (uint8_t)(l4 & 0xff);
    return oracle_raw_cksum(psd, 12);
}

/* rte_ipv4_udptcp_cksum, rte_ip.h:325-349 (IHL ignored: l4_len = tl - 20) */
uint16_t oracle_ipv4_udptcp_cksum(const uint8_t *ip, const uint8_t *l4) {
    uint32_t cksum;
    uint32_t l3_len = be16(ip + 2);
    if (l3_len < 20) return 0;
    uint32_t l4_len = l3_len - 20;
    cksum = oracle_raw_cksum(l4, l4_len);
    cksum += oracle_ipv4_phdr_cksum(ip);
    cksum = ((cksum & 0xffff0000u) >> 16) + (cksum & 0xffffu);
    cksum = (~cksum) & 0xffffu;
    if (cksum == 0 && ip[9] == 17) cksum = 0xffff;
    return (uint16_t)cksum;
}

/* ------------------------------------------------------------------ */
/* Control-block lists (common.c:97-108, 31-55; LL_ADD common.h:43-49).
 * Nodes are heap-allocated one by one and padded to the reference's struct
 * sizes (struct localhost 144 B, struct tcp_stream 160 B: SURVEY §8(a)),
 * so the list walk touches memory the way the reference's does. */

typedef struct host_node {
    uint32_t localip;
    uint16_t localport;
    uint8_t protocol;
    uint32_t index;
    struct host_node *next;
    uint8_t _pad[144 - 24];
} host_node;

typedef struct tcb_node {
    uint32_t sip, dip;
    uint16_t sport, dport;
    uint32_t status;
    uint32_t index;
    struct tcb_node *next;
    uint8_t _pad[160 - 32];
} tcb_node;

struct oracle_tables {
    host_node *g_host; /* g_pstHost */
    tcb_node *tcb_set; /* g_pstTcpTbl->tcb_set */
    host_node **hnodes;
    tcb_node **tnodes;
    uint32_t nu, nt;
};

oracle_tables *oracle_tables_new(const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t,
                                 uint32_t nt) {
    oracle_tables *tb = (oracle_tables *)calloc(1, sizeof(*tb));
    if (!tb) return NULL;
    tb->nu = nu;
    tb->nt = nt;
    tb->hnodes = (host_node **)calloc(nu ? nu : 1, sizeof(host_node *));
    tb->tnodes = (tcb_node **)calloc(nt ? nt : 1, sizeof(tcb_node *));
    for (uint32_t i = 0; i < nu; i++) { /* creation order: LL_ADD = head insert */
        host_node *h = (host_node *)calloc(1, sizeof(host_node));
        h->localip = u[i].localip;
        h->localport = u[i].localport;
        h->protocol = u[i].protocol;
        h->index = i;
        h->next = tb->g_host;
        tb->g_host = h;
        tb->hnodes[i] = h;
    }
    for (uint32_t i = 0; i < nt; i++) {
        tcb_node *s = (tcb_node *)calloc(1, sizeof(tcb_node));
        s->sip = t[i].sip;
        s->dip = t[i].dip;
        s->sport = t[i].sport;
        s->dport = t[i].dport;
        s->status = t[i].status;
        s->index = i;
        s->next = tb->tcb_set;
        tb->tcb_set = s;
        tb->tnodes[i] = s;
    }
    return tb;
}

void oracle_tables_free(oracle_tables *tb) {
    if (!tb) return;
    for (uint32_t i = 0; i < tb->nu; i++) free(tb->hnodes[i]);
    for (uint32_t i = 0; i < tb->nt; i++) free(tb->tnodes[i]);
    free(tb->hnodes);
    free(tb->tnodes);
    free(tb);
}

/* get_hostinfo_fromip_port, common.c:97-108: first match in list order */
uint32_t oracle_lookup_udp(const oracle_tables *tb, uint32_t dip, uint16_t port, uint8_t proto) {
    for (const host_node *h = tb->g_host; h != NULL; h = h->next)
        if (dip == h->localip && port == h->localport && proto == h->protocol) return h->index;
    return RXG_FLOW_NONE;
}

/* tcp_stream_search, common.c:31-55: exact 4-tuple (status ignored), then
 * the first LISTEN block on dport (dst IP ignored) */
uint32_t oracle_lookup_tcp(const oracle_tables *tb, uint32_t sip, uint32_t dip, uint16_t sport,
                           uint16_t dport) {
    for (const tcb_node *it = tb->tcb_set; it != NULL; it = it->next)
        if (it->sip == sip && it->dip == dip && it->sport == sport && it->dport == dport)
            return it->index;
    for (const tcb_node *it = tb->tcb_set; it != NULL; it = it->next)
        if (it->dport == dport && it->status == RXG_TCP_STATUS_LISTEN) return it->index;
    return RXG_FLOW_NONE;
}

/* ------------------------------------------------------------------ */
/* Per-frame front end                                                  */

#define SCRATCH_BYTES (65536 + 128)

/* byte read that yields 0 past caplen (the zero-extension rule) */
static inline uint8_t rd8(const uint8_t *f, uint32_t cap, uint32_t i) { return i < cap ? f[i] : 0; }
static inline uint16_t rd16s(const uint8_t *f, uint32_t cap, uint32_t i) {
    return (uint16_t)(rd8(f, cap, i) | (rd8(f, cap, i + 1) << 8));
}
static inline uint32_t rd32s(const uint8_t *f, uint32_t cap, uint32_t i) {
    return (uint32_t)rd16s(f, cap, i) | ((uint32_t)rd16s(f, cap, i + 2) << 16);
}
static inline uint16_t rdbe16s(const uint8_t *f, uint32_t cap, uint32_t i) {
    return (uint16_t)((rd8(f, cap, i) << 8) | rd8(f, cap, i + 1));
}

/* checksum of the frame with the 2-byte field at `hole` taken as 0 —
 * tcp.c:349-351 zeroes it in place; here the caller's bytes are untouched:
 * the frame is copied (zero-extended past caplen) when it is truncated or
 * the hole must be cleared. */
static uint16_t frame_cksum(const uint8_t *f, uint32_t cap, uint32_t hole, uint32_t need,
                            uint8_t *scratch) {
    uint32_t span = need < 52 ? 52 : need; /* bytes the checksum reads: [14, 34 + l4_len) */
    if (span > SCRATCH_BYTES) span = SCRATCH_BYTES;
    uint32_t ncopy = cap < span ? cap : span;
    memcpy(scratch, f, ncopy);
    if (span > ncopy) memset(scratch + ncopy, 0, span - ncopy);
    if (hole + 2 <= span) {
        scratch[hole] = 0;
        scratch[hole + 1] = 0;
    }
    return oracle_ipv4_udptcp_cksum(scratch + 14, scratch + 34);
}

static void classify_one(const oracle_tables *tb, const uint8_t *f, uint32_t cap, rxg_verdict *v,
                         uint8_t *scratch, uint64_t *counts) {
    memset(v, 0, sizeof(*v));
    v->flow_id = RXG_FLOW_NONE;
    uint32_t need;

    /* netfamily.c:154-156, 172: ether_type compared with the big-endian
     * constants, i.e. bytes {08,06} / {08,00} */
    uint16_t et = rdbe16s(f, cap, 12);
    if (et == 0x0806) { /* ARP branch :156-170, then falls through to KNI :194-199 */
        v->cls = RXG_CLS_ARP;
        v->rc = RXG_RC_KNI;
        need = 14 + 28;
    } else if (et != 0x0800) { /* :194-199 */
        v->cls = RXG_CLS_NON_IP;
        v->rc = RXG_RC_KNI;
        need = 14;
    } else {
        uint8_t proto = rd8(f, cap, 23); /* next_proto_id, :178 */
        uint32_t tl = rdbe16s(f, cap, 16);
        uint32_t l4n = tl >= 20 ? tl - 20 : 0; /* rte_ip.h:330-333, IHL ignored */
        if (proto == 17) {
            /* udp_process, udp.c:11-19: udp = ip + 20 */
            uint32_t dip = rd32s(f, cap, 30);
            uint16_t dport = rd16s(f, cap, 36);
            uint32_t dgram_len = rdbe16s(f, cap, 38); /* udp.c:37 (ntohs) */
            uint32_t host = oracle_lookup_udp(tb, dip, dport, 17);
            v->cls = RXG_CLS_UDP;
            v->payload_off = 42;
            v->payload_len = (uint16_t)(dgram_len > 8 ? dgram_len - 8 : 0);
            v->stored_cksum = rd16s(f, cap, 40);
            if (dgram_len <= 8) v->flags |= RXG_F_UDP_SHORT;
            if (host == RXG_FLOW_NONE) {
                v->rc = RXG_RC_UDP_NO_SOCKET; /* udp.c:15-19 */
            } else {
                v->flow_id = host;
                /* udp.c:38-43: rte_malloc(dgram_len - 8) returns NULL for size 0
                 * (dgram_len == 8) and for the wrapped size_t (dgram_len < 8) */
                v->rc = dgram_len <= 8 ? RXG_RC_UDP_NOMEM : RXG_RC_OK;
            }
            need = 42;
            if (34 + l4n > need) need = 34 + l4n;
            if (v->rc == RXG_RC_OK && 42 + (dgram_len - 8) > need) need = 42 + (dgram_len - 8);
            /* informational checksum (the reference never checks UDP on rx) */
            v->l4_cksum = frame_cksum(f, cap, 40, 34 + l4n, scratch);
            v->cksum_ok = v->stored_cksum == v->l4_cksum;
        } else if (proto == 6) {
            /* tcp_process front, tcp.c:345-371 */
            v->cls = RXG_CLS_TCP;
            v->stored_cksum = rd16s(f, cap, 50);                  /* :349 */
            v->l4_cksum = frame_cksum(f, cap, 50, 34 + l4n, scratch); /* :350-351 */
            v->cksum_ok = v->stored_cksum == v->l4_cksum;
            uint32_t hl = (uint32_t)(rd8(f, cap, 46) >> 4) * 4; /* tcp.c:145 */
            int32_t plen = (int32_t)tl - 20 - (int32_t)hl;        /* tcp.c:146, 391 */
            v->payload_off = (uint16_t)(34 + hl);
            if (plen < 0) {
                v->flags |= RXG_F_TCP_NEGLEN;
                plen = 0;
            }
            v->payload_len = (uint16_t)plen;
            if (!v->cksum_ok) {
                v->rc = RXG_RC_TCP_BAD_CKSUM; /* :352-357 */
            } else {
                uint32_t s = oracle_lookup_tcp(tb, rd32s(f, cap, 26), rd32s(f, cap, 30),
                                               rd16s(f, cap, 34), rd16s(f, cap, 36)); /* :361-362 */
                if (s == RXG_FLOW_NONE) {
                    v->rc = RXG_RC_TCP_NO_TCB; /* :363-371 */
                } else {
                    v->flow_id = s;
                    v->rc = RXG_RC_OK;
                }
            }
            need = 54;
            if (34 + l4n > need) need = 34 + l4n;
        } else { /* :188-191 */
            v->cls = RXG_CLS_IPV4_OTHER;
            v->rc = RXG_RC_KNI;
            need = 24;
        }
    }
    if (need > cap) v->flags |= RXG_F_TRUNC;
    if (counts && v->rc == RXG_RC_OK && v->flow_id != RXG_FLOW_NONE)
        counts[(v->cls == RXG_CLS_TCP ? tb->nu : 0) + v->flow_id] += 1;
}

void oracle_classify(const oracle_tables *tb, const uint8_t *pkts, const uint32_t *off,
                     const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out,
                     uint64_t *counts) {
    uint8_t *scratch = (uint8_t *)malloc(SCRATCH_BYTES);
    for (uint32_t i = 0; i < n; i++)
        classify_one(tb, pkts + ((uint64_t)off[i] << off_unit_log2), len[i], &out[i], scratch,
                     counts);
    free(scratch);
}

/* ------------------------------------------------------------------ */
/* TX checksum fill, in place: what ng_encode_udp_apppkt (udp.c:84-95) and
 * ng_encode_tcp_apppkt (tcp.c:444-463) store — rte_ipv4_cksum of the IPv4
 * header and rte_ipv4_udptcp_cksum of the L4 segment, each with its own field
 * zeroed first — for every IPv4 (UDP/TCP) frame of a burst; bytes past the
 * captured length read as 0 and fields not wholly captured are not written. */
void oracle_tx_cksum(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                     uint32_t off_unit_log2) {
    uint8_t *scratch = (uint8_t *)malloc(SCRATCH_BYTES);
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *f = pkts + ((uint64_t)off[i] << off_unit_log2);
        const uint32_t cap = len[i];
        if (rdbe16s(f, cap, 12) != 0x0800) continue;
        uint8_t ip[20];
        for (uint32_t k = 0; k < 20; k++) ip[k] = rd8(f, cap, 14 + k);
        ip[10] = ip[11] = 0; /* pstIp->hdr_checksum = 0 (udp.c:84, tcp.c:444) */
        const uint16_t hc = oracle_ipv4_cksum(ip);
        if (cap >= 26) memcpy(f + 24, &hc, 2);
        const uint8_t proto = ip[9];
        if (proto != 17 && proto != 6) continue;
        const uint32_t tl = rdbe16s(f, cap, 16);
        const uint32_t hole = proto == 17 ? 40 : 50; /* dgram_cksum / cksum = 0 (udp.c:94, tcp.c:462) */
        const uint16_t c = frame_cksum(f, cap, hole, 34 + (tl >= 20 ? tl - 20 : 0), scratch);
        if (cap >= hole + 2) memcpy(f + hole, &c, 2);
    }
    free(scratch);
}

/* ------------------------------------------------------------------ */
/* Toeplitz RSS with the standard 40-byte key (Microsoft RSS spec)       */

static const uint8_t k_rss_key[40] = {
    0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
    0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
    0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};

uint32_t oracle_rss_hash(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport) {
    uint8_t in[12];
    memcpy(in + 0, &sip, 4); /* raw network-order values: memory order = wire order */
    memcpy(in + 4, &dip, 4);
    memcpy(in + 8, &sport, 2);
    memcpy(in + 10, &dport, 2);
    uint32_t result = 0;
    for (int i = 0; i < 12; i++)
        for (int b = 7; b >= 0; b--)
            if (in[i] & (1u << b)) {
                /* 32-bit key window starting at bit (8*i + 7 - b) */
                int pos = 8 * i + (7 - b);
                uint32_t w = 0;
                for (int k = 0; k < 32; k++) {
                    int bit = pos + k;
                    w = (w << 1) | ((k_rss_key[bit >> 3] >> (7 - (bit & 7))) & 1u);
                }
                result ^= w;
            }
    return result;
}
