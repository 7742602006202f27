/*
 * ref_stack.c — CPU restatement of the reference's DELIVERY half: what happens
 * to a frame after the front end's verdict, and what the socket calls then
 * return.  TEST INFRASTRUCTURE ONLY: the checker that host/nstack.c (the
 * product's socket layer over librxgpu) is compared against frame by frame
 * (tests/test_deliver_oracle.py).  librxgpu/libnstack neither link nor call
 * this code.
 *
 * Restated (reference = hjlogzw/DPDK-TCP-UDP_Protocol_Stack):
 *   pkt_process per frame ............... netfamily.c:152-200
 *   udp_process (lookup, offload, ring) . udp.c:4-57
 *   tcp_process (cksum, search, switch) . tcp.c:333-418
 *   tcp_stream_create ................... tcp.c:3-41
 *   tcp_handle_listen / _syn_rcvd ....... tcp.c:43-87, 89-131
 *   ng_tcp_enqueue_recvbuffer ........... tcp.c:133-185
 *   ng_tcp_send_ackpkt .................. tcp.c:187-216
 *   tcp_handle_established .............. tcp.c:218-297
 *   tcp_handle_close_wait / _last_ack ... tcp.c:299-331
 *   nsocket/nbind/nlisten/naccept ....... common.c:262-416
 *   nrecv / nrecvfrom ................... common.c:462-515, 517-565
 *   nclose .............................. common.c:609-666
 *   get_fd_frombitmap/set_fd ............ common.c:72-95
 *   get_accept_tcb ...................... common.c:58-70
 *   get_hostinfo_fromip_port ............ common.c:97-108
 *   tcp_stream_search ................... common.c:31-55
 * Merge-conflict hunks of tcp.c: the HEAD side (rcv_nxt += payloadlen,
 * :244-248; rcv_nxt + 1, :266-279).  The lists are head-inserted (LL_ADD,
 * common.h:43-49), so a list walk meets the newest block first.
 *
 * Where the reference's behaviour is undefined the oracle defines it, and the
 * product must match these definitions (tested):
 *   - bytes past a frame's captured length read as 0 (the reference reads the
 *     adjacent mbuf memory);
 *   - nrecvfrom copies offload.length = dgram_len bytes out of a buffer of
 *     dgram_len - 8 bytes (udp.c:37-38 vs common.c:558-559): the 8 bytes past
 *     the payload read as 0 here (adjacent heap memory in the reference);
 *   - the initial send sequence number (rand_r seeded with time(NULL),
 *     tcp.c:30-31) is not compared: the tests compare snd_nxt only once an
 *     ACK has set it (tcp.c:249, :275).
 * Deliberate divergences of the product, not restated here: blocking calls
 * (the oracle and the tests use the non-blocking outcome: -2 = would block),
 * get_hostinfo_fromfd's loop bug (common.c:116: the oracle walks correctly,
 * as the product does; the reference loops forever past the second socket).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ref_cpu.h"

#define O_DEFAULT_FD 3     /* D_DEFAULT_FD_NUM, common.h:32 */
#define O_MAX_FD 1024      /* D_MAX_FD_COUNT, common.h:33 */
#define O_WOULD_BLOCK (-2) /* a blocking call that would wait */

enum { ST_CLOSED = 0, ST_LISTEN, ST_SYN_RCVD, ST_SYN_SENT, ST_ESTABLISHED, ST_FIN_WAIT_1,
       ST_FIN_WAIT_2, ST_CLOSING, ST_TIME_WAIT, ST_CLOSE_WAIT, ST_LAST_ACK }; /* tcp.h:10-26 */
enum { F_FIN = 0x01, F_SYN = 0x02, F_PSH = 0x08, F_ACK = 0x10 };

/* a FIFO standing in for rte_ring (enqueue at the tail, dequeue at the head) */
typedef struct o_item {
    void *p;
    struct o_item *next;
} o_item;
typedef struct {
    o_item *head, *tail;
} o_fifo;

static void fifo_put(o_fifo *q, void *p) {
    o_item *it = (o_item *)calloc(1, sizeof(*it));
    it->p = p;
    if (q->tail)
        q->tail->next = it;
    else
        q->head = it;
    q->tail = it;
}
static void *fifo_get(o_fifo *q) {
    o_item *it = q->head;
    if (!it) return NULL;
    q->head = it->next;
    if (!q->head) q->tail = NULL;
    void *p = it->p;
    free(it);
    return p;
}

typedef struct { /* struct offload, udp.h:31-44 */
    uint32_t sip, dip;
    uint16_t sport, dport;
    uint16_t length;
    uint8_t *data; /* `length` readable bytes: payload, then zeros (see header) */
} o_offload;

typedef struct { /* struct tcp_fragment, tcp.h:67-84 */
    uint16_t sport, dport;
    uint32_t seqnum, acknum;
    uint8_t tcp_flags;
    int32_t length;
    uint8_t *data;
} o_frag;

typedef struct o_host { /* struct localhost, udp.h:10-29 */
    int fd;
    uint32_t localip;
    uint16_t localport;
    uint8_t protocol;
    o_fifo rcvbuf;
    struct o_host *next;
} o_host;

typedef struct o_tcb { /* struct tcp_stream, tcp.h:29-55 */
    int fd;
    uint32_t sip, dip;
    uint16_t sport, dport;
    uint8_t protocol;
    int status;
    uint32_t snd_nxt, rcv_nxt;
    int snd_known; /* snd_nxt set from an ACK (not the random ISN) */
    o_fifo rcvbuf, sndbuf;
    struct o_tcb *next;
} o_tcb;

struct oracle_stack {
    o_host *hosts;  /* g_pstHost */
    o_tcb *tcbs;    /* g_pstTcpTbl->tcb_set */
    uint8_t fdbits[O_MAX_FD / 8];
};

oracle_stack *oracle_stack_new(void) { return (oracle_stack *)calloc(1, sizeof(oracle_stack)); }

static void free_fifo(o_fifo *q, int frag) {
    void *p;
    while ((p = fifo_get(q)) != NULL) {
        free(frag ? ((o_frag *)p)->data : ((o_offload *)p)->data);
        free(p);
    }
}

void oracle_stack_free(oracle_stack *st) {
    if (!st) return;
    for (o_host *h = st->hosts, *n; h; h = n) {
        n = h->next;
        free_fifo(&h->rcvbuf, 0);
        free(h);
    }
    for (o_tcb *s = st->tcbs, *n; s; s = n) {
        n = s->next;
        free_fifo(&s->rcvbuf, 1);
        free_fifo(&s->sndbuf, 1);
        free(s);
    }
    free(st);
}

/* common.c:72-95 */
static int fd_get(oracle_stack *st) {
    for (int fd = O_DEFAULT_FD; fd < O_MAX_FD; fd++)
        if (!(st->fdbits[fd / 8] & (1u << (fd % 8)))) {
            st->fdbits[fd / 8] |= (uint8_t)(1u << (fd % 8));
            return fd;
        }
    return -1;
}
static void fd_put(oracle_stack *st, int fd) {
    if (fd >= 0 && fd < O_MAX_FD) st->fdbits[fd / 8] &= (uint8_t)~(1u << (fd % 8));
}

static o_host *host_of_fd(oracle_stack *st, int fd) {
    for (o_host *h = st->hosts; h; h = h->next)
        if (h->fd == fd) return h;
    return NULL;
}
static o_tcb *tcb_of_fd(oracle_stack *st, int fd) {
    for (o_tcb *s = st->tcbs; s; s = s->next)
        if (s->fd == fd) return s;
    return NULL;
}

/* nsocket, common.c:262-340: a fd, a control block head-inserted into its list */
int oracle_nsocket(oracle_stack *st, int type) {
    int fd = fd_get(st);
    if (type == 2) { /* SOCK_DGRAM */
        o_host *h = (o_host *)calloc(1, sizeof(*h));
        h->fd = fd;
        h->protocol = 17;
        h->next = st->hosts;
        st->hosts = h;
    } else if (type == 1) { /* SOCK_STREAM */
        o_tcb *s = (o_tcb *)calloc(1, sizeof(*s));
        s->fd = fd;
        s->protocol = 6;
        s->next = st->tcbs;
        st->tcbs = s;
    }
    return fd;
}

/* nbind, common.c:342-371 (raw network-order ip / port) */
int oracle_nbind(oracle_stack *st, int fd, uint32_t ip, uint16_t port) {
    o_host *h = host_of_fd(st, fd);
    if (h) {
        h->localport = port;
        h->localip = ip;
        return 0;
    }
    o_tcb *s = tcb_of_fd(st, fd);
    if (!s) return -1;
    s->dport = port;
    s->dip = ip;
    s->status = ST_CLOSED;
    return 0;
}

/* nlisten, common.c:373-386 */
int oracle_nlisten(oracle_stack *st, int fd) {
    o_tcb *s = tcb_of_fd(st, fd);
    if (!s) return host_of_fd(st, fd) ? 0 : -1;
    s->status = ST_LISTEN;
    return 0;
}

/* naccept, common.c:388-416 with get_accept_tcb :58-70: the first (newest)
 * tcb on the listener's port without a fd; none = would block */
int oracle_naccept(oracle_stack *st, int fd, uint32_t *sip, uint16_t *sport) {
    o_tcb *l = tcb_of_fd(st, fd);
    if (!l) return -1;
    for (o_tcb *a = st->tcbs; a; a = a->next)
        if (a->dport == l->dport && a->fd == -1) {
            a->fd = fd_get(st);
            if (sip) *sip = a->sip;
            if (sport) *sport = a->sport;
            return a->fd;
        }
    return O_WOULD_BLOCK;
}

/* nclose, common.c:609-666 */
int oracle_nclose(oracle_stack *st, int fd) {
    o_host *h = host_of_fd(st, fd);
    if (h) {
        o_host **pp = &st->hosts;
        while (*pp != h) pp = &(*pp)->next;
        *pp = h->next;
        free_fifo(&h->rcvbuf, 0);
        free(h);
        fd_put(st, fd);
        return 0;
    }
    o_tcb *s = tcb_of_fd(st, fd);
    if (!s) return -1;
    if (s->status != ST_LISTEN) { /* queue FIN|ACK, wait in LAST_ACK */
        o_frag *f = (o_frag *)calloc(1, sizeof(*f));
        f->sport = s->dport;
        f->dport = s->sport;
        f->seqnum = s->snd_nxt;
        f->acknum = s->rcv_nxt;
        f->tcp_flags = F_FIN | F_ACK;
        fifo_put(&s->sndbuf, f);
        s->status = ST_LAST_ACK;
        fd_put(st, fd);
    } else { /* the listener leaves the list (its fd stays taken, :658-662) */
        o_tcb **pp = &st->tcbs;
        while (*pp != s) pp = &(*pp)->next;
        *pp = s->next;
        free_fifo(&s->rcvbuf, 1);
        free_fifo(&s->sndbuf, 1);
        free(s);
    }
    return 0;
}

/* byte reads with the zero-extension rule */
static uint8_t b8(const uint8_t *f, uint32_t cap, uint32_t i) { return i < cap ? f[i] : 0; }
static uint16_t raw16(const uint8_t *f, uint32_t cap, uint32_t i) {
    return (uint16_t)(b8(f, cap, i) | (b8(f, cap, i + 1) << 8));
}
static uint32_t raw32(const uint8_t *f, uint32_t cap, uint32_t i) {
    return (uint32_t)raw16(f, cap, i) | ((uint32_t)raw16(f, cap, i + 2) << 16);
}
static uint32_t be16v(const uint8_t *f, uint32_t cap, uint32_t i) {
    return ((uint32_t)b8(f, cap, i) << 8) | b8(f, cap, i + 1);
}
static uint32_t be32v(const uint8_t *f, uint32_t cap, uint32_t i) {
    return (be16v(f, cap, i) << 16) | be16v(f, cap, i + 2);
}

/* udp_process, udp.c:4-57: the reference's own return codes */
static int udp_rx(oracle_stack *st, const uint8_t *f, uint32_t cap) {
    const uint32_t dip = raw32(f, cap, 30);
    const uint16_t dport = raw16(f, cap, 36);
    o_host *h = NULL;
    for (o_host *x = st->hosts; x; x = x->next) /* get_hostinfo_fromip_port, common.c:97-108 */
        if (x->localip == dip && x->localport == dport && x->protocol == 17) {
            h = x;
            break;
        }
    if (!h) return -3;
    const uint32_t dgram_len = be16v(f, cap, 38); /* udp.c:37 */
    if (dgram_len <= 8) return -2; /* rte_malloc(dgram_len - 8): size 0 / wrapped -> NULL (:38-44) */
    o_offload *o = (o_offload *)calloc(1, sizeof(*o));
    o->sip = raw32(f, cap, 26);
    o->dip = dip;
    o->sport = raw16(f, cap, 34);
    o->dport = dport;
    o->length = (uint16_t)dgram_len;
    o->data = (uint8_t *)calloc(1, dgram_len);
    for (uint32_t k = 0; k < dgram_len - 8; k++) o->data[k] = b8(f, cap, 42 + k); /* :46 */
    fifo_put(&h->rcvbuf, o); /* :48 */
    return 0;
}

/* tcp_stream_search, common.c:31-55 */
static o_tcb *tcb_search(oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport,
                         uint16_t dport) {
    for (o_tcb *s = st->tcbs; s; s = s->next)
        if (s->sip == sip && s->dip == dip && s->sport == sport && s->dport == dport) return s;
    for (o_tcb *s = st->tcbs; s; s = s->next)
        if (s->dport == dport && s->status == ST_LISTEN) return s;
    return NULL;
}

/* ng_tcp_enqueue_recvbuffer, tcp.c:133-185 */
static void enqueue_recv(o_tcb *s, const uint8_t *f, uint32_t cap, int tcplen) {
    o_frag *fr = (o_frag *)calloc(1, sizeof(*fr));
    const uint32_t hdrlen = b8(f, cap, 46) >> 4;
    const int payloadlen = tcplen - (int)hdrlen * 4;
    if (payloadlen > 0) {
        fr->data = (uint8_t *)calloc(1, (size_t)payloadlen + 1);
        for (int k = 0; k < payloadlen; k++) fr->data[k] = b8(f, cap, 34 + hdrlen * 4 + (uint32_t)k);
        fr->length = payloadlen;
    } /* == 0, and < 0 (memset 0): a 0-length fragment */
    fifo_put(&s->rcvbuf, fr);
}

/* ng_tcp_send_ackpkt, tcp.c:187-216 */
static void send_ack(o_tcb *s, const uint8_t *f, uint32_t cap) {
    o_frag *a = (o_frag *)calloc(1, sizeof(*a));
    a->dport = raw16(f, cap, 34);
    a->sport = raw16(f, cap, 36);
    a->acknum = s->rcv_nxt;
    a->seqnum = s->snd_nxt;
    a->tcp_flags = F_ACK;
    fifo_put(&s->sndbuf, a);
}

/* tcp_process, tcp.c:333-418, after the front end's checksum verdict */
static int tcp_rx(oracle_stack *st, const uint8_t *f, uint32_t cap) {
    o_tcb *s = tcb_search(st, raw32(f, cap, 26), raw32(f, cap, 30), raw16(f, cap, 34),
                          raw16(f, cap, 36));
    if (!s) return -2;
    const uint8_t fl = b8(f, cap, 47);
    switch (s->status) {
    case ST_LISTEN: /* tcp_handle_listen, tcp.c:43-87 */
        if (fl & F_SYN) {
            o_tcb *n = (o_tcb *)calloc(1, sizeof(*n)); /* tcp_stream_create, tcp.c:3-41 */
            n->sip = raw32(f, cap, 26);
            n->dip = raw32(f, cap, 30);
            n->sport = raw16(f, cap, 34);
            n->dport = raw16(f, cap, 36);
            n->protocol = 6;
            n->fd = -1;
            n->status = ST_LISTEN;
            n->next = st->tcbs; /* LL_ADD, :52 */
            st->tcbs = n;
            o_frag *sa = (o_frag *)calloc(1, sizeof(*sa));
            sa->sport = raw16(f, cap, 36);
            sa->dport = raw16(f, cap, 34);
            sa->seqnum = n->snd_nxt; /* the random ISN: not compared */
            sa->acknum = be32v(f, cap, 38) + 1;
            n->rcv_nxt = sa->acknum;
            sa->tcp_flags = F_SYN | F_ACK;
            fifo_put(&n->sndbuf, sa);
            n->status = ST_SYN_RCVD;
        }
        break;
    case ST_SYN_RCVD: /* tcp_handle_syn_rcvd, tcp.c:89-131 */
        if (fl & F_ACK) s->status = ST_ESTABLISHED;
        break;
    case ST_ESTABLISHED: { /* tcp_handle_established, tcp.c:218-297 */
        const int tcplen = (int)be16v(f, cap, 16) - 20; /* :391 */
        if (fl & F_PSH) {
            enqueue_recv(s, f, cap, tcplen);
            const int payloadlen = tcplen - (int)(b8(f, cap, 46) >> 4) * 4;
            s->rcv_nxt = s->rcv_nxt + (uint32_t)payloadlen;
            s->snd_nxt = be32v(f, cap, 42);
            s->snd_known = 1;
            send_ack(s, f, cap);
        }
        if (fl & F_FIN) {
            s->status = ST_CLOSE_WAIT;
            enqueue_recv(s, f, cap, b8(f, cap, 46) >> 4); /* tcplen = the data offset field */
            s->rcv_nxt = s->rcv_nxt + 1;
            s->snd_nxt = be32v(f, cap, 42);
            s->snd_known = 1;
            send_ack(s, f, cap);
        }
        break;
    }
    case ST_LAST_ACK: /* tcp_handle_last_ack, tcp.c:312-331 */
        if (fl & F_ACK) {
            o_tcb **pp = &st->tcbs;
            while (*pp != s) pp = &(*pp)->next;
            *pp = s->next;
            free_fifo(&s->rcvbuf, 1);
            free_fifo(&s->sndbuf, 1);
            free(s);
        }
        break;
    default: /* CLOSED, SYN_SENT, FIN_WAIT_*, CLOSING, TIME_WAIT, CLOSE_WAIT */
        break;
    }
    return 0;
}

/* pkt_process loop body, netfamily.c:152-200, for one frame: udp_process /
 * tcp_process return codes, 1 for a frame handed to KNI.  The TCP checksum
 * verdict (tcp.c:349-357) is the front end's (oracle_classify). */
int oracle_rx(oracle_stack *st, const uint8_t *f, uint32_t cap) {
    if (be16v(f, cap, 12) != 0x0800) return 1;
    const uint8_t proto = b8(f, cap, 23);
    if (proto == 17) return udp_rx(st, f, cap);
    if (proto != 6) return 1;
    oracle_tables *none = oracle_tables_new(NULL, 0, NULL, 0);
    uint32_t off = 0;
    uint16_t len = (uint16_t)cap;
    rxg_verdict v;
    oracle_classify(none, f, &off, &len, 1, 4, &v, NULL); /* the checksum half of tcp_process */
    oracle_tables_free(none);
    if (!v.cksum_ok) return -1;
    return tcp_rx(st, f, cap);
}

/* a burst of frames through oracle_rx in order, as the reference's
 * pkt_process loop calls udp_process / tcp_process (the socket-API rate's
 * CPU baseline, bench.py); rcs nullable */
void oracle_rx_burst(oracle_stack *st, const uint8_t *pkts, const uint32_t *off,
                     const uint16_t *len, uint32_t n, uint32_t unit_log2, int32_t *rcs) {
    for (uint32_t i = 0; i < n; i++) {
        const int r = oracle_rx(st, pkts + ((uint64_t)off[i] << unit_log2), len[i]);
        if (rcs) rcs[i] = r;
    }
}

/* the application side of the same baseline: every socket read until empty
 * (nrecvfrom / nrecv), every tcb's queued control fragments dropped (sent);
 * returns the items received, *bytes their returned lengths */
long oracle_drain_all(oracle_stack *st, uint8_t *buf, size_t cap, uint64_t *bytes) {
    long got = 0;
    uint64_t nb = 0;
    for (o_host *h = st->hosts; h; h = h->next) {
        long r;
        while ((r = oracle_nrecvfrom(st, h->fd, buf, cap, NULL, NULL)) >= 0) got++, nb += (uint64_t)r;
    }
    for (o_tcb *s = st->tcbs; s; s = s->next) {
        o_frag *fr;
        while ((fr = (o_frag *)fifo_get(&s->rcvbuf)) != NULL) {
            if (fr->length > 0) {
                memcpy(buf, fr->data, (size_t)fr->length < cap ? (size_t)fr->length : cap);
                got++, nb += (uint64_t)fr->length;
            }
            free(fr->data);
            free(fr);
        }
        while ((fr = (o_frag *)fifo_get(&s->sndbuf)) != NULL) {
            free(fr->data);
            free(fr);
        }
    }
    if (bytes) *bytes = nb;
    return got;
}

/* nrecvfrom, common.c:517-565 (non-blocking outcome) */
long oracle_nrecvfrom(oracle_stack *st, int fd, uint8_t *buf, size_t len, uint32_t *sip,
                      uint16_t *sport) {
    o_host *h = host_of_fd(st, fd);
    if (!h) return -1;
    o_offload *o = (o_offload *)fifo_get(&h->rcvbuf);
    if (!o) return O_WOULD_BLOCK;
    if (sip) *sip = o->sip;
    if (sport) *sport = o->sport;
    if (len < o->length) { /* :542-556: len bytes out, the rest to the TAIL of the ring */
        memcpy(buf, o->data, len);
        const uint16_t rest = (uint16_t)(o->length - len);
        uint8_t *p = (uint8_t *)calloc(1, rest);
        memcpy(p, o->data + len, rest);
        free(o->data);
        o->data = p;
        o->length = rest;
        fifo_put(&h->rcvbuf, o);
        return (long)len;
    }
    const long n = o->length; /* :558-564 */
    memcpy(buf, o->data, o->length);
    free(o->data);
    free(o);
    return n;
}

/* nrecv, common.c:462-515 (non-blocking outcome) */
long oracle_nrecv(oracle_stack *st, int fd, uint8_t *buf, size_t len) {
    o_tcb *s = tcb_of_fd(st, fd);
    if (!s) return host_of_fd(st, fd) ? 0 : -1;
    o_frag *fr = (o_frag *)fifo_get(&s->rcvbuf);
    if (!fr) return O_WOULD_BLOCK;
    if ((size_t)fr->length > len) { /* :483-496: shift, re-enqueue, return the REST's length */
        memcpy(buf, fr->data, len);
        for (uint32_t i = 0; i < (uint32_t)fr->length - len; i++) fr->data[i] = fr->data[len + i];
        fr->length = fr->length - (int32_t)len;
        const long r = fr->length;
        fifo_put(&s->rcvbuf, fr);
        return r;
    }
    if (fr->length == 0) { /* :497-501: EOF */
        free(fr->data);
        free(fr);
        return 0;
    }
    const long r = fr->length; /* :502-511 */
    memcpy(buf, fr->data, (size_t)fr->length);
    free(fr->data);
    free(fr);
    return r;
}

/* state of the tcb with this exact 4-tuple (raw network order): -1 none,
 * 1 found with snd_nxt set by an ACK, 0 found with snd_nxt the random ISN */
int oracle_tcb_state(const oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport,
                     uint16_t dport, int32_t *status, uint32_t *rcv_nxt, uint32_t *snd_nxt,
                     int32_t *fd) {
    for (const o_tcb *s = st->tcbs; s; s = s->next)
        if (s->sip == sip && s->dip == dip && s->sport == sport && s->dport == dport) {
            if (status) *status = s->status;
            if (rcv_nxt) *rcv_nxt = s->rcv_nxt;
            if (snd_nxt) *snd_nxt = s->snd_known ? s->snd_nxt : 0;
            if (fd) *fd = s->fd;
            return s->snd_known ? 1 : 0;
        }
    return -1;
}

/* the k-th fragment queued for transmission by that tcb (sndbuf): flags,
 * acknum, and seqnum when it is not the random ISN; 0 found */
int oracle_tcb_sndq(const oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport,
                    uint16_t dport, uint32_t k, uint8_t *flags, uint32_t *acknum) {
    for (const o_tcb *s = st->tcbs; s; s = s->next)
        if (s->sip == sip && s->dip == dip && s->sport == sport && s->dport == dport) {
            const o_item *it = s->sndbuf.head;
            for (uint32_t i = 0; it && i < k; i++) it = it->next;
            if (!it) return -1;
            const o_frag *fr = (const o_frag *)it->p;
            if (flags) *flags = fr->tcp_flags;
            if (acknum) *acknum = fr->acknum;
            return 0;
        }
    return -1;
}

/* test hook: a tcb installed as tcp_stream_create + LL_ADD would leave it
 * (tcp.c:3-52), with the given status (e.g. ESTABLISHED, as after a
 * handshake); the counterpart of nstack_tcb_add, for tests that need many
 * connections without running their handshakes through both stacks */
int oracle_tcb_add(oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport,
                   int status) {
    o_tcb *n = (o_tcb *)calloc(1, sizeof(*n));
    if (!n) return -1;
    n->sip = sip;
    n->dip = dip;
    n->sport = sport;
    n->dport = dport;
    n->protocol = 6;
    n->fd = -1;
    n->status = status;
    n->next = st->tcbs; /* LL_ADD */
    st->tcbs = n;
    return 0;
}

/* number of tcbs in the list (control blocks the stack holds) */
uint32_t oracle_tcb_count(const oracle_stack *st) {
    uint32_t n = 0;
    for (const o_tcb *s = st->tcbs; s; s = s->next) n++;
    return n;
}
