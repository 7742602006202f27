/*
 * rxgpu.h — C ABI of the MI355X receive front end (librxgpu.so).
 *
 * Replaces the per-frame body of the reference's protocol lcore loop
 * (pkt_process, netfamily.c:152-200) and the front halves of
 *   int udp_process(struct rte_mbuf *)   udp.h:6,  udp.c:4-57
 *   int tcp_process(struct rte_mbuf *)   tcp.h:6,  tcp.c:333-371
 * together with the two flow lookups they call
 *   get_hostinfo_fromip_port(dip, port, proto)       common.c:97-108
 *   tcp_stream_search(sip, dip, sport, dport)        common.c:31-55
 * and the DPDK 19.11.12 checksum they call (rte_ip.h:121-349, inlined
 * into the reference as rte_ipv4_udptcp_cksum).
 *
 * A per-frame GPU call is meaningless, so the boundary is a BURST: the
 * caller hands over N frames (packed buffer + offsets + lengths) and gets
 * back N 16-byte verdicts that carry exactly what the reference functions
 * decide per frame (return code, matched control block, payload window,
 * checksum).  Plain pointers and sizes only; no C++ or torch types.
 *
 * Threading: one rxg_ctx per rx thread; a context is not thread-safe.
 * Streams: bursts may run on any streams; the stream of a context's most
 * recent burst call must still exist at the context's next call (table
 * writes are ordered after it by an event recorded then).
 * Every call that touches the device switches the calling thread to the
 * context's device and back: the thread's current device is unchanged.
 * Errors: API calls return 0 or a negative RXG_E* code (rxg_strerror);
 * the library never exits the process (the reference rte_exit()s).
 */
#ifndef RXGPU_H
#define RXGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- verdict --------------------------------------------------------- */

#define RXG_FLOW_NONE 0xFFFFFFFFu

/* frame class: the branch pkt_process takes (netfamily.c:156-199) */
enum {
    RXG_CLS_ARP = 0,        /* ether_type == BE 0x0806 (then also KNI, :194-199) */
    RXG_CLS_NON_IP = 1,     /* any other non-IPv4 ether_type -> KNI (:194-199) */
    RXG_CLS_IPV4_OTHER = 2, /* IPv4, next_proto_id not 6/17 -> KNI (:188-191) */
    RXG_CLS_UDP = 3,        /* IPv4 proto 17 -> udp_process (:178-181) */
    RXG_CLS_TCP = 4         /* IPv4 proto 6  -> tcp_process (:183-186) */
};

/* per-frame return codes, identical to the reference's */
enum {
    RXG_RC_OK = 0,              /* udp.c:56 / tcp.c:417 */
    RXG_RC_TCP_BAD_CKSUM = -1,  /* tcp.c:352-357 */
    RXG_RC_TCP_NO_TCB = -2,     /* tcp.c:363-371 */
    RXG_RC_UDP_NOMEM = -2,      /* udp.c:38-43: rte_malloc(dgram_len-8) fails when
                                   dgram_len <= 8 (size 0 or wrapped size_t) */
    RXG_RC_UDP_NO_SOCKET = -3,  /* udp.c:15-19 */
    RXG_RC_KNI = 1              /* non-TCP/UDP frame handed to KNI */
};

/* verdict.flags */
#define RXG_F_TRUNC 0x01     /* the reference would read past the captured frame
                                (ip total_length or dgram_len beyond caplen): the
                                bytes past caplen are taken as zero here; the
                                reference reads adjacent memory (parity undefined) */
#define RXG_F_TCP_NEGLEN 0x02 /* TCP tl-20-hl < 0 (reference enqueues 0-length, tcp.c:157) */
#define RXG_F_UDP_SHORT 0x04  /* UDP dgram_len <= 8 (rc -2, see RXG_RC_UDP_NOMEM) */

typedef struct rxg_verdict {
    uint32_t flow_id;      /* stable id of the matched control block (UDP and TCP
                              ids are separate spaces): id i for block i of the
                              arrays given to rxg_flows_sync, or the id
                              rxg_flows_add assigned.  A removed block's id may be
                              reused by a later add.  RXG_FLOW_NONE if no match /
                              not looked up */
    uint16_t payload_off;  /* UDP: 42 (udp.c:46 copies from udp+1); TCP: 34+hl */
    uint16_t payload_len;  /* UDP: dgram_len-8 (udp.c:38); TCP: tl-20-hl (tcp.c:145-159);
                              clamped at 0 (see flags) */
    uint16_t l4_cksum;     /* rte_ipv4_udptcp_cksum with the L4 checksum field
                              taken as 0 (tcp.c:349-351); 0 for non TCP/UDP */
    uint8_t cls;           /* RXG_CLS_* */
    int8_t rc;             /* RXG_RC_* */
    uint8_t cksum_ok;      /* stored == l4_cksum (TCP verdict input; informational
                              for UDP, which the reference never verifies) */
    uint8_t flags;         /* RXG_F_* */
    uint16_t stored_cksum; /* the L4 checksum field as stored in the frame (LE u16) */
} rxg_verdict;

/* Compact 8-byte verdict (rxg_classify_dev8): the same decision in half the
 * bytes, for the device-resident burst loop, where the verdict array is a
 * quarter of the HBM traffic at 64-B frames.  It carries everything the
 * reference decides per frame (return code, matched block, payload window,
 * checksum pass/fail, class, flags); only the two checksum VALUES of the
 * 16-byte form (l4_cksum, stored_cksum) are left out — cksum_ok is their
 * comparison.  Field for field it equals rxg_verdict8_of(the 16-byte verdict). */
typedef struct rxg_verdict8 {
    uint32_t flow_id;     /* = rxg_verdict.flow_id */
    uint16_t payload_len; /* = rxg_verdict.payload_len */
    uint8_t off_neg;      /* bits 0-6: payload_off (0, 42 or 34 + 4*hl <= 94);
                             bit 7: RXG_F_TCP_NEGLEN */
    uint8_t status;       /* bits 0-2: cls; bits 3-5: rc (3-bit two's complement);
                             bit 6: cksum_ok; bit 7: RXG_F_TRUNC */
} rxg_verdict8;

#define RXG_V8_PAYLOAD_OFF(v) ((uint32_t)((v).off_neg & 0x7Fu))
#define RXG_V8_CLS(v) ((uint32_t)((v).status & 7u))
#define RXG_V8_RC(v) ((int32_t)(((v).status >> 3) & 7u) - (int32_t)((((v).status >> 3) & 4u) << 1))
#define RXG_V8_CKSUM_OK(v) ((uint32_t)(((v).status >> 6) & 1u))
/* RXG_F_* of the 16-byte form (UDP_SHORT: a UDP frame with payload_len 0) */
#define RXG_V8_FLAGS(v)                                                                 \
    ((uint32_t)((v).status >> 7) | ((uint32_t)((v).off_neg >> 7) << 1) |              \
     ((RXG_V8_CLS(v) == RXG_CLS_UDP && (v).payload_len == 0) ? (uint32_t)RXG_F_UDP_SHORT : 0u))

static inline rxg_verdict8 rxg_verdict8_of(const rxg_verdict *v) {
    rxg_verdict8 r;
    r.flow_id = v->flow_id;
    r.payload_len = v->payload_len;
    r.off_neg = (uint8_t)((v->payload_off & 0x7Fu) | ((v->flags & RXG_F_TCP_NEGLEN) ? 0x80u : 0u));
    r.status = (uint8_t)((v->cls & 7u) | (((uint32_t)(uint8_t)v->rc & 7u) << 3) |
                         ((v->cksum_ok & 1u) << 6) | ((v->flags & RXG_F_TRUNC) ? 0x80u : 0u));
    return r;
}

/* ---- control-block snapshot (flow table source) ---------------------- */

/* One UDP socket = one `struct localhost` of the reference (udp.h:10-29).
 * Fields are raw network-order values exactly as the reference stores them
 * (nbind, common.c:350-353). */
typedef struct rxg_udp_sock {
    uint32_t localip;
    uint16_t localport;
    uint8_t protocol; /* IPPROTO_UDP for every socket nsocket() makes */
    uint8_t _pad;
} rxg_udp_sock;

/* One `struct tcp_stream` (tcp.h:29-55): key fields + status. sip/sport are
 * the remote side as read from the packet (tcp_stream_create, tcp.c:16-19). */
typedef struct rxg_tcb {
    uint32_t sip;
    uint32_t dip;
    uint16_t sport;
    uint16_t dport;
    uint32_t status; /* TCP_STATUS_* of tcp.h:10-26; LISTEN == 1 */
} rxg_tcb;

#define RXG_TCP_STATUS_LISTEN 1u

/* ---- mbuf-shaped descriptor (rte_mbuf field offsets, DPDK 19.11) ------- */
typedef struct rxg_mbuf {
    void *buf_addr;        /* @0  */
    uint8_t _r0[8];
    uint16_t data_off;     /* @16 */
    uint16_t refcnt;       /* @18: references (rte_mbuf_refcnt); librxgpu never reads it,
                              libnstack's in-place delivery holds frames with it */
    uint8_t _r1[20];
    uint16_t data_len;     /* @40 */
    uint8_t _r2[86];
} rxg_mbuf;                /* 128 bytes, like rte_mbuf */

/* ---- error codes ------------------------------------------------------ */
enum {
    RXG_OK = 0,
    RXG_EINVAL = -22,
    RXG_ENOMEM = -12,
    RXG_ENODEV = -19,
    RXG_ERANGE = -34,
    RXG_EHIP = -1000, /* HIP runtime error (details: rxg_last_hip_error) */
    RXG_ECOMM = -1001 /* RCCL error (details: rxg_last_hip_error) */
};

typedef struct rxg_ctx rxg_ctx;

/* device argument of rxg_open for a control-plane-only context: flow tables
 * and host lookups work, every burst call returns RXG_ENODEV */
#define RXG_HOST_ONLY (-1)

/* Open a context on HIP device `device`. max_pkts / max_bytes size the pinned
 * host staging and device buffers used by rxg_classify (host-buffer path);
 * rxg_classify_dev needs neither. */
int rxg_open(rxg_ctx **ctx, int device, uint32_t max_pkts, uint64_t max_bytes);
void rxg_close(rxg_ctx *ctx);
const char *rxg_strerror(int err);
const char *rxg_last_hip_error(void);

/* Mirror of the reference's control-block lists, given in CREATION order
 * (oldest first = the reverse of the head-inserted list, common.h:43-49), so
 * that on duplicate keys the highest index (the newest block) wins exactly as
 * the reference's first-match list scan does.  Builds the device flow tables
 * (linear-probed exact keys under the context's random hash seed, direct
 * port tables for listeners and UDP sockets).  Blocking: waits for this
 * context's own bursts still reading the old tables (never for other work on
 * the device), uploads, and returns with the tables in place. */
int rxg_flows_sync(rxg_ctx *ctx, const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t,
                   uint32_t nt);

/* Incremental control-block changes, between bursts.  The reference creates
 * a tcb on every SYN (tcp_stream_create + LL_ADD, tcp.c:3-52), creates and
 * binds sockets (nsocket / nbind / nlisten, common.c:262-386) and frees
 * blocks on the last ACK and on close (tcp.c:321, common.c:620,660); these
 * calls mirror exactly that on the context's tables in O(1) host work each,
 * instead of a rebuild through rxg_flows_sync.
 *
 * Flow ids are stable: rxg_flows_sync gives block i of its arrays id i; an
 * added block gets a free id (freed ids are reused, else the id space grows)
 * and keeps it until removed.  Verdicts name blocks by these ids, and the
 * per-flow counts are laid out as UDP ids [0, rxg_num_udp_ids()) followed by
 * TCP ids (count index rxg_num_udp_ids() + id); rxg_num_flows() = the length.
 * An added block is the NEWEST (it wins duplicate keys, as LL_ADD's head
 * insert makes it); an update keeps the block's creation order (nbind and
 * nlisten do not move a block in the list) and changes its key and/or
 * status; removing the newest of a duplicate key exposes the next older one.
 *
 * Changes are host-side until committed: rxg_flows_commit(stream), or
 * implicitly by the next burst call, on that burst's stream.  A commit writes
 * only the changed table slots (a small kernel on `stream`), ordered after
 * every earlier burst of this context on any stream and before every later
 * one: it never synchronises the device or the host (a table past load 1/2,
 * or a probe sequence past the cap, is rebuilt whole: that commit waits for
 * its host-to-device copies).
 *
 * rxg_flows_add returns 1 (not an error) when it grew the UDP id space, i.e.
 * moved the TCP count indices: callers keeping their own d_counts vectors
 * re-size them to rxg_num_flows(); the context's own counts move by themselves. */
int rxg_flows_add(rxg_ctx *ctx, const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t, uint32_t nt,
                  uint32_t *udp_ids, uint32_t *tcp_ids);
int rxg_flows_remove(rxg_ctx *ctx, const uint32_t *udp_ids, uint32_t nu, const uint32_t *tcp_ids,
                     uint32_t nt);
int rxg_flows_update_udp(rxg_ctx *ctx, uint32_t id, const rxg_udp_sock *u);
int rxg_flows_update_tcb(rxg_ctx *ctx, uint32_t id, const rxg_tcb *t);
int rxg_flows_commit(rxg_ctx *ctx, void *stream);
/* UDP part of the count layout (see above) */
uint32_t rxg_num_udp_ids(const rxg_ctx *ctx);
/* whole-table rebuilds so far (growth, reseeds): diagnostics */
uint32_t rxg_flows_rebuilds(const rxg_ctx *ctx);

/* Device-resident burst: all pointers are device pointers.  Frame i starts at
 * d_pkts + (d_off[i] << off_unit_log2) (off_unit_log2 >= 4: 16-byte aligned
 * starts) and has d_len[i] captured bytes; the buffer must extend to the next
 * 16-byte boundary after every frame.  len_hint = typical frame length (picks
 * lanes per frame; 0 = 1518).  If d_counts != NULL, per-flow packet counts are
 * added into it (u64[nu + nt]: UDP flows first, then TCP).  Asynchronous on
 * `stream` (a hipStream_t; NULL = the null stream). */
int rxg_classify_dev(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                     const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                     uint32_t len_hint, rxg_verdict *d_out, uint64_t *d_counts,
                     void *stream);

/* rxg_classify_dev with the per-flow counts on a second stream: the verdicts
 * are written on `stream` as above; d_counts is complete once `count_stream`
 * (ordered after this burst's classify) has reached this point, not `stream`.
 * Above 8192 flows the counts are two passes after the classify kernel
 * (DESIGN.md §4); on count_stream they overlap the NEXT burst's classify on
 * `stream` (the context double-buffers its count indices), which is how a
 * burst loop hides them.  The caller orders readers of d_counts (a copy, the
 * RCCL all-reduce) after count_stream.  count_stream NULL or == stream: same
 * as rxg_classify_dev.  Replaces no reference call: the reference keeps no
 * per-flow counters; this is the statistic the multi-GPU path all-reduces. */
int rxg_classify_dev_cs(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        uint32_t len_hint, rxg_verdict *d_out, uint64_t *d_counts,
                        void *stream, void *count_stream);

/* rxg_classify_dev_cs writing compact 8-byte verdicts (d_out: n x 8 bytes,
 * 8-byte aligned); kernels, counts and streams exactly as there. */
int rxg_classify_dev8(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                      const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                      uint32_t len_hint, rxg_verdict8 *d_out, uint64_t *d_counts, void *stream,
                      void *count_stream);

/* Host-buffer burst (PCIe-inclusive): copies frames + descriptors to the
 * device, classifies, copies verdicts back, accumulates the context's own
 * per-flow counts.  Synchronous. */
int rxg_classify(rxg_ctx *ctx, const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                 uint32_t n, uint32_t off_unit_log2, rxg_verdict *out);

/* Same, with the caller stating how many bytes of `pkts` the burst spans
 * (every frame end <= span_bytes); skips the O(n) scan rxg_classify makes. */
int rxg_classify_span(rxg_ctx *ctx, const uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
                      const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out);

/* The reference's calling convention: a burst of mbuf pointers as dequeued at
 * netfamily.c:147.  Frames are gathered into the context's staging buffer. */
int rxg_process_mbufs(rxg_ctx *ctx, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out);

/* Register host memory that holds frames — the mbuf pool's memory, as DPDK
 * hands it out (rte_mempool_mem_iter) — with the context: it is pinned and
 * mapped for the device once, and from then on an mbuf burst
 * (rxg_process_mbufs*) whose frames all lie in registered memory, 16-B
 * aligned with their 16-B rounded ends inside it, is pulled by the device
 * straight from that memory over PCIe (the DMA a NIC does into its ring)
 * instead of being gathered into pinned staging by a host memcpy and copied.
 * Other bursts take the host gather as before.  Memory registered elsewhere
 * already is accepted (and left registered at close).  Unregister waits for
 * this context's bursts. */
int rxg_register_host(rxg_ctx *ctx, void *base, uint64_t bytes);
int rxg_unregister_host(rxg_ctx *ctx, void *base);

/* Pipelined host-buffer bursts (PCIe-inclusive, overlapped).  The context owns
 * RXG_PIPE_DEPTH staging slots (each sized by rxg_open's max_pkts/max_bytes);
 * burst t copies in while burst t-1 is classified and burst t-2's verdicts
 * copy out.  rxg_submit returns at once with a ticket; the caller keeps pkts,
 * off, len and out untouched until rxg_wait(ticket) returns (pass pinned host
 * memory, e.g. hipHostMalloc'd or hipHostRegister'ed, or the copies are not
 * asynchronous).  Tickets complete in submission order.  rxg_classify_span is
 * rxg_submit + rxg_wait. */
#define RXG_PIPE_DEPTH 3
int rxg_submit(rxg_ctx *ctx, const uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
               const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out,
               uint64_t *ticket);
int rxg_wait(rxg_ctx *ctx, uint64_t ticket);

/* ---- UDP delivery on the GPU: per-socket payload compaction ------------
 * The delivery half of udp_process (udp.c:25-52): for every datagram that
 * found its socket (verdict rc 0) the reference mallocs an offload, copies
 * dgram_len - 8 payload bytes from udp + 1 and enqueues it on that socket's
 * ring, frame by frame.  Here one device pass groups a classified burst's
 * delivered datagrams by socket — inside a socket in burst order, the order
 * its ring would have — and gathers their captured payload bytes into one
 * buffer, socket after socket, so the host hands each socket one contiguous
 * slice.  UDP id spaces up to RXG_COMPACT_MAX_FLOWS (the reference's socket
 * layer has at most 1024 descriptors, common.h:34). */
#define RXG_COMPACT_MAX_FLOWS 1024u
typedef struct rxg_dgram {
    uint32_t frame;  /* burst index of the datagram's frame */
    uint32_t offset; /* its payload's first byte in the compacted buffer (16-B aligned) */
    uint32_t sip;    /* raw source address (offload.sip, udp.c:31) */
    uint16_t sport;  /* raw source port (offload.sport) */
    uint16_t len;    /* payload bytes, dgram_len - 8 (udp.c:38); only the captured ones,
                        min(len, caplen - 42), are in the buffer: the rest read as 0 */
} rxg_dgram;
/* Device form, asynchronous on `stream`: d_v = the burst's verdicts; the
 * datagrams of UDP id f get ranks [d_first[f], d_first[f+1]) of d_dgram (so
 * d_first has rxg_num_udp_ids() + 1 entries, d_dgram room for n); d_totals =
 * {datagrams, payload bytes used, 1 if payload_cap was too small (those
 * payloads are not written)}.  RXG_ERANGE above RXG_COMPACT_MAX_FLOWS ids. */
int rxg_udp_compact_dev(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        const rxg_verdict *d_v, rxg_dgram *d_dgram, uint32_t *d_first,
                        uint8_t *d_payload, uint64_t payload_cap, uint32_t *d_totals, void *stream);
/* rxg_process_mbufs followed by the compaction: verdicts into `out` as there;
 * the datagram records, the per-id first ranks and the compacted payload stay
 * in pinned buffers the context owns, valid until its next burst call
 * (*dgram: *ndgram records; *first: rxg_num_udp_ids() + 1 entries; *payload:
 * *nbytes bytes).  Synchronous. */
int rxg_process_mbufs_udp(rxg_ctx *ctx, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out,
                          const rxg_dgram **dgram, const uint32_t **first, const uint8_t **payload,
                          uint32_t *ndgram, uint64_t *nbytes);

/* ---- TCP delivery on the GPU: per-connection segment sort + payload gather
 * The delivery half of tcp_process for segments that found a tcb (verdict
 * rc 0): the reference walks them frame by frame through the state machine
 * (tcp.c:373-415); an ESTABLISHED one with PSH gets a malloc'd fragment with
 * a copy of its payload (ng_tcp_enqueue_recvbuffer, tcp.c:133-185) and an ACK
 * (tcp.c:218-297).  Here one device pass sorts a classified burst's rc-0 TCP
 * segments by tcb id — stable, so a connection's segments keep burst order,
 * the order its state machine must see them in — decodes the header fields
 * the state machine reads, and gathers the payload of every PSH segment into
 * one buffer, connection after connection (each at a 16-B aligned offset), so
 * the host runs each connection's segments in order with one allocation and
 * one copy per connection per burst.  Any tcb id space. */
typedef struct rxg_segment {
    uint32_t frame;  /* burst index of the segment's frame */
    uint32_t flow;   /* tcb id (the verdict's flow_id) */
    uint32_t seq;    /* sent_seq, host order (ntohl of frame bytes 38-41) */
    uint32_t ack;    /* recv_ack, host order (ntohl of frame bytes 42-45) */
    int32_t plen;    /* total_length - 20 - 4*hl (signed: tcp.c:145-146, 391) */
    uint32_t offset; /* first payload byte in the payload buffer (16-B aligned); records
                        only (no payload buffer, RXG_DLV_TCP_IN_PLACE): the payload's
                        offset in its frame, 34 + 4*hl */
    uint16_t sport;  /* raw (network order) source port, frame bytes 34-35 */
    uint16_t dport;  /* raw destination port, frame bytes 36-37 */
    uint16_t ncopy;  /* payload bytes in the buffer: min(plen, caplen - 34 - 4*hl) for a
                        PSH segment with plen > 0, else 0; the rest of a fragment's plen
                        bytes read as 0 */
    uint8_t flags;   /* tcp_flags, frame byte 47 */
    uint8_t hl;      /* data_off >> 4, frame byte 46 */
} rxg_segment;       /* 32 bytes; bytes past the captured length read as 0 */
/* Device form, asynchronous on `stream`: d_v = the burst's verdicts; d_seg
 * (room for n) gets the rc-0 TCP segments with a tcb id below the id space,
 * sorted by (flow, frame); d_totals = {segments, payload bytes used, 1 if
 * payload_cap was too small (those payloads are not written)}.  d_payload
 * NULL: the records only (offset = the payload's offset in its frame, no
 * payload gathered).  The device
 * workspace grows on demand (stream-ordered). */
int rxg_tcp_compact_dev(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        const rxg_verdict *d_v, rxg_segment *d_seg, uint8_t *d_payload,
                        uint64_t payload_cap, uint32_t *d_totals, void *stream);

/* One mbuf burst through the whole device half of delivery: classify
 * (rxg_process_mbufs), then the UDP compaction (when the UDP id space is at
 * most RXG_COMPACT_MAX_FLOWS; else dgram/first are NULL and ndgram 0) and
 * the TCP segment sort and gather, all in one pass over the staged burst.
 * Verdicts into `out`; the other results stay in pinned buffers the context
 * owns (one set per burst in flight, RXG_DELIVER_DEPTH sets used in turn),
 * valid until the set is reused: RXG_DELIVER_DEPTH delivery calls later.  `ms` (nullable, 8 floats): the
 * phases of this burst in ms — [0] host gather of the mbufs into pinned
 * staging; from HIP events on the device: [1] copy in, [2] classify (K1),
 * [3] the compactions (K3 + K4), [4] copy out of their results; [5] the
 * whole call (host clock); [6], [7] 0.  Synchronous. */
typedef struct rxg_delivery {
    const rxg_dgram *dgram;     /* UDP: as rxg_process_mbufs_udp */
    const uint32_t *first;
    const uint8_t *udp_payload;
    uint32_t ndgram;
    uint32_t nseg;              /* TCP: segments, sorted by (tcb id, frame) */
    uint64_t udp_bytes;
    const rxg_segment *seg;
    const uint8_t *tcp_payload;
    uint64_t tcp_bytes;
    int32_t tcp_payload_ref;    /* >= 0: tcp_payload is pooled buffer `ref`, which the caller
                                   may keep longer with rxg_payload_hold (and must then
                                   rxg_payload_release); -1: valid while the set is (above) */
    uint32_t set;               /* the context's delivery set holding this burst, 1-based
                                   (written by rxg_deliver_submit, read by rxg_deliver_wait) */
} rxg_delivery;
int rxg_process_mbufs_deliver(rxg_ctx *ctx, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out,
                              rxg_delivery *d, float ms[8]);
/* rxg_process_mbufs_deliver in two halves, so the caller can let other work
 * run while the burst is on the GPU: rxg_deliver_submit stages the burst and
 * queues every device step and copy (d gets its buffer pointers), and
 * rxg_deliver_wait(ctx, d, ms) waits for them and fills in d's counts and
 * the phase times.  Up to RXG_DELIVER_DEPTH delivery bursts in flight per
 * context, waited for in any order (a submit while the next set in turn is
 * still in flight is RXG_EINVAL): burst k+1's frames cross PCIe while burst
 * k's results come back and the host delivers burst k-1.  The verdicts of a
 * burst submitted before an earlier one was delivered were classified against
 * the flow tables of that submit.  Between the calls the context's control plane
 * (rxg_flows_add / remove / update / commit-free changes) may run from another
 * thread: rxg_deliver_wait reads none of the flow-table state; any other call
 * on the context waits for rxg_deliver_wait first. */
int rxg_deliver_submit(rxg_ctx *ctx, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out,
                       rxg_delivery *d);
int rxg_deliver_wait(rxg_ctx *ctx, rxg_delivery *d, float ms[8]);

/* Delivery options (0 = the default).  RXG_DLV_TCP_IN_PLACE: the TCP payloads
 * stay where they are, in the caller's frames — the DPDK zero-copy receive,
 * where the socket's fragment points into the mbuf and holds it
 * (rte_mbuf_refcnt_update) until the application has read it, instead of the
 * rte_malloc + rte_memcpy of ng_tcp_enqueue_recvbuffer (tcp.c:133-185).  The
 * device sorts the segments and decodes their records as before but gathers
 * no payload, and only the 32-B records cross PCIe back:
 * rxg_delivery.tcp_payload is NULL and each record's offset is its payload's
 * offset in its frame (34 + 4*hl; ncopy captured bytes).  The caller keeps
 * the frames in place for as long as it points into them. */
#define RXG_DLV_TCP_IN_PLACE 0x1u
int rxg_tune_deliver(rxg_ctx *ctx, uint32_t flags);

/* Keep a burst's TCP payload buffer (rxg_delivery.tcp_payload_ref) alive past
 * the context's next burst call — e.g. while receive fragments that point into
 * it wait in a socket's ring — and let it go again.  Holds are counted; a
 * buffer is reused once none is left.  RXG_PAYLOAD_BUFS buffers of max_bytes
 * are pinned at most; with all of them held, the payloads of a burst come in
 * the context's own buffer (tcp_payload_ref -1) and must be copied.  Both
 * calls are safe from any thread (atomic counts). */
#define RXG_PAYLOAD_BUFS 6
#define RXG_DELIVER_DEPTH 2
int rxg_payload_hold(rxg_ctx *ctx, int32_t ref);
int rxg_payload_release(rxg_ctx *ctx, int32_t ref);

/* TX checksum generation (the send side's per-frame work, udp.c:84-95 and
 * tcp.c:444-463): for every IPv4 frame of the burst, the IPv4 header checksum
 * (rte_ipv4_cksum, rte_ip.h:255-265) is written at frame offset 24, and for
 * IPv4 UDP/TCP frames the L4 checksum (rte_ipv4_udptcp_cksum, :325-349; UDP
 * 0 -> 0xFFFF) at offset 40 / 50, each computed with its own field taken as 0
 * and the reference's rx conventions (L4 at ip+20, length tl-20, bytes past
 * the captured length read as 0).  Frames are modified in place; fields not
 * wholly inside the captured length and non-IPv4 frames are left as they are.
 * Device form: asynchronous on `stream`.  Host form: pkts (span_bytes, pinned
 * for speed) is copied to the device, checksummed and copied back; synchronous. */
int rxg_tx_cksum_dev(rxg_ctx *ctx, uint8_t *d_pkts, const uint32_t *d_off, const uint16_t *d_len,
                     uint32_t n, uint32_t off_unit_log2, uint32_t len_hint, void *stream);
int rxg_tx_cksum(rxg_ctx *ctx, uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
                 const uint16_t *len, uint32_t n, uint32_t off_unit_log2);

/* Tuning hook: force the kernel variant (lanes per frame 1 or 4..64, passes
 * loaded up front, frames per lane group, pipeline mode; 0xFFFFFFFF = the
 * default pipeline); lanes_per_frame = 0 with pipeline 0xFFFFFFFF =
 * automatic from len_hint; lanes_per_frame = 0 with any other pipeline =
 * that frame-size-independent variant (20: size-class binned path; 30 and
 * up: stream and SH kernel variants; csrc/rx_classify.hip k_variants).  A
 * combination that is not compiled in returns RXG_EINVAL.  Every variant of
 * the product library gives the same verdicts; diagnostic ablations (wrong
 * verdicts by construction) exist only in the RX_DIAG tuning build
 * (librxgpu_diag.so), never in librxgpu.so. */
int rxg_tune(rxg_ctx *ctx, uint32_t lanes_per_frame, uint32_t passes, uint32_t frames_per_group,
             uint32_t pipeline);

/* The classify variant a burst with this len_hint runs on this context (the
 * rxg_tune override, else the default for len_hint): variant = {lanes per
 * frame, passes, frames per group, pipeline}; name (nullable, name_cap bytes
 * with the NUL) = the kernel it dispatches as a kernel trace names it
 * (rocprofv3), without template arguments.  Diagnostics: it lets a benchmark
 * line name the dispatch a profiler shows. */
int rxg_kernel_variant(const rxg_ctx *ctx, uint32_t len_hint, uint32_t variant[4], char *name,
                       uint32_t name_cap);

/* Tuning hook: cap the resident 256-thread blocks per CU the launch uses
 * (0 = as many as the occupancy allows). */
int rxg_tune_grid(rxg_ctx *ctx, uint32_t blocks_per_cu);

/* Tuning hook for the TX checksum kernel: force entry `variant` of its
 * variant table (csrc/tx_cksum.hip k_tx; RXG_TX_AUTO = chosen from len_hint)
 * and cap its resident blocks per CU (0 = the variant's default). */
#define RXG_TX_AUTO 0xFFFFFFFFu
int rxg_tune_tx(rxg_ctx *ctx, uint32_t variant, uint32_t blocks_per_cu);

/* Tuning hook for the exact-key flow tables: load factor <= 2^-load_log2
 * (1 = 1/2, 2 = 1/4, up to 4; 0 = the default), applied by the next
 * rxg_flows_sync.  Verdicts do not depend on it; the table's cache footprint
 * and probe length do. */
int rxg_tune_flow_load(rxg_ctx *ctx, uint32_t load_log2);

/* Tuning hook: flow-table layout flags (0 = the default layout).
 * RXG_TT_NO_UDP_PORT (applied by the next rxg_flows_sync): no direct UDP port
 * table; every UDP lookup probes the hashed table.  RXG_TT_COUNT_4B (applied
 * at once): the 8193..2M-flow count path keeps 4-B count indices even at
 * <= 65536 flows.  RXG_TT_COUNT_2BUF (applied at once): see below.  Verdicts
 * and counts depend on none of them. */
#define RXG_TT_NO_UDP_PORT 0x1u
#define RXG_TT_COUNT_4B 0x2u
#define RXG_TT_COUNT_2BUF 0x4u /* rxg_classify_dev_cs: two count-index buffers instead of
                                  three (each burst then waits for the count of the
                                  burst before the previous one) */
#define RXG_TT_SLAB_HALF 0x8u     /* the count's slab pass on half / a quarter of the CUs */
#define RXG_TT_SLAB_QUARTER 0x10u /* (fewer, larger slabs; applied at once) */

int rxg_tune_tables(rxg_ctx *ctx, uint32_t flags);

/* Tuning hook: how mbuf bursts whose frames lie in registered memory
 * (rxg_register_host) reach the GPU.  RXG_INGEST_AUTO (the default): a burst
 * dense in one region (its covering span at most 1.4x its frames' bytes and
 * within the staging slot) is copied as that one span by the copy engine,
 * any other registered burst is pulled by the device frame by frame;
 * RXG_INGEST_PULL: always pulled; RXG_INGEST_GATHER: always gathered on the
 * host.  Outputs do not depend on it.  In both registered forms the frames
 * are read after the call returns: they must stay in place until the burst
 * is waited for (rxg_deliver_wait; the synchronous calls return after it). */
#define RXG_INGEST_AUTO 0u
#define RXG_INGEST_PULL 1u
#define RXG_INGEST_GATHER 2u
int rxg_tune_ingest(rxg_ctx *ctx, uint32_t mode);

/* Context-owned per-flow counts (accumulated by rxg_classify / rxg_process_mbufs). */
int rxg_flow_counts(rxg_ctx *ctx, uint64_t *counts, uint32_t ncounts);
int rxg_counts_reset(rxg_ctx *ctx);
uint32_t rxg_num_flows(const rxg_ctx *ctx);

/* Diagnostics: flow table `which` (0 UDP slots, 1 TCP slots, 2 listeners,
 * 3 the lane kernel's compact UDP table (8-B slots {dip, dport | flow << 16}),
 * 4 its UDP port window (u16 flow ids, 0xFFFF none)) as the device holds it
 * (device_copy != 0; after this context's bursts drain) or as the host image
 * is, up to `bytes`; info (nullable) = {device tcp_mask, tcp_probe, hseed,
 * host tcp mask, probe, seed, changes pending, slots} for 0-2, and for 3-4
 * {slots - 1 of the compact table, its longest probe, hseed, compact keys off
 * the window's address, window's first port (host order), window length,
 * window's address (raw), entries of `which`}. */
int rxg_ft_dump(rxg_ctx *ctx, uint32_t which, int device_copy, void *dst, uint64_t bytes,
                uint32_t info[8]);

/* Host-side lookups through the built flow table (same code path as the
 * device probe, for control-plane use and tests). */
uint32_t rxg_ft_lookup_udp(const rxg_ctx *ctx, uint32_t dip, uint16_t dport);
uint32_t rxg_ft_lookup_tcp(const rxg_ctx *ctx, uint32_t sip, uint32_t dip, uint16_t sport,
                           uint16_t dport);

/* RSS: Toeplitz hash (standard 40-byte key) over sip,dip,sport,dport in
 * network byte order, as a multi-queue NIC computes it; shard = hash % n. */
uint32_t rxg_rss_hash(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport);

/* ---- multi-GPU: RSS split, shard gather, per-flow count all-reduce ------
 * The reference runs one rx queue (ng_init_port, netfamily.c:38-39) and one
 * pkt_process lcore (netfamily.c:427) over the burst it dequeues at
 * netfamily.c:147.  Across G GPUs of a node the burst is split by RSS, as the
 * multi-queue NIC the README assumes (README.md:13) would: each GPU holds a
 * replica of the flow tables (rxg_flows_sync with the same lists) and
 * classifies its shard; the per-flow counts are the only exchange. */
#define RXG_MAX_SHARDS 64

/* Shard of a frame = rxg_rss_hash(sip, dip, sport, dport) % n_shards for IPv4
 * TCP/UDP, rxg_rss_hash(sip, dip, 0, 0) % n_shards for other IPv4, 0 for
 * non-IPv4 frames (bytes past the captured length read as 0).  perm[] gets
 * the frame indices grouped by shard, in burst order inside a shard;
 * first[s] = start of shard s in perm, first[n_shards] = n (n_shards + 1
 * entries).  Host form: host buffers, synchronous.  Device form: device
 * buffers, asynchronous on `stream` (workspace grown on demand, between
 * bursts). */
int rxg_rss_split(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                  uint32_t off_unit_log2, uint32_t n_shards, uint32_t *first, uint32_t *perm);
int rxg_rss_split_dev(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                      const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t n_shards,
                      uint32_t *d_first, uint32_t *d_perm, void *stream);

/* Gather frames d_idx[0..count) of a device burst into a packed device burst
 * (the DMA of one RSS queue's frames into its ring): frame k at
 * d_dst + (d_dst_off[k] << 6), 64-B aligned, zero-filled to its 64-B end,
 * d_dst_len[k] = its captured length (so the result is classified with
 * off_unit_log2 = 6).  *span = bytes the packed burst occupies.  Synchronises
 * `stream` (setup-time operation); RXG_ERANGE if the packed burst exceeds
 * dst_cap (frames past dst_cap are not copied). */
int rxg_gather_dev(rxg_ctx *ctx, const uint8_t *d_pkts, const uint32_t *d_off,
                   const uint16_t *d_len, uint32_t off_unit_log2, const uint32_t *d_idx,
                   uint32_t count, uint8_t *d_dst, uint64_t dst_cap, uint32_t *d_dst_off,
                   uint16_t *d_dst_len, uint64_t *span, void *stream);

/* A communicator over the GPUs of the node (RCCL over xGMI), one rank per
 * GPU/process.  Rank 0 makes the id with rxg_group_id and the caller hands it
 * to every rank by its own means (a file, a socket, MPI, torch.distributed);
 * every rank then calls rxg_group_open with it (collective: returns once all
 * nranks have joined). */
#define RXG_GROUP_ID_BYTES 128
typedef struct rxg_group rxg_group;
int rxg_group_id(uint8_t id[RXG_GROUP_ID_BYTES]);
int rxg_group_open(rxg_group **g, int device, uint32_t nranks, uint32_t rank,
                   const uint8_t id[RXG_GROUP_ID_BYTES]);
void rxg_group_close(rxg_group *g);
/* The communicator's size and this process's rank as RCCL reports them
 * (ncclCommCount / ncclCommUserRank); either pointer may be NULL. */
int rxg_group_size(const rxg_group *g, uint32_t *nranks, uint32_t *rank);
/* Sum of a device u64 count vector over the ranks, in place, asynchronous on
 * `stream` (every rank must call it with the same n). */
int rxg_counts_allreduce(rxg_group *g, uint64_t *d_counts, uint32_t n, void *stream);
/* The same for the context-owned counts (rxg_classify / rxg_process_mbufs),
 * after every burst submitted so far; synchronous.  Only the increment since
 * the previous call is reduced and then added to the running total, so the
 * context's counts (rxg_flow_counts) are the global totals after each call,
 * however often it is called. */
int rxg_ctx_counts_allreduce(rxg_ctx *ctx, rxg_group *g);

/* ---- pcap ingest (the NIC stand-in: rte_eth_rx_burst into the in-ring,
 * netfamily.c:438-440) -------------------------------------------------- */
/* Classic libpcap files, LINKTYPE_ETHERNET, either byte order, us or ns
 * stamps.  A file is mapped once and read burst by burst in capture order. */
typedef struct rxg_pcap rxg_pcap;
int rxg_pcap_open(rxg_pcap **p, const char *path);
void rxg_pcap_close(rxg_pcap *p);
int rxg_pcap_rewind(rxg_pcap *p);
/* Pack up to max_frames next frames into pkts (cap_bytes) in the burst layout:
 * frame k at off[k] << off_unit_log2, captured length len[k], zero fill to the
 * next 16-B boundary.  *n = frames packed (0 at end of file), *span = bytes
 * used.  A record longer than 65535 bytes is RXG_ERANGE; a truncated file is
 * RXG_EINVAL. */
int rxg_pcap_read_burst(rxg_pcap *p, uint8_t *pkts, uint64_t cap_bytes, uint32_t *off,
                        uint16_t *len, uint32_t max_frames, uint32_t off_unit_log2, uint32_t *n,
                        uint64_t *span);
/* Write n frames of a burst as a pcap file (capture order = burst order). */
int rxg_pcap_write(const char *path, const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                   uint32_t n, uint32_t off_unit_log2);

/* ---- synthetic traffic (pktgen) --------------------------------------- */
/* Deterministic counter-based generator: frame i is a pure function of
 * (cfg, i), identical on host and device.  Frames are written at
 * off[i] = i * (slot_bytes >> off_unit_log2), or packed (cfg.packed). */
typedef struct rxg_gen_cfg {
    uint64_t seed;
    uint32_t size_mode;     /* 0 fixed frame_len, 1 IMIX 64/576/1500 at 7:4:1 */
    uint32_t frame_len;     /* fixed-size frames (>= 64 for TCP/UDP) */
    uint32_t slot_bytes;    /* bytes reserved per frame (multiple of 16, >= max frame) */
    uint32_t proto_mode;    /* 0 UDP only, 1 TCP only, 2 TCP/UDP 50/50 */
    uint32_t n_udp;         /* UDP sockets: local_ip:(udp_base_port + k) */
    uint32_t n_tcp;         /* established tcbs: (10.128.x.y : 1024+..) -> local_ip:tcp_port */
    uint32_t local_ip;      /* network order (192.168.100.77 = netfamily.c:11) */
    uint16_t udp_base_port; /* host order */
    uint16_t tcp_port;      /* host order (9999 = netfamily.c:270) */
    uint32_t bad_cksum_per10k; /* one flipped payload bit after the checksum */
    uint32_t unknown_per10k;   /* destination port with no socket / listener */
    uint32_t other_per10k;     /* ICMP or ARP frames */
    uint32_t shard;         /* keep only tuples whose rxg_rss_hash % n_shards == shard */
    uint32_t n_shards;      /* 1 = no sharding */
    uint32_t packed;        /* 0: frame i in slot i (slot_bytes apart); 1: frames packed
                               back to back at 64-B alignment (what rxg_process_mbufs
                               staging produces); slot_bytes then bounds one frame */
    uint32_t src_ip;        /* network order; != 0: every UDP frame to a bound socket
                               comes from src_ip:src_port (one 5-tuple, e.g. the echo
                               client of BASELINE configs[0]); 0: random sources */
    uint16_t src_port;      /* host order */
    uint16_t _pad;
} rxg_gen_cfg;

/* Flow set the generator assumes (the sockets/tcbs a test or bench binds). */
int rxg_gen_flows(const rxg_gen_cfg *cfg, rxg_udp_sock *u, rxg_tcb *t);
/* Host generation of frames [first, first+n) into caller buffers (slot i-first;
 * the buffer must hold n * slot_bytes bytes in either layout). */
int rxg_gen_host(const rxg_gen_cfg *cfg, uint64_t first, uint32_t n, uint8_t *pkts,
                 uint32_t *off, uint16_t *len, uint32_t off_unit_log2);
/* Device generation (same frames), asynchronous on stream. */
int rxg_gen_dev(const rxg_gen_cfg *cfg, uint64_t first, uint32_t n, uint8_t *d_pkts,
                uint32_t *d_off, uint16_t *d_len, uint32_t off_unit_log2, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RXGPU_H */
