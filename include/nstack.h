/*
 * nstack.h — socket-style API of the stack, host C, over librxgpu.
 *
 * Same names, signatures and return conventions as the reference's socket
 * layer (common.h:189-200, bodies common.c:262-666), so an application
 * written against the reference (netfamily.c:211-383) links unchanged.  The
 * control blocks are the reference's (struct localhost udp.h:10-29, struct
 * tcp_stream tcp.h:29-55) in the same head-inserted lists; what changes is
 * the receive path: instead of per-frame udp_process/tcp_process calls on the
 * protocol lcore, a burst goes through nstack_rx_burst(), which classifies it
 * on the GPU (rxg_process_mbufs) and then delivers UDP payloads into the
 * sockets' receive rings with the reference's `struct offload` semantics
 * (udp.c:25-52), where nrecvfrom() picks them up.
 *
 * Deliberate differences (DESIGN.md §Socket layer):
 *   - the lists are guarded by a lock (the reference mutates them from the
 *     app lcore while the protocol lcore walks them, common.c:302,336,620,660);
 *   - control blocks are reference-counted: a call blocked in nrecv /
 *     nrecvfrom / naccept on a block that another thread closes (or whose
 *     last ACK frees it) wakes and returns -1 (errno EBADF) instead of
 *     waiting on freed memory;
 *   - get_hostinfo_fromfd walks the list correctly (common.c:116 advances
 *     from the list head and never terminates past the second socket);
 *   - nrecvfrom/nrecv/naccept honour MSG_DONTWAIT in `flags` (the reference
 *     ignores flags and always blocks); naccept has no flags: it blocks;
 *   - the 8 bytes nrecvfrom returns past the payload (offload.length =
 *     dgram_len, udp.c:37, but only dgram_len-8 bytes are stored, udp.c:38) read
 *     as zeros instead of adjacent heap memory.
 * TCP segments that pass classify drive the reference's state machine
 * (tcp.c:43-331, dispatch :373-415) on the host, frame by frame in burst
 * order: LISTEN+SYN creates a tcb and queues SYN|ACK, SYN_RCVD+ACK
 * establishes and wakes naccept, ESTABLISHED+PSH queues the payload for
 * nrecv and an ACK, +FIN queues the EOF marker and moves to CLOSE_WAIT,
 * LAST_ACK+ACK frees the tcb.  A burst is classified against one snapshot of
 * the tcb list; once the burst's own segments change that list (SYN, final
 * ACK), later segments of the burst are looked up again on the live list
 * (through the host image of the flow tables, O(1) per lookup), so the
 * outcome is the reference's sequential one (a SYN and its ACK may share a
 * burst).  Segments of a tcb in ESTABLISHED (or a state whose segments are
 * no-ops) depend on no other frame of the burst: the GPU sorts them per
 * connection and gathers their payloads (rxg_process_mbufs_deliver), and
 * they run connection by connection, each connection's fragments and ACKs
 * queued as one batch (one allocation); every other frame keeps the
 * frame-by-frame path.  Unresolved merge-conflict hunks of tcp.c take the
 * HEAD side.
 */
#ifndef NSTACK_H
#define NSTACK_H

#include <stdint.h>
#include <sys/socket.h>
#include <sys/types.h>

#include "rxgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Process-wide stack, like the reference's globals (netfamily.c:16-18).
 * device = HIP ordinal, or RXG_HOST_ONLY for a stack without a GPU (socket
 * API + nstack_deliver work; nstack_rx_burst returns RXG_ENODEV). */
int nstack_init(int device, uint32_t max_burst, uint64_t max_bytes);
void nstack_fini(void);

/* socket API (common.h:189-200) */
int nsocket(int domain, int type, int protocol);
int nbind(int sockfd, const struct sockaddr *addr, socklen_t addrlen);
int nlisten(int sockfd, int backlog);
int naccept(int sockfd, struct sockaddr *addr, socklen_t *addrlen);
ssize_t nsend(int sockfd, const void *buf, size_t len, int flags);
ssize_t nrecv(int sockfd, void *buf, size_t len, int flags);
ssize_t nrecvfrom(int sockfd, void *buf, size_t len, int flags, struct sockaddr *src_addr,
                  socklen_t *addrlen);
ssize_t nsendto(int sockfd, const void *buf, size_t len, int flags, const struct sockaddr *dest_addr,
                socklen_t addrlen);
int nclose(int fd);

/* Receive burst: the loop body of pkt_process (netfamily.c:152-200) for n
 * frames at once (as two halves in flight together, see nstack_set_halves;
 * the outcome is the same).  rc_out[i] (nullable) = what udp_process/tcp_process would
 * have returned (KNI frames: 1); v_out (nullable) = the verdicts.
 * Returns the number of UDP datagrams delivered, or a negative RXG_E* code.
 * A burst run as two halves whose second half could not go through the GPU
 * after the first was delivered returns, when rc_out is given, the first
 * half's count: the second half's rc_out entries hold the (negative RXG_E*)
 * error and its v_out entries are zero, so the caller can pass those frames
 * again.  With rc_out NULL it returns the error code.
 * Called by one protocol thread, which also runs nstack_tx_burst (as
 * pkt_process runs udp_out / tcp_out); while the burst is on the GPU the
 * stack's lock is released, so application threads' socket calls run beside
 * it (a second concurrent nstack_rx_burst gets RXG_EINVAL). */
int nstack_rx_burst(rxg_mbuf *const *m, uint32_t n, int *rc_out, rxg_verdict *v_out);

/* Pipelined receive: the same delivery as nstack_rx_burst, with the next
 * burst on the GPU (copy in, K1/K3/K4, copy out) while the protocol thread
 * delivers the previous one.  nstack_rx_submit queues a burst and returns at
 * once (RXG_DELIVER_DEPTH = 2 bursts submitted and not completed at most;
 * RXG_EINVAL past that, or while an nstack_rx_burst runs); nstack_rx_complete
 * waits for the oldest submitted burst and delivers it, frame order and
 * outcomes as nstack_rx_burst's, and returns its UDP datagrams delivered (or
 * a negative RXG_E* code: the burst was not delivered, RXG_EINVAL when none
 * is pending).  A burst's frames, rc_out and v_out must stay valid until its
 * complete.  A burst classified before the previous one was delivered is
 * delivered frame by frame on the live lists when that delivery or a socket
 * call changed a lookup (the reference's sequential outcome, netfamily.c:
 * 147-200 taking burst k+1 only after burst k).  The loop:
 *     nstack_rx_submit(b0); for (k...) { nstack_rx_submit(b[k+1]); nstack_rx_complete(); }
 * nstack_rx_pending: bursts submitted and not completed.  nstack_rx_burst and
 * nstack_deliver are refused while any is pending; nstack_fini waits for them
 * and drops them. */
int nstack_rx_submit(rxg_mbuf *const *m, uint32_t n, int *rc_out, rxg_verdict *v_out);
int nstack_rx_complete(void);
int nstack_rx_pending(void);

/* Delivery half only: apply verdicts computed by rxg_* to the frames (UDP ->
 * socket receive rings, TCP -> state machine).  Verdict flow ids are the
 * blocks' stable ids (nstack_flow_ids).  `gen` = the generation nstack_flows
 * returned with the lists the verdicts were classified against: if the lists
 * changed since (a block created, rebound, made a listener or freed — a freed
 * id may be reused), every frame of the burst is looked up again on the live
 * lists, as the reference's per-frame lookups would, instead of trusting the
 * flow ids.  rc_out (nullable) as for nstack_rx_burst. */
int nstack_deliver(rxg_mbuf *const *m, uint32_t n, const rxg_verdict *v, uint64_t gen,
                   int *rc_out);

/* Install a tcb as tcp_stream_create + LL_ADD do on a SYN (tcp.c:3-52) and
 * wake a blocked naccept (tcp.c:108-116).  All values raw network order. */
int nstack_tcb_add(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport, int status);

/* The control blocks in creation order (the lists rxg_flows_sync would
 * take) and the generation of the lists (nullable; for nstack_deliver).
 * Counts are always written; arrays up to their capacities.  Every block is
 * registered with the context's GPU flow tables as it is created, bound,
 * made a listener and freed (nsocket / nbind / nlisten / SYN / last ACK /
 * nclose: rxg_flows_add / update / remove, committed with the next burst), so
 * no burst ever waits for a table rebuild. */
int nstack_flows(rxg_udp_sock *u, uint32_t cap_u, uint32_t *nu, rxg_tcb *t, uint32_t cap_t,
                 uint32_t *nt, uint64_t *gen);
/* The stable flow id (verdict flow_id, count index) of each block of the
 * nstack_flows arrays, in the same order. */
int nstack_flow_ids(uint32_t *uid, uint32_t cap_u, uint32_t *tid, uint32_t cap_t);

/* Diagnostics (tests): the flow id the library's flow tables (the host image
 * of what the device probes) give a key — UDP (dst ip, dst port), TCP (the
 * exact 4-tuple, else the listener on dport); RXG_FLOW_NONE if none. */
uint32_t nstack_lookup_udp(uint32_t dip, uint16_t dport);
/* The mbuf pool's memory (rxg_register_host on the stack's context): bursts
 * whose frames lie in it are pulled by the GPU instead of gathered on the
 * host (DPDK: once per memory chunk of the pool, rte_mempool_mem_iter). */
int nstack_register_host(void *base, uint64_t bytes);
/* the library context the socket layer classifies with (diagnostics) */
rxg_ctx *nstack_ctx(void);
uint32_t nstack_lookup_tcp(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport);

/* Diagnostics (tests): the tcb with this exact 4-tuple (raw network order):
 * status, rcv_nxt, snd_nxt, fd; and the k-th fragment queued in its send
 * ring (TCP flags, acknum).  0 = found, -1 = none.  nstack_tcb_count = tcbs
 * in the list (listeners included). */
int nstack_tcb_state(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport, int32_t *status,
                     uint32_t *rcv_nxt, uint32_t *snd_nxt, int32_t *fd);
int nstack_tcb_sndq(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport, uint32_t k,
                    uint8_t *flags, uint32_t *acknum);
uint32_t nstack_tcb_count(void);

/* ---- TX (the udp_out / tcp_out pass of the protocol loop, netfamily.c:205-206)
 * Local identity: gLocalIp (netfamily.c:11) and the port MAC g_stCpuMac
 * (netfamily.c:415).  Frames leave from this MAC (copied into sockets at
 * nbind and into tcbs at creation, as common.c:356,365 / tcp.c:32 do); an
 * ARP frame addressed to this IP teaches the ARP table.  Raw network-order ip. */
int nstack_set_local(uint32_t ip, const uint8_t mac[6]);
/* ng_arp_entry_insert (common.c:177-204): 1 = inserted, 0 = already known */
int nstack_arp_insert(uint32_t ip, const uint8_t mac[6]);
/* One udp_out + tcp_out pass (udp.c:123-164, tcp.c:492-555): at most one
 * queued datagram per UDP socket and one fragment per tcb, in list order,
 * encoded as frames (ng_encode_udp_apppkt udp.c:59-98, ng_encode_tcp_apppkt
 * tcp.c:420-466) into pkts/off/len (the rx burst layout, off in 64-B units).
 * A destination with no ARP entry gets an ARP request (ng_send_arp,
 * common.c:206-260) and its item is queued again, as the reference does.
 * cksum != 0: both checksums are filled on the GPU (rxg_tx_cksum) before the
 * call returns; 0: both fields are left 0.  Items that do not fit stay queued.
 * Returns the number of frames (or a negative RXG_E* code); *span = bytes used. */
int nstack_tx_burst(uint8_t *pkts, uint64_t cap_bytes, uint32_t *off, uint16_t *len,
                    uint32_t max_frames, int cksum, uint64_t *span);

/* The application side of a benchmark, in one call: every UDP socket read
 * with nrecvfrom until empty, every tcb's receive queue read (nrecv) and its
 * queued ACKs taken off its send ring (as one tcp_out pass would).  buf/cap =
 * the receive buffer each call uses.  Returns the datagrams + fragments
 * received (EOF fragments are read and not counted, as oracle_drain_all does;
 * a negative RXG_E* code on error); *bytes = the bytes the calls returned.
 * Never takes the stack's lock: a short lock of the id maps is held to take
 * a reference on the next 8192 blocks; the reads run under each block's own
 * mutex, so a concurrent nstack_rx_burst delivers beside them, and a block
 * freed meanwhile (last ACK) stays valid until the call lets go of it.
 * nrecv / nrecvfrom / nsendto look their descriptor up the same way. */
int64_t nstack_drain_all(void *buf, size_t cap, uint64_t *bytes);
/* nstack_drain_all, and *sum = the sum (mod 2^64) over every datagram and
 * fragment read of the FNV-1a 64 hash of the bytes the read returned: an
 * order-free check of the content the application received (tests). */
int64_t nstack_drain_all_sum(void *buf, size_t cap, uint64_t *bytes, uint64_t *sum);

/* In-place TCP receive (DPDK zero-copy; off by default).  on != 0: a
 * receive fragment whose payload was captured whole is not copied (the
 * rte_malloc + rte_memcpy of ng_tcp_enqueue_recvbuffer, tcp.c:133-185): it
 * points into its frame, and the stack takes a reference on the frame's mbuf
 * (rxg_mbuf.refcnt += 1, atomically, as rte_mbuf_refcnt_update) until the
 * application has read it.  The GPU then sends back only the segment
 * records, no payload (RXG_DLV_TCP_IN_PLACE).  The put that drops an mbuf's
 * count to 0 calls release(m, arg) (nullable; e.g. the mempool's free, as
 * rte_pktmbuf_free).  The caller holds its own reference on each mbuf it
 * passes (refcnt >= 1) and drops it after nstack_rx_burst / nstack_deliver
 * returns (nstack_mbufs_put); an mbuf's frame must stay in place until its
 * count is 0. */
int nstack_set_rx_inplace(int on, void (*release)(rxg_mbuf *m, void *arg), void *arg);
/* Items the application has read (fragments, datagram batches) are handed
 * back to the protocol thread and freed by its next nstack_rx_burst (while
 * that burst is on the GPU) / nstack_tx_burst / nstack_deliver call (or
 * nstack_reclaim, a protocol-thread call): in place, a frame's mbuf count
 * reaches 0 there.  A thread that made
 * one of those calls frees what it reads at once. */
void nstack_reclaim(void);
/* drop one reference on each of n mbufs (rte_pktmbuf_free of a burst):
 * release(m, arg) of nstack_set_rx_inplace for each whose count reaches 0 */
void nstack_mbufs_put(rxg_mbuf *const *m, uint32_t n);

/* Where the last nstack_rx_burst's time went, in ms: [0] gather of the mbufs
 * into pinned staging (host), [1] copy in, [2] classify (K1), [3] UDP
 * compaction + TCP segment sort (K3 + K4), [4] copy out of their results
 * (device, HIP events), [5] the library calls (submit + wait, host clock),
 * then host delivery: [6] UDP batches to the sockets, [7] TCP connections
 * from the segment sort, [8] the frame-by-frame loop over the rest, [9] the
 * whole nstack_rx_burst; [10] segments sorted, [11] datagrams compacted.  A
 * burst run as two halves adds up both halves' phases, so [1]-[4] may exceed
 * the wall time they took.  A protocol-thread call: like nstack_rx_burst it
 * takes the stack's lock ahead of an application loop (nstack_drain_all). */
int nstack_last_burst_phases(float ms[12]);
/* Bursts of at least 2 * min_half frames run as two halves, both on the GPU
 * at once (rxg_deliver_submit twice: the second half's copy in overlaps the
 * first half's copy out, and the host delivers the first half while the
 * second is on the GPU); 0 (the default) = never.  Measured on MI355X: no
 * gain for 16K-32K-frame bursts, hence off. */
int nstack_set_halves(uint32_t min_half);

/* counters: 0 = UDP datagrams delivered, 1 = dropped (a receive ring full),
 * 2 = TCP segments dispatched to the state machine, 3 = frames handed to KNI,
 * 4 = TCP fragments (payload or EOF) queued for nrecv, 5 = bursts (or burst
 * halves) delivered frame by frame because the lists changed while they were
 * on the GPU, 6 = TCP payload bytes copied on the host (the sorted segments'
 * payloads are otherwise queued in place, in a pooled pinned buffer the
 * library holds until the application has read them; copied when no pooled
 * buffer was free, or for a segment cut short by its capture), 7 = fragment
 * batches now queued that hold such a buffer (read without the lock); 8-10 =
 * nstack_drain_all's time in ns (read without the lock): waiting for the
 * id maps' lock (never the stack's), stepping aside for the protocol thread
 * (0 since round 5: nothing to step aside from), reading out what it took
 * from the blocks (outside every lock but the block's own); 11 = bursts
 * that waited for a pooled payload buffer while an application thread was
 * draining (at most 20 ms each; the stack's lock released meanwhile); 12 =
 * bursts delivered (nstack_rx_burst, nstack_deliver), read without any lock: a
 * polling application that reads a value it has not seen finds that burst's
 * items in its next nstack_drain_all (bumped with release order after the
 * deliveries, read with acquire).  Counter 1 also counts TX items dropped (a
 * send ring full, or a datagram too long for a frame). */
uint64_t nstack_stat(int which);

#ifdef __cplusplus
}
#endif
#endif
