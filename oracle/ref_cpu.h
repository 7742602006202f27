/*
 * ref_cpu.h — CPU restatement of the reference receive front end.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker (and the CPU
 * baseline timed by bench.py's cpu_baseline leg).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline may load it; the
 * product path (librxgpu.so) never links, calls or falls back to it.
 *
 * Parity pin status: see ref_cpu.c header.
 */
#ifndef REF_CPU_H
#define REF_CPU_H

#include <stdint.h>

#include "../include/rxgpu.h" /* verdict / control-block layouts only (types, no code) */

#ifdef __cplusplus
extern "C" {
#endif

/* DPDK 19.11.12 rte_ip.h restatements */
uint32_t oracle_raw_cksum_acc(const void *buf, uint32_t len, uint32_t sum); /* __rte_raw_cksum */
uint16_t oracle_raw_cksum(const void *buf, uint32_t len);                  /* rte_raw_cksum */
uint16_t oracle_ipv4_phdr_cksum(const uint8_t *ipv4_hdr);                  /* rte_ipv4_phdr_cksum */
uint16_t oracle_ipv4_udptcp_cksum(const uint8_t *ipv4_hdr, const uint8_t *l4); /* rte_ipv4_udptcp_cksum */
uint16_t oracle_ipv4_cksum(const uint8_t *ipv4_hdr);                       /* rte_ipv4_cksum */

/* control-block lists in the reference's own shape (head-inserted lists) */
typedef struct oracle_tables oracle_tables;
oracle_tables *oracle_tables_new(const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t, uint32_t nt);
void oracle_tables_free(oracle_tables *tb);
/* get_hostinfo_fromip_port / tcp_stream_search: return creation index or RXG_FLOW_NONE */
uint32_t oracle_lookup_udp(const oracle_tables *tb, uint32_t dip, uint16_t port, uint8_t proto);
uint32_t oracle_lookup_tcp(const oracle_tables *tb, uint32_t sip, uint32_t dip, uint16_t sport,
                           uint16_t dport);

/* pkt_process loop body + udp_process/tcp_process fronts, per frame.
 * counts (nullable): u64[nu+nt], += 1 per frame with flow_id != NONE. */
void oracle_classify(const oracle_tables *tb, const uint8_t *pkts, const uint32_t *off,
                     const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out,
                     uint64_t *counts);

/* TX checksum fill in place (udp.c:84-95, tcp.c:444-463), see ref_cpu.c */
void oracle_tx_cksum(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                     uint32_t off_unit_log2);

/* Toeplitz RSS (same definition as rxg_rss_hash, written independently) */
uint32_t oracle_rss_hash(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport);

/* ---- delivery half (ref_stack.c): the socket layer and the per-frame
 * udp_process / tcp_process effects, in the reference's list shapes.
 * Blocking calls return -2 where the reference would wait. */
typedef struct oracle_stack oracle_stack;
oracle_stack *oracle_stack_new(void);
void oracle_stack_free(oracle_stack *st);
int oracle_nsocket(oracle_stack *st, int type); /* 1 SOCK_STREAM, 2 SOCK_DGRAM */
int oracle_nbind(oracle_stack *st, int fd, uint32_t ip, uint16_t port);
int oracle_nlisten(oracle_stack *st, int fd);
int oracle_naccept(oracle_stack *st, int fd, uint32_t *sip, uint16_t *sport);
int oracle_nclose(oracle_stack *st, int fd);
int oracle_rx(oracle_stack *st, const uint8_t *frame, uint32_t caplen);
void oracle_rx_burst(oracle_stack *st, const uint8_t *pkts, const uint32_t *off,
                     const uint16_t *len, uint32_t n, uint32_t unit_log2, int32_t *rcs);
long oracle_drain_all(oracle_stack *st, uint8_t *buf, size_t cap, uint64_t *bytes);
long oracle_nrecvfrom(oracle_stack *st, int fd, uint8_t *buf, size_t len, uint32_t *sip,
                      uint16_t *sport);
long oracle_nrecv(oracle_stack *st, int fd, uint8_t *buf, size_t len);
int oracle_tcb_state(const oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport,
                     uint16_t dport, int32_t *status, uint32_t *rcv_nxt, uint32_t *snd_nxt,
                     int32_t *fd);
int oracle_tcb_sndq(const oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport,
                    uint16_t dport, uint32_t k, uint8_t *flags, uint32_t *acknum);
uint32_t oracle_tcb_count(const oracle_stack *st);
/* test hook: install a tcb with this status (tcp_stream_create + LL_ADD) */
int oracle_tcb_add(oracle_stack *st, uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport,
                   int status);

#ifdef __cplusplus
}
#endif
#endif
