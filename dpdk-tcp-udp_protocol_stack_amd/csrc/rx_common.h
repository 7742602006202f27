// rx_common.h — helpers shared by the host side of librxgpu and its gfx950
// kernels (compiled by hipcc only): flow-table hashing and layout, Toeplitz
// RSS, the counter-based RNG and the synthetic frame builder.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rxgpu.h"

#define RX_HD __host__ __device__ __forceinline__

// ---------------------------------------------------------------------------
// Flow table (device image).  Exact-key tables use linear probing over 16-B
// slots {a, b, c, flow} at a load factor <= 1/4 (expected ~1.2 slot reads per
// lookup); flow == RX_SLOT_EMPTY marks a free slot.  A one-frame-per-lane
// kernel reads slots one by one; a lane group reads a window of 4 consecutive
// slots (one 64-B access) and __ballots the compare.  Keys are the raw
// network-order values the reference compares (common.c:101-103, 36-38):
//   UDP:  a = dst ip, b = dst port, c = 17           (get_hostinfo_fromip_port)
//   TCP:  a = src ip, b = dst ip, c = sport | dport<<16   (tcp_stream_search pass 1)
// Listeners (tcp_stream_search pass 2: dport + LISTEN, dst ip ignored) are a
// direct u32[65536] table indexed by the raw dport.
#define RX_SLOT_EMPTY 0xFFFFFFFFu
#define RX_FT_MIRROR 3 // slots past the table's end that mirror its first ones
#define RX_WINDOW 4

struct rx_ft_dev {
    const uint4 *udp;   // udp_mask + 1 slots
    const uint4 *tcp;   // tcp_mask + 1 slots
    const uint32_t *listen; // 65536 entries
    uint32_t udp_mask, tcp_mask;   // slots - 1 (power of two)
    uint32_t udp_probe, tcp_probe; // longest probe sequence (slots) of any present key
    uint32_t nu, nt;   // count layout: UDP ids [0, nu), then TCP ids at nu + id
    uint32_t hseed;    // rx_hash3s seed of every hashed table (exact keys, compact UDP)
    // compact UDP table for small socket sets (null otherwise), copied into LDS
    // by the lane kernel: slot = {dip, dport | flow << 16}, empty = y ~0u
    const uint2 *udpc;
    uint32_t udpc_mask, udpc_probe;
    // compact keys not bound to udp_dip: with a port window and none of them,
    // every UDP frame is decided without a probe (a miss outside the window is
    // a miss), so the probe-sequence length the per-context hash seed gives
    // the generator's unknown-flow key (:7) never enters the kernel's time
    uint32_t udpc_other;
    // UDP direct port table (null: not built): u32[65536] indexed by the raw
    // dst port, for sockets bound to udp_dip (the address most sockets share:
    // the host's own); see rx_udp_port_decide
    const uint32_t *udp_port;
    uint32_t udp_dip;
    // UDP port window (null: not built), with the compact table only: u16
    // flow ids (0xFFFF = none) of the sockets bound to udp_dip on host-order
    // ports [udpw_lo, udpw_lo + udpw_n), copied into LDS beside the compact
    // table so such keys are decided by one LDS read instead of a probe loop
    const uint16_t *udpw;
    uint32_t udpw_lo, udpw_n;
    // per-launch output, set by rx_classify_launch on its copy: on the slab
    // count path every kernel writes frame i's count index (UDP flow k -> k,
    // TCP flow k -> nu + k; all ones = not counted) to count_idx[i], which
    // the slab pass reads instead of the 16-B verdicts; null otherwise.  u16
    // indices when cidx16 (at most 65535 flows: one slab range), u32 otherwise
    void *count_idx;
    uint32_t cidx16;
    // 2-B indices with exactly 65536 flows: all ones would be both flow 65535
    // and "not counted", so the classify kernel adds flow 65535's frames to
    // this count itself (wave-aggregated atomics; its slab bin stays 0 and the
    // reduce never writes it), and all ones always means "not counted" to the
    // slab pass — which then never reads the verdicts (a later burst may be
    // rewriting them on another stream).  Null otherwise.
    unsigned long long *count_ffff;
    // rxg_tune_tables(RXG_TT_COUNT_4B): 4-B count indices whatever the flow
    // count (the round-1 count path, for A/B)
    uint32_t count_4b;
    // rxg_tune_tables(RXG_TT_SLAB_HALF / _QUARTER): the slab pass on 1/2 or 1/4 of
    // the CUs (log2 of the divisor; 0 = one 1024-thread block per CU)
    uint32_t slab_div_log2;
    // host side only: the burst's verdict format (0 = 16-B rxg_verdict, 1 =
    // 8-B rxg_verdict8, rxg_classify_dev8), which picks the launcher of the
    // RX_V8 build of rx_classify.hip; the kernels never read it
    uint32_t v8;
    // host side only: resident blocks per CU the launch may use (0 = as many
    // as the occupancy allows): rxg_tune_grid's cap, else the variant's
    // measured default (k_variants), set on rx_classify_launch's copy
    uint32_t bpc_cap;
};

// rx_classify_launch phases (host side)
enum { RX_PH_ALL = 0, RX_PH_CLASSIFY = 1, RX_PH_COUNT = 2 };

// frame p's count index (idx = ~0u: not counted) on the slab count path
RX_HD void rx_put_count_idx(const rx_ft_dev &ft, uint64_t p, uint32_t idx) {
    if (ft.cidx16)
        static_cast<uint16_t *>(ft.count_idx)[p] = (uint16_t)idx;
    else
        static_cast<uint32_t *>(ft.count_idx)[p] = idx;
}
#define RX_PORT_NONE 0x7FFFFFFFu   // udp_port entry: no socket (udp_dip, port)
#define RX_PORT_HASHED 0x80000000u // some socket on this port is bound to another ip

// UDP lookup (get_hostinfo_fromip_port, common.c:97-108) through the port
// table entry e = udp_port[dport]: true = decided (*flow set); false = the key
// must be probed in the hashed table (a socket on this port has another ip)
RX_HD bool rx_udp_port_decide(uint32_t e, uint32_t dip, uint32_t udp_dip, uint32_t *flow) {
    if (dip == udp_dip) {
        const uint32_t f = e & RX_PORT_NONE;
        *flow = f == RX_PORT_NONE ? RXG_FLOW_NONE : f;
        return true;
    }
    if (e & RX_PORT_HASHED) return false;
    *flow = RXG_FLOW_NONE;
    return true;
}
#define RX_UDPC_MAX_FLOWS 1024u // load <= 1/2: <= 2048 slots = 16 KiB of LDS
#define RX_UDPW_MAX_PORTS 4096u // port window: <= 8 KiB of LDS
#define RX_FT_LOAD_LOG2 2u      // exact-key tables: load <= 1/4 by default (rxg_tune_flow_load)

// Host: CU count of the calling thread's current device and the resident
// blocks per CU of kernel `fn` (`threads` per block, `lds` bytes of dynamic
// LDS) on it.  Cached per thread and keyed by (device, kernel, lds), so rx
// threads with their own contexts (and devices) never share mutable state.
hipError_t rx_occupancy(const void *fn, uint32_t threads, size_t lds, int *cu, int *occ);

// seed: per context (rx_ft_dev::hseed, drawn at rxg_open), so the slot a key
// lands in cannot be predicted from the key alone
RX_HD uint32_t rx_hash3s(uint32_t seed, uint32_t a, uint32_t b, uint32_t c) {
    uint32_t h = seed ^ a;
    h *= 0x85EBCA6Bu;
    h ^= h >> 15;
    h += b;
    h *= 0xC2B2AE35u;
    h ^= h >> 13;
    h += c;
    h *= 0x27D4EB2Fu;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}

RX_HD uint32_t rx_bswap16(uint32_t v) { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); }

// ---------------------------------------------------------------------------
// Toeplitz RSS with the standard 40-byte Microsoft key.  Input = sip, dip,
// sport, dport in wire order (raw network-order values, LE memory order).
// Only the first 16 key bytes are ever windowed for a 12-byte input.
RX_HD uint32_t rx_rss_window(uint32_t pos) {
    const uint64_t hi = 0x6d5a56da255b0ec2ull, lo = 0x4167253d43a38fb0ull;
    uint64_t w;
    if (pos == 0)
        w = hi;
    else if (pos < 64)
        w = (hi << pos) | (lo >> (64 - pos));
    else
        w = lo << (pos - 64);
    return (uint32_t)(w >> 32);
}

RX_HD uint32_t rx_rss_hash(uint32_t sip, uint32_t dip, uint32_t sport, uint32_t dport) {
    uint32_t r = 0;
    uint32_t words[3] = {sip, dip, (sport & 0xFFFFu) | (dport << 16)};
#pragma unroll
    for (int w = 0; w < 3; ++w) {
#pragma unroll
        for (int byte = 0; byte < 4; ++byte) {
            uint32_t v = (words[w] >> (8 * byte)) & 0xFFu;
#pragma unroll
            for (int bit = 7; bit >= 0; --bit)
                if (v & (1u << bit)) r ^= rx_rss_window((uint32_t)(32 * w + 8 * byte + (7 - bit)));
        }
    }
    return r;
}

// RSS hash of one frame from its first 40 bytes as little-endian dwords w[0..9]
// (bytes past the captured length already zero): the queue key a multi-queue
// NIC hashes — (sip, dip, sport, dport) for IPv4 TCP/UDP, (sip, dip) for other
// IPv4 — and 0 (queue 0) for non-IPv4 frames, which carry no IP tuple.
RX_HD uint32_t rx_rss_frame(const uint32_t *w) {
    if ((w[3] & 0xFFFFu) != 0x0008u) return 0; // ether_type bytes {08, 00}
    const uint32_t proto = w[5] >> 24;          // byte 23
    const uint32_t sip = (w[6] >> 16) | (w[7] << 16), dip = (w[7] >> 16) | (w[8] << 16);
    const bool l4 = proto == 6u || proto == 17u;
    return rx_rss_hash(sip, dip, l4 ? (w[8] >> 16) : 0u, l4 ? (w[9] & 0xFFFFu) : 0u);
}

#define RX_MAX_SHARDS 64u

// ---------------------------------------------------------------------------
// Counter-based RNG: value k of frame i is a pure function of (seed, i, k).
RX_HD uint64_t rx_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
RX_HD uint64_t rx_rng(uint64_t seed, uint64_t i, uint64_t k) {
    return rx_mix64(seed ^ rx_mix64(i * 0xD1B54A32D192ED03ull + k));
}

// ---------------------------------------------------------------------------
// Synthetic frame description (header fields decided from the RNG).
struct rx_frame_plan {
    uint32_t len;       // frame bytes
    uint32_t kind;      // 0 UDP, 1 TCP, 2 ICMP, 3 ARP
    uint32_t sip, dip;  // raw network order
    uint32_t sport, dport; // raw network order (LE u16 of the wire bytes)
    uint32_t bad;       // flip one payload bit after the checksum
    uint32_t seq;
};

RX_HD uint32_t rx_hton16(uint32_t host) { return rx_bswap16(host); }
RX_HD uint32_t rx_ip_net(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return a | (b << 8) | (c << 16) | (d << 24);
}

// Flow tuple of established tcb k of the generator's flow set.
RX_HD void rx_gen_tcb(const rxg_gen_cfg &cfg, uint32_t k, uint32_t *sip, uint32_t *sport) {
    // 10.128.0.0/9 + k, distinct per k; sport spread over 1024..61023
    uint32_t host = 0x800000u + k; // 23 bits
    *sip = rx_ip_net(10, (host >> 16) & 0xFF, (host >> 8) & 0xFF, host & 0xFF);
    *sport = rx_hton16(1024u + (k * 7919u) % 60000u);
}

RX_HD uint32_t rx_gen_len(const rxg_gen_cfg &cfg, uint64_t i) {
    if (cfg.size_mode == 1) {
        uint32_t r = (uint32_t)(rx_rng(cfg.seed, i, 2) % 12u);
        return r < 7 ? 64u : (r < 11 ? 576u : 1500u);
    }
    return cfg.frame_len;
}

RX_HD rx_frame_plan rx_gen_plan(const rxg_gen_cfg &cfg, uint64_t i) {
    rx_frame_plan pl;
    pl.len = rx_gen_len(cfg, i);
    pl.seq = (uint32_t)rx_rng(cfg.seed, i, 5);
    const uint32_t nsh = cfg.n_shards ? cfg.n_shards : 1;
    for (uint32_t a = 0;; ++a) {
        const uint64_t k0 = 16ull * a;
        uint32_t r = (uint32_t)(rx_rng(cfg.seed, i, k0 + 0) % 10000u);
        uint32_t tcp;
        if (cfg.proto_mode == 0)
            tcp = 0;
        else if (cfg.proto_mode == 1)
            tcp = 1;
        else
            tcp = (uint32_t)(rx_rng(cfg.seed, i, k0 + 1) & 1u);
        if (tcp && cfg.n_tcp == 0) tcp = 0;
        if (!tcp && cfg.n_udp == 0 && cfg.n_tcp) tcp = 1;
        uint64_t rsrc = rx_rng(cfg.seed, i, k0 + 4);
        uint32_t rnd_sip = rx_ip_net(10, (uint32_t)(rsrc >> 8) & 0x7F, (uint32_t)(rsrc >> 16) & 0xFF,
                                     (uint32_t)(rsrc >> 24) & 0xFF);
        uint32_t rnd_sport = rx_hton16(1024u + (uint32_t)((rsrc >> 32) % 60000u));
        pl.bad = 0;
        pl.dip = cfg.local_ip;
        uint32_t rss_ok_any = 0;
        if (r < cfg.other_per10k) {
            pl.kind = (rsrc & 1u) ? 2u : 3u;
            pl.sip = rnd_sip;
            pl.sport = 0;
            pl.dport = 0;
            rss_ok_any = (pl.kind == 3u); // ARP carries no IP tuple: any queue
        } else {
            uint32_t unknown = r < cfg.other_per10k + cfg.unknown_per10k;
            pl.bad = !unknown && r < cfg.other_per10k + cfg.unknown_per10k + cfg.bad_cksum_per10k;
            if (tcp) {
                pl.kind = 1;
                if (unknown) {
                    pl.sip = rnd_sip;
                    pl.sport = rnd_sport;
                    pl.dport = rx_hton16(7); // no listener on :7
                } else {
                    uint32_t k = (uint32_t)(rx_rng(cfg.seed, i, k0 + 3) % cfg.n_tcp);
                    rx_gen_tcb(cfg, k, &pl.sip, &pl.sport);
                    pl.dport = rx_hton16(cfg.tcp_port);
                }
            } else {
                pl.kind = 0;
                pl.sip = rnd_sip;
                pl.sport = rnd_sport;
                if (cfg.src_ip && !unknown) { // one client 5-tuple (BASELINE configs[0])
                    pl.sip = cfg.src_ip;
                    pl.sport = rx_hton16(cfg.src_port);
                }
                if (unknown) {
                    pl.dport = rx_hton16(7); // no socket bound to :7
                } else {
                    uint32_t k = (uint32_t)(rx_rng(cfg.seed, i, k0 + 3) % cfg.n_udp);
                    pl.dport = rx_hton16((uint32_t)cfg.udp_base_port + k);
                }
            }
        }
        if (nsh <= 1 || rss_ok_any || a >= 4096) break;
        uint32_t h = rx_rss_hash(pl.sip, pl.dip, pl.sport, pl.dport);
        if (h % nsh == cfg.shard) break;
    }
    if (pl.kind >= 2 && pl.len < 60) pl.len = 60;
    return pl;
}

// Payload word: frame bytes [4j, 4j+4) for every j past the headers.
RX_HD uint32_t rx_payload_word(const rxg_gen_cfg &cfg, uint64_t i, uint32_t j) {
    return (uint32_t)rx_rng(cfg.seed, i, 64u + j);
}

// Header bytes of a planned frame into hdr[0..63] (64 bytes, zero padded);
// returns the header length.  The L4 checksum field is written as computed
// by rte_ipv4_udptcp_cksum (rte_ip.h:325-349) over the whole frame so that a
// clean frame verifies; `bad` flips bit 0 of the last payload byte afterwards.
struct rx_hdr64 {
    uint32_t w[16];
};

RX_HD void rx_put8(rx_hdr64 &h, uint32_t pos, uint32_t v) {
    uint32_t sh = 8u * (pos & 3u);
    h.w[pos >> 2] = (h.w[pos >> 2] & ~(0xFFu << sh)) | ((v & 0xFFu) << sh);
}
RX_HD void rx_put16le(rx_hdr64 &h, uint32_t pos, uint32_t v) {
    rx_put8(h, pos, v & 0xFF);
    rx_put8(h, pos + 1, (v >> 8) & 0xFF);
}
RX_HD void rx_put16be(rx_hdr64 &h, uint32_t pos, uint32_t v) {
    rx_put8(h, pos, (v >> 8) & 0xFF);
    rx_put8(h, pos + 1, v & 0xFF);
}
RX_HD void rx_put32raw(rx_hdr64 &h, uint32_t pos, uint32_t v) {
    rx_put16le(h, pos, v & 0xFFFF);
    rx_put16le(h, pos + 2, v >> 16);
}
RX_HD uint32_t rx_get16le(const rx_hdr64 &h, uint32_t pos) {
    uint32_t lo = (h.w[pos >> 2] >> (8u * (pos & 3u))) & 0xFFu;
    uint32_t hi = (h.w[(pos + 1) >> 2] >> (8u * ((pos + 1) & 3u))) & 0xFFu;
    return lo | (hi << 8);
}

RX_HD uint32_t rx_fold(uint32_t s) {
    s = (s >> 16) + (s & 0xFFFFu);
    s = (s >> 16) + (s & 0xFFFFu);
    return s;
}

// Sum of LE 16-bit words of frame bytes [from, len) where bytes below hdr_len
// come from h and the rest from payload words. from is even.
RX_HD uint32_t rx_frame_sum(const rxg_gen_cfg &cfg, uint64_t i, const rx_hdr64 &h, uint32_t hdr_len,
                            uint32_t from, uint32_t len) {
    uint32_t s = 0;
    uint32_t q = from;
    for (; q + 1 < len && q < hdr_len; q += 2) {
        // header word (hdr_len is even, so q+1 < hdr_len)
        s += rx_get16le(h, q);
    }
    // q is now hdr_len (even) or past len
    if (q < len && (q & 2u)) { // finish the straddling 32-bit payload word
        uint32_t w = rx_payload_word(cfg, i, q >> 2);
        if (q + 1 < len)
            s += w >> 16;
        else
            s += (w >> 16) & 0xFFu;
        q += 2;
    }
    for (; q + 3 < len; q += 4) {
        uint32_t w = rx_payload_word(cfg, i, q >> 2);
        s += (w & 0xFFFFu) + (w >> 16);
    }
    if (q < len) { // 1..3 trailing bytes
        uint32_t w = rx_payload_word(cfg, i, q >> 2);
        uint32_t rem = len - q;
        if (rem == 1)
            s += w & 0xFFu;
        else if (rem == 2)
            s += w & 0xFFFFu;
        else
            s += (w & 0xFFFFu) + ((w >> 16) & 0xFFu);
    }
    return s;
}

RX_HD uint32_t rx_build_header(const rxg_gen_cfg &cfg, uint64_t i, const rx_frame_plan &pl,
                               rx_hdr64 &h) {
    for (int k = 0; k < 16; ++k) h.w[k] = 0;
    // Ethernet: dst 00:0c:29:6a:01:4d (arbitrary local MAC), src from RNG
    const uint32_t dmac[6] = {0x00, 0x0c, 0x29, 0x6a, 0x01, 0x4d};
    uint64_t rm = rx_rng(cfg.seed, i, 6);
    for (int k = 0; k < 6; ++k) rx_put8(h, k, dmac[k]);
    rx_put8(h, 6, 0x02); // locally administered
    for (int k = 1; k < 6; ++k) rx_put8(h, 6 + k, (uint32_t)(rm >> (8 * k)));
    if (pl.kind == 3) { // ARP request for local_ip
        rx_put16be(h, 12, 0x0806);
        rx_put16be(h, 14, 1);      // htype ethernet
        rx_put16be(h, 16, 0x0800); // ptype ipv4
        rx_put8(h, 18, 6);
        rx_put8(h, 19, 4);
        rx_put16be(h, 20, 1); // request
        for (int k = 0; k < 6; ++k) rx_put8(h, 22 + k, (k == 0) ? 0x02 : (uint32_t)(rm >> (8 * k)));
        rx_put32raw(h, 28, pl.sip);
        rx_put32raw(h, 38, pl.dip);
        return 42;
    }
    rx_put16be(h, 12, 0x0800);
    const uint32_t tl = pl.len - 14;
    const uint32_t proto = pl.kind == 0 ? 17u : (pl.kind == 1 ? 6u : 1u);
    rx_put8(h, 14, 0x45);
    rx_put8(h, 15, 0);
    rx_put16be(h, 16, tl);
    rx_put16be(h, 18, (uint32_t)i & 0xFFFFu);
    rx_put16be(h, 20, 0x4000); // DF
    rx_put8(h, 22, 64);
    rx_put8(h, 23, proto);
    rx_put32raw(h, 26, pl.sip);
    rx_put32raw(h, 30, pl.dip);
    // IPv4 header checksum (rte_ipv4_cksum, rte_ip.h:255-265)
    {
        uint32_t s = 0;
        for (uint32_t q = 14; q < 34; q += 2) s += rx_get16le(h, q);
        uint32_t c = rx_fold(s);
        c = (c == 0xFFFFu) ? c : (~c & 0xFFFFu);
        rx_put16le(h, 24, c);
    }
    uint32_t hdr_len, hole;
    if (pl.kind == 0) {
        rx_put16le(h, 34, pl.sport);
        rx_put16le(h, 36, pl.dport);
        rx_put16be(h, 38, tl - 20);
        hdr_len = 42;
        hole = 40;
    } else if (pl.kind == 1) {
        rx_put16le(h, 34, pl.sport);
        rx_put16le(h, 36, pl.dport);
        rx_put16be(h, 38, pl.seq >> 16);
        rx_put16be(h, 40, pl.seq & 0xFFFF);
        uint32_t ack = (uint32_t)rx_rng(cfg.seed, i, 7);
        rx_put16be(h, 42, ack >> 16);
        rx_put16be(h, 44, ack & 0xFFFF);
        rx_put8(h, 46, 0x50);
        rx_put8(h, 47, 0x18); // PSH|ACK
        rx_put16be(h, 48, 14600);
        rx_put16be(h, 52, 0);
        hdr_len = 54;
        hole = 50;
    } else { // ICMP echo request
        rx_put8(h, 34, 8);
        rx_put8(h, 35, 0);
        rx_put16be(h, 38, (uint32_t)i & 0xFFFF);
        rx_put16be(h, 40, 1);
        return 42;
    }
    // L4 checksum over pseudo header + [34, len) with the field at 0
    uint32_t s = rx_frame_sum(cfg, i, h, hdr_len, 26, pl.len); // src/dst + l4
    s += proto << 8;
    s += rx_bswap16(tl - 20);
    uint32_t c = (~rx_fold(s)) & 0xFFFFu;
    if (c == 0 && proto == 17) c = 0xFFFFu;
    rx_put16le(h, hole, c);
    return hdr_len;
}

// Frame word j (bytes [4j, 4j+4)) of frame i.
RX_HD uint32_t rx_frame_word(const rxg_gen_cfg &cfg, uint64_t i, const rx_frame_plan &pl,
                             const rx_hdr64 &h, uint32_t hdr_len, uint32_t j) {
    uint32_t w;
    if (4 * j + 4 <= hdr_len) {
        w = h.w[j];
    } else if (4 * j >= hdr_len) {
        w = rx_payload_word(cfg, i, j);
    } else { // straddles (hdr_len % 4 == 2)
        w = (h.w[j] & 0x0000FFFFu) | (rx_payload_word(cfg, i, j) & 0xFFFF0000u);
    }
    if (pl.bad && j == (pl.len - 1) / 4) w ^= 1u << (8 * ((pl.len - 1) & 3u));
    // bytes past the frame end inside its last word are zero
    if (4 * j + 4 > pl.len) {
        uint32_t keep = pl.len - 4 * j; // 1..3
        w &= (1u << (8 * keep)) - 1u;
    }
    return w;
}
