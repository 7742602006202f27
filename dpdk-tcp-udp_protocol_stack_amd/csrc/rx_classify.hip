// rx_classify.hip — K1: fused parse + L4 checksum + flow classify (gfx950).
//
// Three kernel shapes, picked per typical frame length by rx_pick_variant
// (bottom of this file); every shape is correct for any layout and length:
//   lane kernel   (rx_classify_lane_kernel)   one frame per lane: 64-B frames
//                 (heads staged through LDS by coalesced 1-KiB wave loads,
//                 two tiles' bytes (a grid stride apart) issued per trip,
//                 descriptors one trip ahead, UDP table and port window in LDS);
//   group kernel  (rx_classify_kernel)        G lanes per frame: 1500-B frames
//                 (described below);
//   stream kernel (rx_classify_stream_kernel) heads per thread, tails streamed
//                 by the block as one contiguous span with prefix sums: mixed
//                 sizes (IMIX) and jumbo frames.
// The variant table (k_variants) holds the defaults and a few measured
// alternatives; tuning shapes and diagnostic ablations (wrong verdicts by
// construction) compile only into the RX_DIAG build (librxgpu_diag.so).
//
// Group kernel work decomposition
//   A frame is owned by a lane GROUP of G lanes (G = 4..64, power of two).
//   Lane k of the group reads the 16-B chunks k, k+G, k+2G, ... of the frame;
//   one "pass" of the group covers 16*G contiguous frame bytes, so a wave
//   instruction loads 64 x 16 B = 1 KiB of contiguous HBM (frames are packed).
//   Each group handles FPG frames per loop trip, and each frame's first P
//   passes are loaded up front: all FPG*P loads of a lane are in flight before
//   the first one is consumed (memory-level parallelism without LDS staging;
//   the bytes are touched once, so there is nothing to reuse from LDS).
//   A block (256 threads) covers a tile of (256/G)*FPG consecutive frames per
//   trip; blocks stride over tiles, and the grid is sized to the number of
//   blocks the chip keeps resident, so every block gets the same share.
//
// Per frame (reference behaviour, see ../../include/rxgpu.h)
//   pkt_process demux           netfamily.c:152-200
//   udp_process front           udp.c:11-19, 37-46
//   tcp_process front           tcp.c:345-371 (checksum with the field zeroed)
//   rte_ipv4_udptcp_cksum       rte_ip.h:325-349 (DPDK 19.11.12; IHL ignored)
//   get_hostinfo_fromip_port    common.c:97-108   -> UDP bucket probe
//   tcp_stream_search           common.c:31-55    -> TCP bucket probe, then listener table
//
// Checksum arithmetic
//   The reference value is fold(S), S = plain sum of the little-endian 16-bit
//   words of [ip.src, ip+tl) plus the pseudo words {0,proto} and be16(tl-20),
//   with the L4 checksum field read as 0; fold = end-around-carry reduction,
//   0 iff S == 0.  fold only depends on S mod 0xFFFF and on S == 0, so any
//   split of the words over lanes works as long as partial sums are exact
//   integers: each lane adds its dwords' two halves with v_dot2_u32_u16
//   (x.lo*1 + x.hi*1 + acc), the group adds lane sums with DPP / swizzle, and
//   the one fold happens at the end.  Bytes outside [26, min(34+tl-20, caplen))
//   and the 2-byte checksum field are masked out: lanes 0..3 of pass 0 own the
//   header bytes (compile-time masks), only the chunk that straddles the end
//   needs a computed mask.
//
// Flow probe
//   Buckets are 4 slots x 16 B = one 64-B line; lanes 0..3 of the group load
//   the 4 slots of a bucket in one coalesced access and __ballot the compare.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rx_common.h"
#include "rx_device.h"

// This file is compiled twice (Makefile): RX_V8 = 0 writes the 16-B
// rxg_verdict, RX_V8 = 1 the 8-B rxg_verdict8 (rxg_classify_dev8).  The
// second build exports only rx_classify_launch8, so the
// format is a compile-time choice in every kernel: no branch on either path
// (a run-time switch measured 0.2-0.6% slower on the 16-B path, r03e).
#ifndef RX_V8
#define RX_V8 0
#endif
#if RX_V8
#define RX_K1_NAME(x) x##8
#else
#define RX_K1_NAME(x) x
#endif

namespace {


// Frames of one lane group for one trip: descriptors and the first P passes.
// flow 65535 at exactly 65536 flows with 2-B count indices (rx_ft_dev::
// count_ffff): its frames are added here, one atomic per wave
__device__ __forceinline__ void count_ffff(const rx_ft_dev &ft, uint32_t idx) {
    const bool hit = idx == 0xFFFFu; // (not counted = 0xFFFFFFFF)
    const uint64_t m = __ballot(hit);
    if (m && hit && __lane_id() == (uint32_t)__builtin_ctzll(m))
        atomicAdd(ft.count_ffff, (unsigned long long)__popcll(m));
}

// per-lane count index (lane kernels, group kernels)
__device__ __forceinline__ void put_count_idx(const rx_ft_dev &ft, uint64_t p, uint32_t idx) {
    if (ft.count_ffff) count_ffff(ft, idx);
    rx_put_count_idx(ft, p, idx);
}

// The verdict store.  RX_V8: the compact 8-B verdict
// (rxg_verdict8, include/rxgpu.h) packed from the 16-B one: flow id; then
// payload_len | payload_off (7 bits) + TCP_NEGLEN << 7 | cls | rc (3-bit
// two's complement) << 3 | cksum_ok << 6 | TRUNC << 7.  Everything the
// reference decides per frame; only the two checksum values (l4_cksum,
// stored_cksum: cksum_ok is their comparison) stay in the 16-B form.
__device__ __forceinline__ uint64_t verdict8_of(uint4 v) {
    const uint32_t hi = (v.y >> 16) | ((v.y & 0x7Fu) << 16) | ((v.w & 0x200u) << 14) |
                        (((v.z >> 16) & 7u) << 24) | (((v.z >> 24) & 7u) << 27) |
                        ((v.w & 1u) << 30) | ((v.w & 0x100u) << 23);
    return (uint64_t)v.x | ((uint64_t)hi << 32);
}
// WT: write-through (sc1) stores; PLAIN: ordinary stores; else non-temporal
template <bool WT = false, bool PLAIN = false>
__device__ __forceinline__ void st_verdict(const rx_ft_dev &ft, uint4 *__restrict__ out, uint64_t p,
                                           uint4 v) {
    if constexpr (RX_V8) {
        uint64_t *o = reinterpret_cast<uint64_t *>(out) + p;
        const uint64_t w = verdict8_of(v);
        if constexpr (WT)
            asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(o), "v"(w) : "memory");
        else if constexpr (PLAIN)
            *o = w;
        else
            __builtin_nontemporal_store(w, o);
    } else if constexpr (WT) {
        stg16_wt(&out[p], v);
    } else if constexpr (PLAIN) {
        out[p] = v;
    } else {
        stg16(&out[p], v);
    }
}

template <int FPG, int P>
struct group_frames {
    uint64_t pf[FPG]; // frame index (the verdict slot)
    bool valid[FPG];
    const uint8_t *fb[FPG];
    int32_t cap[FPG];
    uint4 c[FPG][P];
};

template <int G, int FPG, int P>
__device__ __forceinline__ void group_desc(group_frames<FPG, P> &S, uint64_t tile, uint32_t n,
                                           uint32_t grp, const uint8_t *__restrict__ pkts,
                                           const uint32_t *__restrict__ off,
                                           const uint16_t *__restrict__ len, uint32_t unit_log2,
                                           const uint32_t *__restrict__ idx = nullptr) {
    constexpr uint32_t GPB = 256 / G;
#pragma unroll
    for (int f = 0; f < FPG; ++f) {
        const uint64_t pos = tile * (GPB * FPG) + (uint64_t)f * GPB + grp;
        S.valid[f] = pos < n;
        const uint64_t pp = S.valid[f] ? pos : 0;
        const uint64_t q = idx ? (uint64_t)idx[pp] : pp;
        S.pf[f] = q;
        S.fb[f] = pkts + ((uint64_t)off[q] << unit_log2);
        S.cap[f] = S.valid[f] ? (int32_t)len[q] : 0;
    }
}

template <int G, int FPG, int P, bool NTL = true>
__device__ __forceinline__ void group_load(group_frames<FPG, P> &S, int32_t s0) {
#pragma unroll
    for (int f = 0; f < FPG; ++f)
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const int32_t s = s0 + q * 16 * G;
            S.c[f][q] = make_uint4(0, 0, 0, 0);
            if (s < S.cap[f]) S.c[f][q] = ldg16<NTL>(S.fb[f] + s);
        }
}

// parse + checksum + probe + verdict for the FPG frames of S.
// RI = 0: passes past the first P are summed frame by frame in batches of 4
// (one HBM round trip per batch and frame).  RI > 0: the remaining passes of
// all FPG frames are loaded together, RI passes per frame per batch (FPG*RI
// loads of a lane in flight; a pass past a frame's end loads the frame's first
// chunk again, an L1/L2 hit, and adds nothing), which keeps enough bytes in
// flight for jumbo frames.
template <int G, int P, int FPG, bool NTL = true, int RI = 0, bool WT = false, bool H16 = false>
__device__ __forceinline__ void group_process(group_frames<FPG, P> &S, uint32_t gl, uint32_t gbase,
                                              int32_t s0, const rx_ft_dev &ft,
                                              uint4 *__restrict__ out,
                                              unsigned long long *__restrict__ counts,
                                              uint32_t *hist, uint32_t lds_bins,
                                              uint4 *vb = nullptr) {
    constexpr int32_t STEP = 16 * G;
    // ---- phase C: parse + checksum per frame
    uint32_t cls[FPG], ck[FPG], stored[FPG], tl[FPG], dgl[FPG], hl[FPG], need[FPG];
    uint32_t ka[FPG], kb[FPG], kc[FPG], dport[FPG];
    uint32_t accs[FPG], protos[FPG];
    int32_t ends[FPG];
    bool ok[FPG], sums[FPG];
#pragma unroll
    for (int f = 0; f < FPG; ++f) {
        const int32_t cp = S.cap[f];
        uint4 x0 = S.c[f][0];
        if (s0 < cp && s0 + 16 > cp) x0 = chunk_below(x0, s0, cp); // bytes past caplen read 0
        const uint32_t h03 = gbcast<G, 0>(x0.w); // bytes 12..15
        const uint32_t h10 = gbcast<G, 1>(x0.x); // 16..19
        const uint32_t h11 = gbcast<G, 1>(x0.y); // 20..23
        const uint32_t h12 = gbcast<G, 1>(x0.z); // 24..27
        const uint32_t h13 = gbcast<G, 1>(x0.w); // 28..31
        const uint32_t h20 = gbcast<G, 2>(x0.x); // 32..35
        const uint32_t h21 = gbcast<G, 2>(x0.y); // 36..39
        const uint32_t h22 = gbcast<G, 2>(x0.z); // 40..43
        const uint32_t h23 = gbcast<G, 2>(x0.w); // 44..47
        const uint32_t h30 = gbcast<G, 3>(x0.x); // 48..51

        const uint32_t et = h03 & 0xFFFFu; // LE view of bytes 12,13
        tl[f] = rx_bswap16(h10 & 0xFFFFu);
        const uint32_t proto = h11 >> 24;
        const uint32_t sip = (h12 >> 16) | (h13 << 16);
        const uint32_t dip = (h13 >> 16) | (h20 << 16);
        const uint32_t sport = h20 >> 16;
        dport[f] = h21 & 0xFFFFu;
        dgl[f] = rx_bswap16(h21 >> 16);
        hl[f] = ((h23 >> 16) & 0xFFu) >> 4;

        uint32_t cl, nd;
        if (et == 0x0608u) {
            cl = RXG_CLS_ARP;
            nd = 42;
        } else if (et != 0x0008u) {
            cl = RXG_CLS_NON_IP;
            nd = 14;
        } else if (proto == 17u) {
            cl = RXG_CLS_UDP;
            nd = 42;
        } else if (proto == 6u) {
            cl = RXG_CLS_TCP;
            nd = 54;
        } else {
            cl = RXG_CLS_IPV4_OTHER;
            nd = 24;
        }
        const bool is_udp = cl == RXG_CLS_UDP, is_tcp = cl == RXG_CLS_TCP;
        const bool l4 = is_udp || is_tcp;
        const uint32_t l4n = tl[f] >= 20u ? tl[f] - 20u : 0u;
        const bool do_sum = l4 && tl[f] >= 20u;
        if (l4 && 34u + l4n > nd) nd = 34u + l4n;
        cls[f] = cl;
        need[f] = nd;

        // checksum region [26, e): e = min(34 + l4n, caplen)
        int32_t e = do_sum ? 34 + (int32_t)l4n : 0;
        if (e > cp) e = cp;
        uint32_t acc = 0;
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const int32_t s = s0 + q * STEP;
            uint4 v = S.c[f][q];
            if (s + 16 > e) v = chunk_below(v, s, e);
            if (q == 0) { // header bytes [0,26) and the checksum field are not summed
                if (gl == 0) v = make_uint4(0, 0, 0, 0);
                if (gl == 1) {
                    v.x = 0;
                    v.y = 0;
                    v.z &= 0xFFFF0000u;
                }
                if (gl == 2 && is_udp) v.z &= 0xFFFF0000u; // UDP cksum at 40..41
                if (gl == 3 && is_tcp) v.x &= 0x0000FFFFu; // TCP cksum at 50..51
            }
            acc = add_halves(acc, v.x);
            acc = add_halves(acc, v.y);
            acc = add_halves(acc, v.z);
            acc = add_halves(acc, v.w);
        }
        // frames longer than P passes: the rest in batches of 4 passes
        for (int32_t sb = P * STEP; RI == 0 && sb < e; sb += 4 * STEP) { // group-uniform
            uint4 r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int32_t s = s0 + sb + u * STEP;
                r[u] = make_uint4(0, 0, 0, 0);
                if (s < e) r[u] = ldg16(S.fb[f] + s);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int32_t s = s0 + sb + u * STEP;
                uint4 v = r[u];
                if (s + 16 > e) v = chunk_below(v, s, e);
                acc = add_halves(acc, v.x);
                acc = add_halves(acc, v.y);
                acc = add_halves(acc, v.z);
                acc = add_halves(acc, v.w);
            }
        }
        accs[f] = acc;
        ends[f] = e;
        protos[f] = proto;
        sums[f] = do_sum;
        stored[f] = is_udp ? (h22 & 0xFFFFu) : (is_tcp ? (h30 >> 16) : 0u);
        ka[f] = is_udp ? dip : sip;
        kb[f] = is_udp ? dport[f] : dip;
        kc[f] = is_udp ? 17u : (sport | (dport[f] << 16));
    }
    if constexpr (RI > 0) { // the remaining passes of all frames, RI per frame in flight
        int32_t emax = ends[0];
#pragma unroll
        for (int f = 1; f < FPG; ++f) emax = ends[f] > emax ? ends[f] : emax;
        for (int32_t sb = P * STEP; sb < emax; sb += RI * STEP) {
            uint4 r[FPG][RI];
#pragma unroll
            for (int f = 0; f < FPG; ++f)
#pragma unroll
                for (int u = 0; u < RI; ++u) { // unconditional: partial wait counts
                    const int32_t s = s0 + sb + u * STEP;
                    r[f][u] = ldg16<NTL>(S.fb[f] + (s < ends[f] ? s : 0));
                }
#pragma unroll
            for (int f = 0; f < FPG; ++f)
#pragma unroll
                for (int u = 0; u < RI; ++u) {
                    const int32_t s = s0 + sb + u * STEP;
                    uint4 v = r[f][u];
                    if (s + 16 > ends[f]) v = chunk_below(v, s, ends[f]); // all-zero past the end
                    uint32_t a = accs[f];
                    a = add_halves(a, v.x);
                    a = add_halves(a, v.y);
                    a = add_halves(a, v.z);
                    accs[f] = add_halves(a, v.w);
                }
        }
    }
#pragma unroll
    for (int f = 0; f < FPG; ++f) {
        uint32_t sum = gsum<G>(accs[f]);
        uint32_t k = 0;
        if (sums[f]) {
            sum += protos[f] << 8;                    // psd {zero, proto}
            sum += rx_bswap16((uint32_t)tl[f] - 20u); // psd be16(l4_len)
            k = (~fold16(sum)) & 0xFFFFu;
            if (k == 0u && protos[f] == 17u) k = 0xFFFFu;
        }
        ck[f] = k;
        ok[f] = (cls[f] == RXG_CLS_UDP || cls[f] == RXG_CLS_TCP) && stored[f] == k;
    }

    // ---- phase D: flow probes, a 4-slot window per lane group, the first
    // window of every frame in flight
    uint32_t flow[FPG], slot[FPG];
    uint4 sl[FPG];
    bool probe[FPG];
#pragma unroll
    for (int f = 0; f < FPG; ++f) {
        probe[f] = S.valid[f] && (cls[f] == RXG_CLS_UDP || (cls[f] == RXG_CLS_TCP && ok[f]));
        const bool udp = cls[f] == RXG_CLS_UDP;
        // UDP through the direct port table (one entry, the same for the whole
        // group); only keys it cannot decide go on to the hashed probe
        uint32_t fd = RXG_FLOW_NONE;
        if (probe[f] && udp && ft.udp_port &&
            rx_udp_port_decide(ft.udp_port[dport[f]], ka[f], ft.udp_dip, &fd))
            probe[f] = false;
        flow[f] = fd;
        const uint32_t mask = udp ? ft.udp_mask : ft.tcp_mask;
        slot[f] = rx_hash3s(ft.hseed, ka[f], kb[f], kc[f]) & mask;
        sl[f] = make_uint4(0, 0, 0, RX_SLOT_EMPTY);
        if (probe[f] && gl < RX_WINDOW) sl[f] = ld_slot((udp ? ft.udp : ft.tcp) + ((slot[f] + gl) & mask));
    }
#pragma unroll
    for (int f = 0; f < FPG; ++f) {
        const bool udp = cls[f] == RXG_CLS_UDP;
        const uint4 *tbl = udp ? ft.udp : ft.tcp;
        const uint32_t mask = udp ? ft.udp_mask : ft.tcp_mask;
        const uint32_t maxp = udp ? ft.udp_probe : ft.tcp_probe;
        uint4 s = sl[f];
        uint32_t b = slot[f];
        for (uint32_t pr = 0; pr < maxp; pr += RX_WINDOW) { // trips are group-uniform
            const bool hit = probe[f] && gl < RX_WINDOW && s.w != RX_SLOT_EMPTY &&
                             s.x == ka[f] && s.y == kb[f] && s.z == kc[f];
            const bool emp = probe[f] && gl < RX_WINDOW && s.w == RX_SLOT_EMPTY;
            const uint32_t gh = (uint32_t)(__ballot(hit) >> gbase) & 0xFu;
            const uint32_t ge = (uint32_t)(__ballot(emp) >> gbase) & 0xFu;
            // linear probing: the first hit-or-empty slot of the window decides
            const uint32_t first = (uint32_t)__ffs(gh | ge) - 1u; // 31 if neither (ffs 0)
            const uint32_t v = __shfl(s.w, gbase + (first & 3u));
            if (!probe[f]) break; // probe[f], gh, ge are uniform across the group
            if ((gh | ge) != 0u) {
                if (gh & (1u << first)) flow[f] = v;
                break;
            }
            b = (b + RX_WINDOW) & mask;
            s = make_uint4(0, 0, 0, RX_SLOT_EMPTY);
            if (gl < RX_WINDOW) s = ld_slot(tbl + ((b + gl) & mask));
        }
        if (S.valid[f] && cls[f] == RXG_CLS_TCP && ok[f] && flow[f] == RXG_FLOW_NONE)
            flow[f] = ft.listen[dport[f]];
    }

    // ---- phase E: verdicts (reference return codes) + counts
#pragma unroll
    for (int f = 0; f < FPG; ++f) {
        int32_t rc;
        uint32_t poff = 0, plen = 0, flags = 0, nd = need[f];
        if (cls[f] == RXG_CLS_UDP) {
            rc = flow[f] == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                          : (dgl[f] <= 8u ? RXG_RC_UDP_NOMEM : RXG_RC_OK);
            poff = 42;
            plen = dgl[f] > 8u ? dgl[f] - 8u : 0u;
            if (dgl[f] <= 8u) flags |= RXG_F_UDP_SHORT;
            if (rc == RXG_RC_OK && 42u + plen > nd) nd = 42u + plen;
        } else if (cls[f] == RXG_CLS_TCP) {
            const int32_t pl = (int32_t)tl[f] - 20 - 4 * (int32_t)hl[f];
            poff = 34u + 4u * hl[f];
            if (pl < 0) flags |= RXG_F_TCP_NEGLEN;
            plen = pl < 0 ? 0u : (uint32_t)pl;
            rc = !ok[f] ? RXG_RC_TCP_BAD_CKSUM
                        : (flow[f] == RXG_FLOW_NONE ? RXG_RC_TCP_NO_TCB : RXG_RC_OK);
        } else {
            rc = RXG_RC_KNI;
        }
        if ((int32_t)nd > S.cap[f]) flags |= RXG_F_TRUNC;
        if (gl == 0 && S.valid[f]) {
            uint4 v;
            v.x = flow[f];
            v.y = (poff & 0xFFFFu) | (plen << 16);
            v.z = ck[f] | (cls[f] << 16) | (((uint32_t)rc & 0xFFu) << 24);
            v.w = (ok[f] ? 1u : 0u) | (flags << 8) | (stored[f] << 16);
            if (vb) // write-batched (WB): the trip's slot in the block's LDS batch
                vb[(uint32_t)f * (256u / G) + threadIdx.x / G] = v;
            else
                st_verdict<WT>(ft, out, S.pf[f], v);
            const bool counted = rc == RXG_RC_OK && flow[f] != RXG_FLOW_NONE;
            const uint32_t idx = (cls[f] == RXG_CLS_TCP ? ft.nu : 0u) + flow[f];
            if (counts && counted) {
                if (lds_bins) {
                    if constexpr (H16) // 16-bit bin pairs (the launch bounds a block's frames < 65536)
                        atomicAdd(&hist[idx >> 1], 1u << ((idx & 1u) * 16u));
                    else
                        atomicAdd(&hist[idx], 1u);
                } else {
                    atomicAdd(&counts[idx], 1ull);
                }
            }
            if (ft.count_idx) put_count_idx(ft, S.pf[f], counted ? idx : 0xFFFFFFFFu);
        }
    }
}

// PIPE = 1: trip t+1's descriptors are fetched one trip ahead and its frame
// bytes are issued before trip t is processed (one extra frame set of
// registers), so both HBM round trips overlap the previous trip's work.
// WT: write-through (sc1) verdict stores, which leave the XCD's L2 (A/B, pipe 40)
// WB > 0 (write-batched, PIPE 0, not in index-list mode): block b owns the
// contiguous tiles [b*per, (b+1)*per) instead of every gridDim-th tile, keeps
// the verdicts of WB consecutive tiles in LDS and writes them out together,
// WB * TILE * 16 contiguous bytes (sc1 when WT).  The verdicts are a sparse
// write stream beside 1500-B frames (1% of the bytes): a burst read with one
// 16-B store per slot ran 12-14% slower than the same read without it, and
// the same stores bunched per block 2-3% faster than per trip
// (tools/membw_cfg3, profiles/r06c, r06d).
// H16: the per-block LDS histogram in 16-bit bin pairs (half the LDS; the
// launch uses it only when no block classifies 65536 frames or more)
template <int G, int P, int FPG, int PIPE, bool NTL = true, int RI = 0, int MINW = 1, bool WT = false,
          int WB = 0, bool H16 = false>
__global__ __launch_bounds__(256, MINW) void rx_classify_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t n, uint32_t unit_log2, rx_ft_dev ft,
    uint4 *__restrict__ out, unsigned long long *__restrict__ counts, uint32_t lds_bins,
    const uint32_t *__restrict__ idx, const uint32_t *__restrict__ n_dev) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    if (n_dev) n = min(n, *n_dev); // index-list mode: the list length lives on the device
    static_assert(G >= 4 && G <= 64 && (G & (G - 1)) == 0, "G must be a power of two in [4,64]");
    constexpr uint32_t GPB = 256 / G;     // frame groups per block
    constexpr uint32_t TILE = GPB * FPG;  // frames per block per trip

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t gbase = lane & ~(uint32_t)(G - 1);
    const uint32_t grp = tid / G;
    const int32_t s0 = 16 * (int32_t)gl;

    const uint32_t hwords = H16 ? (lds_bins + 1u) / 2u : lds_bins; // histogram words
    if (lds_bins) {
        for (uint32_t i = tid; i < hwords; i += 256) hist[i] = 0;
        __syncthreads();
    }
    // the block's histogram into the global counts (H16: two bins per word)
    auto flush_hist = [&]() {
        for (uint32_t i = tid; i < hwords; i += 256) {
            const uint32_t c = hist[i];
            if constexpr (H16) {
                if (c & 0xFFFFu) atomicAdd(&counts[2 * i], (unsigned long long)(c & 0xFFFFu));
                if ((c >> 16) && 2 * i + 1 < lds_bins) atomicAdd(&counts[2 * i + 1], (unsigned long long)(c >> 16));
            } else {
                if (c) atomicAdd(&counts[i], (unsigned long long)c);
            }
        }
    };

    if constexpr (WB > 0) {
        if (!idx) { // block-uniform
            uint4 *vb = reinterpret_cast<uint4 *>(hist + ((hwords + 3u) & ~3u));
            const uint64_t tiles = ((uint64_t)n + TILE - 1) / TILE;
            const uint64_t per = (tiles + gridDim.x - 1) / gridDim.x;
            const uint64_t t0 = (uint64_t)blockIdx.x * per;
            const uint64_t t1 = t0 + per < tiles ? t0 + per : tiles;
            group_frames<FPG, P> A;
            if (t0 < t1) {
                group_desc<G>(A, t0, n, grp, pkts, off, len, unit_log2);
                group_load<G, FPG, P, NTL>(A, s0);
            }
            uint32_t k = 0;
            uint64_t first = t0;
            for (uint64_t tile = t0; tile < t1; ++tile) { // block-uniform trips
                group_process<G, P, FPG, NTL, RI, WT, H16>(A, gl, gbase, s0, ft, out, counts, hist,
                                                           lds_bins, vb + k * TILE);
                if (tile + 1 < t1) { // the next tile's loads go out before the batch is written
                    group_desc<G>(A, tile + 1, n, grp, pkts, off, len, unit_log2);
                    group_load<G, FPG, P, NTL>(A, s0);
                }
                if (++k == (uint32_t)WB || tile + 1 == t1) {
                    __syncthreads();
                    const uint64_t b0 = first * TILE;
                    const uint64_t m64 = (uint64_t)k * TILE < (uint64_t)n - b0 ? (uint64_t)k * TILE
                                                                              : (uint64_t)n - b0;
                    const uint32_t m = (uint32_t)m64;
                    for (uint32_t i = tid; i < m; i += 256) st_verdict<WT>(ft, out, b0 + i, vb[i]);
                    __syncthreads();
                    k = 0;
                    first = tile + 1;
                }
            }
            if (lds_bins) {
                __syncthreads();
                flush_hist();
            }
            return;
        }
    }
    uint64_t tile = blockIdx.x;
    group_frames<FPG, P> A;
    if (tile * TILE < n) {
        group_desc<G>(A, tile, n, grp, pkts, off, len, unit_log2, idx);
        group_load<G, FPG, P, NTL>(A, s0);
    }
    if constexpr (PIPE) {
        group_frames<FPG, P> B;
        group_desc<G>(B, tile + gridDim.x, n, grp, pkts, off, len, unit_log2, idx);
        for (; tile * TILE < n; tile += gridDim.x) {
            group_load<G, FPG, P, NTL>(B, s0); // no-op lanes past the end (cap 0)
            group_process<G, P, FPG, NTL, RI, WT, H16>(A, gl, gbase, s0, ft, out, counts, hist, lds_bins);
            A = B;
            group_desc<G>(B, tile + 2 * (uint64_t)gridDim.x, n, grp, pkts, off, len, unit_log2, idx);
        }
    } else {
        for (; tile * TILE < n; tile += gridDim.x) {
            group_process<G, P, FPG, NTL, RI, WT, H16>(A, gl, gbase, s0, ft, out, counts, hist, lds_bins);
            group_desc<G>(A, tile + gridDim.x, n, grp, pkts, off, len, unit_log2, idx);
            group_load<G, FPG, P, NTL>(A, s0);
        }
    }

    if (lds_bins) {
        __syncthreads();
        flush_hist();
    }
}

template <int G, int P, int FPG, int PIPE = 0, bool NTL = true, int RI = 0, int MINW = 1,
          bool WT = false, int WB = 0, bool H16 = false>
hipError_t launch_v(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                    uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out, unsigned long long *counts,
                    uint32_t lds_bins, hipStream_t s, const uint32_t *idx = nullptr,
                    const uint32_t *n_dev = nullptr) {
    static_assert(WB == 0 || PIPE == 0, "write batching: PIPE 0 only");
    constexpr uint32_t TILE = (256 / G) * FPG;
    const uint32_t hwords = H16 ? (lds_bins + 1u) / 2u : lds_bins;
    const size_t lds = (size_t)((hwords + 3u) & ~3u) * 4u + (size_t)WB * TILE * 16u;
    // resident blocks: one wave of blocks, equal shares, no tail
    int cu = 0, bpc = 0;
    hipError_t e = rx_occupancy(
        reinterpret_cast<const void *>(rx_classify_kernel<G, P, FPG, PIPE, NTL, RI, MINW, WT, WB, H16>), 256,
        lds, &cu, &bpc);
    if (e != hipSuccess) return e;
    const uint64_t tiles = ((uint64_t)n + TILE - 1) / TILE;
    uint64_t occ = (uint64_t)bpc;
    if (ft.bpc_cap && occ > ft.bpc_cap) occ = ft.bpc_cap;
    uint64_t blocks = (uint64_t)cu * occ;
    if (blocks > tiles) blocks = tiles;
    if (blocks == 0) blocks = 1;
    if constexpr (H16) {
        // a 16-bit bin holds at most 65535: every block's share of the burst
        // (index-list mode: n_dev may shorten it, never lengthen) stays below
        // that, else the 32-bit histogram
        if (lds_bins && ((tiles + blocks - 1) / blocks) * TILE > 65535u)
            return launch_v<G, P, FPG, PIPE, NTL, RI, MINW, WT, WB, false>(
                pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, s, idx, n_dev);
    }
    hipLaunchKernelGGL((rx_classify_kernel<G, P, FPG, PIPE, NTL, RI, MINW, WT, WB, H16>), dim3((uint32_t)blocks), dim3(256), lds, s,
                       pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, idx, n_dev);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// G = 1: one frame per lane.  For small frames (<= 64 B) the per-frame work
// (header decode, hash, probe, verdict) dominates the bytes, and a lane that
// owns a whole frame does it once instead of once per group lane.  The lane
// loads its first 64 B as four 16-B loads; longer frames continue in a
// per-lane loop (correct for any length, only efficient for small frames).
// Verdict stores are 16 B per lane, contiguous across the wave.
__device__ __forceinline__ uint32_t lane_chunk_sum(uint32_t acc, uint4 v, int32_t s, int32_t e) {
    if (s + 16 > e) v = chunk_below(v, s, e);
    acc = add_halves(acc, v.x);
    acc = add_halves(acc, v.y);
    acc = add_halves(acc, v.z);
    return add_halves(acc, v.w);
}

// Per-lane frame state between the load and the verdict.
struct lane_frame {
    uint64_t p;
    const uint8_t *fb;
    int32_t cap;
    bool valid;
    uint4 c[4];
};

// p = position in the burst (or in the index list idx, when given); L.p =
// the frame index the verdict belongs to
__device__ __forceinline__ void lane_desc(lane_frame &L, uint64_t p, uint32_t n,
                                          const uint8_t *__restrict__ pkts,
                                          const uint32_t *__restrict__ off,
                                          const uint16_t *__restrict__ len, uint32_t unit_log2,
                                          const uint32_t *__restrict__ idx = nullptr) {
    L.valid = p < n;
    const uint64_t pp = L.valid ? p : 0;
    const uint64_t q = idx ? (uint64_t)idx[pp] : pp;
    L.p = q;
    L.fb = pkts + ((uint64_t)off[q] << unit_log2);
    L.cap = L.valid ? (int32_t)len[q] : 0;
}

// lane_desc without an index list and without a branch around a load (PIPE
// 14: a branch here would make the compiler drain the prefetched frame bytes)
__device__ __forceinline__ void lane_desc_nb(lane_frame &L, uint64_t p, uint32_t n,
                                             const uint8_t *__restrict__ pkts,
                                             const uint32_t *__restrict__ off,
                                             const uint16_t *__restrict__ len, uint32_t unit_log2) {
    L.valid = p < n;
    const uint64_t q = L.valid ? p : 0;
    L.p = q;
    const uint32_t o = off[q];
    const uint32_t l = len[q];
    L.fb = pkts + ((uint64_t)o << unit_log2);
    L.cap = L.valid ? (int32_t)l : 0;
}

template <bool NTL>
__device__ __forceinline__ void lane_load(lane_frame &L) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        L.c[j] = make_uint4(0, 0, 0, 0);
        if (16 * j < L.cap) L.c[j] = ldg16<NTL>(L.fb + 16 * j);
    }
}

// The first 64 B of the wave's 64 frames when they sit in consecutive 64-B
// slots starting at b: stage64_load (rx_device.h), four coalesced 1-KiB loads
// through this wave's 4-KiB LDS stage, replacing four per-lane strided 16-B
// loads (64 distinct 64-B segments per instruction); bytes past a frame's
// caplen are masked later, as for lane_load.
__device__ __forceinline__ void lane_load_staged(lane_frame &L, const uint8_t *b, uint4 *st,
                                                 uint32_t lane) {
    stage64_load(b, st, lane, L.c);
}

// Pipelined form of lane_load_staged (PIPE 14): issue the four 16-B loads of
// L's first 64 B into v and return whether the wave's 64 frames sit in
// consecutive 64-B slots (wave-uniform).  Coalesced: lane l loads chunk
// q*64 + l of the wave's 4 KiB; otherwise lane l loads its own frame's chunk q
// (chunks past caplen read chunk 0 and are masked by lane_verdict).  No branch
// around the loads.
__device__ __forceinline__ bool lane_issue(const lane_frame &L, const uint8_t *pkts, uint32_t lane,
                                           uint4 (&v)[4]) {
    const uint64_t fpos = (uint64_t)(L.fb - pkts);
    const uint64_t f0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(fpos >> 32)) << 32) |
                        __builtin_amdgcn_readfirstlane((uint32_t)fpos);
    // (the 4 KiB must lie inside the buffer: slots 0..62 end where the next
    // frame starts, slot 63 only if its frame reaches past byte 48)
    const bool co =
        __ballot(L.valid && fpos == f0 + 64ull * lane && (lane != 63u || L.cap > 48)) == ~0ull;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint8_t *a = co ? pkts + f0 + 16u * (q * 64u + lane) : L.fb + (16 * q < L.cap ? 16 * q : 0);
        v[q] = ldg16<true>(a);
    }
    return co;
}

// Consume lane_issue's loads: through the wave's 4-KiB LDS stage, transposed
// (coalesced: the stage64_load layout) or in place (per-lane), into L.c
__device__ __forceinline__ void lane_stage(lane_frame &L, const uint4 (&v)[4], bool co, uint4 *st,
                                           uint32_t lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t k = q * 64u + lane, f = k >> 2;
        const uint32_t wc = f * 4u + (((k & 3u) + (f >> 2)) & 3u);
        const uint32_t wl = lane * 4u + ((q + (lane >> 2)) & 3u);
        st[co ? wc : wl] = v[q];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) L.c[k] = st[lane * 4u + ((k + (lane >> 2)) & 3u)];
    __builtin_amdgcn_wave_barrier();
}

// Parse + checksum + probe + verdict of one lane-owned frame.  `next` (may be
// null) is the following trip's frame: its loads are issued here, after the
// current frame's arithmetic and before the current frame's bucket probe, so
// the bulk bytes of trip t+1 are in flight across the probe latency of trip t.
// ABL (diagnostic builds only, never selected automatically): 1 = no bucket
// probe, 4 = no verdict store, 8 = no checksum arithmetic.
// Verdict of one lane-owned frame (everything but the store): returns the
// 16-B verdict and the per-flow count slot (~0u = not counted).
template <int ABL = 0, bool NTL = true, bool LDT = false>
__device__ __forceinline__ uint4 lane_verdict(lane_frame &L, lane_frame *next, const rx_ft_dev &ft,
                                              uint32_t *count_idx, const uint2 *lt = nullptr,
                                              const uint16_t *lw = nullptr) {
    const int32_t cp = L.cap;
    if (cp < 64) { // bytes past caplen read as 0 (rare: runts)
#pragma unroll
        for (int j = 0; j < 4; ++j) L.c[j] = chunk_below(L.c[j], 16 * j, cp);
    }
    const uint4 c0 = L.c[0], c1 = L.c[1], c2 = L.c[2], c3 = L.c[3];
    const uint32_t et = c0.w & 0xFFFFu;
    const uint32_t tl = rx_bswap16(c1.x & 0xFFFFu);
    const uint32_t proto = c1.y >> 24;
    const uint32_t sip = (c1.z >> 16) | (c1.w << 16);
    const uint32_t dip = (c1.w >> 16) | (c2.x << 16);
    const uint32_t sport = c2.x >> 16;
    const uint32_t dport = c2.y & 0xFFFFu;
    const uint32_t dgl = rx_bswap16(c2.y >> 16);
    const uint32_t hl = ((c2.w >> 16) & 0xFFu) >> 4;

    uint32_t cl, nd;
    if (et == 0x0608u) {
        cl = RXG_CLS_ARP;
        nd = 42;
    } else if (et != 0x0008u) {
        cl = RXG_CLS_NON_IP;
        nd = 14;
    } else if (proto == 17u) {
        cl = RXG_CLS_UDP;
        nd = 42;
    } else if (proto == 6u) {
        cl = RXG_CLS_TCP;
        nd = 54;
    } else {
        cl = RXG_CLS_IPV4_OTHER;
        nd = 24;
    }
    const bool is_udp = cl == RXG_CLS_UDP, is_tcp = cl == RXG_CLS_TCP;
    const bool l4 = is_udp || is_tcp;
    const uint32_t l4n = tl >= 20u ? tl - 20u : 0u;
    const bool do_sum = l4 && tl >= 20u;
    if (l4 && 34u + l4n > nd) nd = 34u + l4n;

    // checksum over [26, e), field at 40 (UDP) / 50 (TCP) read as 0
    int32_t e = do_sum ? 34 + (int32_t)l4n : 0;
    if (e > cp) e = cp;
    uint4 h1 = c1, h2 = c2, h3 = c3;
    h1.x = 0;
    h1.y = 0;
    h1.z &= 0xFFFF0000u;
    if (is_udp) h2.z &= 0xFFFF0000u;
    if (is_tcp) h3.x &= 0x0000FFFFu;
    uint32_t acc = 0;
    if (!(ABL & 8)) {
    acc = lane_chunk_sum(acc, h1, 16, e);
    acc = lane_chunk_sum(acc, h2, 32, e);
    acc = lane_chunk_sum(acc, h3, 48, e);
    }
    for (int32_t s = 64; s < e && !(ABL & 8); s += 64) { // longer frames: per-lane loop
        uint4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            r[u] = make_uint4(0, 0, 0, 0);
            if (s + 16 * u < e) r[u] = ldg16<NTL>(L.fb + s + 16 * u);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = lane_chunk_sum(acc, r[u], s + 16 * u, e);
    }
    uint32_t ck = 0;
    if (do_sum) {
        acc += proto << 8;
        acc += rx_bswap16(l4n);
        ck = (~fold16(acc)) & 0xFFFFu;
        if (ck == 0u && proto == 17u) ck = 0xFFFFu;
    }
    const uint32_t stored = is_udp ? (c2.z & 0xFFFFu) : (is_tcp ? (c3.x >> 16) : 0u);
    const bool ok = l4 && stored == ck;

    if (next) lane_load<NTL>(*next); // trip t+1 bytes in flight from here on

    // flow probe: the whole 64-B bucket per lane
    uint32_t flow = RXG_FLOW_NONE;
    const bool probe = L.valid && (is_udp || (is_tcp && ok));
    if (ABL & 1) {
        flow = probe ? (dport & 0x3FFu) : RXG_FLOW_NONE;
    } else if (LDT && probe && is_udp) { // compact UDP table in LDS
        const uint32_t k = rx_bswap16(dport) - ft.udpw_lo;
        // with a port window: on udp_dip the window holds every bound port
        // (outside it, no socket), elsewhere only the udpc_other keys can match
        const bool win = ft.udpw_n != 0u;
        if (win && dip == ft.udp_dip) { // the port window decides (one LDS read)
            const uint32_t e = k < ft.udpw_n ? lw[k] : 0xFFFFu;
            flow = e == 0xFFFFu ? RXG_FLOW_NONE : e;
        } else if (win && ft.udpc_other == 0u) {
            flow = RXG_FLOW_NONE;
        } else {
            uint32_t i = rx_hash3s(ft.hseed, dip, dport, 17u) & ft.udpc_mask;
            for (uint32_t pr = 0; pr < ft.udpc_probe; ++pr, i = (i + 1) & ft.udpc_mask) {
                const uint2 sl = lt[i];
                if (sl.y == 0xFFFFFFFFu) break;
                if (sl.x == dip && (sl.y & 0xFFFFu) == dport) {
                    flow = sl.y >> 16;
                    break;
                }
            }
        }
    } else if (probe) {
        const uint32_t ka = is_udp ? dip : sip;
        const uint32_t kb = is_udp ? dport : dip;
        const uint32_t kc = is_udp ? 17u : (sport | (dport << 16));
        const uint4 *tbl = is_udp ? ft.udp : ft.tcp;
        const uint32_t mask = is_udp ? ft.udp_mask : ft.tcp_mask;
        uint32_t maxp = is_udp ? ft.udp_probe : ft.tcp_probe;
        if (is_udp && ft.udp_port && rx_udp_port_decide(ft.udp_port[dport], dip, ft.udp_dip, &flow))
            maxp = 0; // decided by the direct port table
        uint32_t i = rx_hash3s(ft.hseed, ka, kb, kc) & mask;
        for (uint32_t pr = 0; pr < maxp; ++pr, i = (i + 1) & mask) { // ~1.2 trips expected
            const uint4 sl = ld_slot(tbl + i);
            if (sl.w == RX_SLOT_EMPTY) break;
            if (sl.x == ka && sl.y == kb && sl.z == kc) {
                flow = sl.w;
                break;
            }
        }
        if (is_tcp && flow == RXG_FLOW_NONE) flow = ft.listen[dport];
        // consume the listener load inside this branch: left pending, the merge
        // with the LDS-table path makes the compiler wait for every outstanding
        // load (vmcnt(0)) before the verdict, draining PIPE 14's prefetch
        asm volatile("" ::"v"(flow));
    }

    int32_t rc;
    uint32_t poff = 0, plen = 0, flags = 0;
    if (is_udp) {
        rc = flow == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                   : (dgl <= 8u ? RXG_RC_UDP_NOMEM : RXG_RC_OK);
        poff = 42;
        plen = dgl > 8u ? dgl - 8u : 0u;
        if (dgl <= 8u) flags |= RXG_F_UDP_SHORT;
        if (rc == RXG_RC_OK && 42u + plen > nd) nd = 42u + plen;
    } else if (is_tcp) {
        const int32_t pl = (int32_t)tl - 20 - 4 * (int32_t)hl;
        poff = 34u + 4u * hl;
        if (pl < 0) flags |= RXG_F_TCP_NEGLEN;
        plen = pl < 0 ? 0u : (uint32_t)pl;
        rc = !ok ? RXG_RC_TCP_BAD_CKSUM : (flow == RXG_FLOW_NONE ? RXG_RC_TCP_NO_TCB : RXG_RC_OK);
    } else {
        rc = RXG_RC_KNI;
    }
    if ((int32_t)nd > cp) flags |= RXG_F_TRUNC;
    uint4 v;
    v.x = flow;
    v.y = (poff & 0xFFFFu) | (plen << 16);
    v.z = ck | (cl << 16) | (((uint32_t)rc & 0xFFu) << 24);
    v.w = (ok ? 1u : 0u) | (flags << 8) | (stored << 16);
    *count_idx = (L.valid && rc == RXG_RC_OK && flow != RXG_FLOW_NONE)
                     ? (is_tcp ? ft.nu : 0u) + flow
                     : 0xFFFFFFFFu;
    return v;
}

// The common case of lane_verdict in straight-line code (LDS tables with a
// port window): every lane of the wave invalid, or not TCP, with its checksum
// span ending exactly at byte 64 when it has one, and, when UDP, decided by the
// port window (dip == udp_dip) or by the absence of other keys.  Returns false
// (wave-uniform) when some lane is not such a frame; the caller then runs
// lane_verdict, whose result for these lanes this one equals field by field
// (the same parse, class, checksum, probe and verdict rules, computed with
// selects: lane_verdict's nested per-lane branches cost about as many scalar
// mask instructions as vector ones, and the kernel is issue-bound once the
// bytes are in flight: profiles/r06aa).
__device__ __forceinline__ bool lane_verdict_fast(lane_frame &L, const rx_ft_dev &ft, uint4 *vout,
                                                  uint32_t *count_idx, const uint16_t *lw) {
    const int32_t cp = L.cap;
    if (cp < 64) { // bytes past caplen read as 0 (rare: runts)
#pragma unroll
        for (int j = 0; j < 4; ++j) L.c[j] = chunk_below(L.c[j], 16 * j, cp);
    }
    const uint4 c0 = L.c[0], c1 = L.c[1], c2 = L.c[2], c3 = L.c[3];
    const uint32_t et = c0.w & 0xFFFFu;
    const uint32_t tl = rx_bswap16(c1.x & 0xFFFFu);
    const uint32_t proto = c1.y >> 24;
    const uint32_t dip = (c1.w >> 16) | (c2.x << 16);
    const uint32_t dport = c2.y & 0xFFFFu;
    const uint32_t dgl = rx_bswap16(c2.y >> 16);
    const bool is_ip = et == 0x0008u, is_arp = et == 0x0608u;
    const bool is_udp = is_ip && proto == 17u, is_tcp = is_ip && proto == 6u;
    const uint32_t l4n = tl >= 20u ? tl - 20u : 0u;
    const bool do_sum = is_udp && tl >= 20u; // (no TCP lane on this path)
    const int32_t e = min(34 + (int32_t)l4n, cp);
    const bool win_key = dip == ft.udp_dip;
    const bool fast = !L.valid || (!is_tcp && (!do_sum || e == 64) &&
                                   (!is_udp || win_key || ft.udpc_other == 0u));
    if (ft.udpw_n == 0u || __ballot(!fast) != 0ull) return false; // wave-uniform

    const uint32_t cl = is_arp ? RXG_CLS_ARP
                               : (!is_ip ? RXG_CLS_NON_IP
                                         : (is_udp ? RXG_CLS_UDP : RXG_CLS_IPV4_OTHER));
    uint32_t nd = (is_arp || is_udp) ? 42u : (is_ip ? 24u : 14u);
    if (is_udp && 34u + l4n > nd) nd = 34u + l4n;
    // the checksum words [26, 64) in two independent chains (no dependent
    // v_dot2 back to back), field at 40 read as 0
    const uint32_t a0 = add_halves(add_halves(add_halves(0u, c1.z & 0xFFFF0000u), c2.x), c2.z & 0xFFFF0000u);
    const uint32_t a1 = add_halves(add_halves(add_halves(0u, c1.w), c2.y), c2.w);
    const uint32_t a2 = add_halves(add_halves(a0, c3.x), c3.z);
    const uint32_t a3 = add_halves(add_halves(a1, c3.y), c3.w);
    uint32_t ck = (~fold16(a2 + a3 + (proto << 8) + rx_bswap16(l4n))) & 0xFFFFu;
    if (ck == 0u) ck = 0xFFFFu; // UDP
    ck = do_sum ? ck : 0u;
    const uint32_t stored = is_udp ? (c2.z & 0xFFFFu) : 0u;
    const bool ok = is_udp && stored == ck;
    // the port window (one LDS read per lane, from entry 0 when not needed)
    const bool probe = L.valid && is_udp;
    const uint32_t k = rx_bswap16(dport) - ft.udpw_lo;
    const bool in_win = probe && win_key && k < ft.udpw_n;
    const uint32_t we = lw[in_win ? k : 0u];
    const uint32_t flow = (in_win && we != 0xFFFFu) ? we : RXG_FLOW_NONE;
    const int32_t rc = is_udp ? (flow == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                                       : (dgl <= 8u ? RXG_RC_UDP_NOMEM : RXG_RC_OK))
                              : RXG_RC_KNI;
    const uint32_t plen = (is_udp && dgl > 8u) ? dgl - 8u : 0u;
    if (rc == RXG_RC_OK && 42u + plen > nd) nd = 42u + plen;
    const uint32_t flags = ((is_udp && dgl <= 8u) ? RXG_F_UDP_SHORT : 0u) | ((int32_t)nd > cp ? RXG_F_TRUNC : 0u);
    uint4 v;
    v.x = flow;
    v.y = (is_udp ? 42u : 0u) | (plen << 16);
    v.z = ck | (cl << 16) | (((uint32_t)rc & 0xFFu) << 24);
    v.w = (ok ? 1u : 0u) | (flags << 8) | (stored << 16);
    *vout = v;
    *count_idx = (L.valid && rc == RXG_RC_OK && flow != RXG_FLOW_NONE) ? flow : 0xFFFFFFFFu;
    return true;
}

__device__ __forceinline__ void lane_count(uint32_t idx, unsigned long long *__restrict__ counts,
                                           uint32_t *hist, uint32_t lds_bins) {
    if (counts && idx != 0xFFFFFFFFu) {
        if (lds_bins)
            atomicAdd(&hist[idx], 1u);
        else
            atomicAdd(&counts[idx], 1ull);
    }
}

// The count indices of a wave's 64 consecutive frames (frame p = p0 + lane,
// p0 a multiple of 64; every lane active) stored as whole 16-B pieces: lane
// 8k (2-B indices) or 4k (4-B indices) gathers its neighbours' indices over
// DPP row shifts and stores them, non-temporally (the slab pass reads them
// from HBM anyway; in the L2 they would displace the flow table the SH
// kernel probes at the end of each block); the slab pass reads
// indices past n never, so the last wave's pieces may cover frames >= n (the
// index buffer has room for 4 B per frame, rounded to 256 B).
__device__ __forceinline__ void put_count_idx_wave(const rx_ft_dev &ft, uint64_t p, uint32_t idx,
                                                   uint32_t lane, uint32_t lim = 64) {
    if (!ft.count_idx) return;
    if (ft.count_ffff) count_ffff(ft, idx);
    if (ft.cidx16) {
        const uint32_t v = idx & 0xFFFFu;
        const uint32_t x1 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x101, 0xF, 0xF, false));
        const uint32_t x2 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x102, 0xF, 0xF, false));
        const uint32_t x3 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x103, 0xF, 0xF, false));
        const uint32_t x4 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x104, 0xF, 0xF, false));
        const uint32_t x5 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x105, 0xF, 0xF, false));
        const uint32_t x6 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x106, 0xF, 0xF, false));
        const uint32_t x7 = pin(__builtin_amdgcn_update_dpp(0u, v, 0x107, 0xF, 0xF, false));
        if ((lane & 7u) == 0u && lane < lim) {
            const rx_u32x4 w = {v | (x1 << 16), x2 | (x3 << 16), x4 | (x5 << 16), x6 | (x7 << 16)};
            st_stream16(reinterpret_cast<rx_u32x4 *>(static_cast<uint16_t *>(ft.count_idx) + p), w);
        }
    } else {
        const uint32_t x1 = pin(__builtin_amdgcn_update_dpp(0u, idx, 0x101, 0xF, 0xF, false));
        const uint32_t x2 = pin(__builtin_amdgcn_update_dpp(0u, idx, 0x102, 0xF, 0xF, false));
        const uint32_t x3 = pin(__builtin_amdgcn_update_dpp(0u, idx, 0x103, 0xF, 0xF, false));
        if ((lane & 3u) == 0u && lane < lim) {
            const rx_u32x4 w = {idx, x1, x2, x3};
            st_stream16(reinterpret_cast<rx_u32x4 *>(static_cast<uint32_t *>(ft.count_idx) + p), w);
        }
    }
}

template <bool ST_NT>
__device__ __forceinline__ void lane_store(const rx_ft_dev &ft, uint4 *__restrict__ out, uint64_t p,
                                           uint4 v) {
    st_verdict<false, !ST_NT>(ft, out, p, v);
}

// the original one-shot form: verdict, store, count
// the store and count half of lane_process (PIPE 23 defers it to the trip's end)
template <int ABL = 0, bool ST_NT = true>
__device__ __forceinline__ void lane_finish(const lane_frame &L, uint4 v, uint32_t idx,
                                            const rx_ft_dev &ft, uint4 *__restrict__ out,
                                            unsigned long long *__restrict__ counts, uint32_t *hist,
                                            uint32_t lds_bins) {
    if (L.valid) {
        if (ABL & 4)
            asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
        else
            lane_store<ST_NT>(ft, out, L.p, v);
        lane_count(idx, counts, hist, lds_bins);
        if (ft.count_idx) put_count_idx(ft, L.p, idx);
    }
}

// LEAN (PIPE 16): lane_verdict_fast first, lane_verdict for the waves it declines
template <int ABL = 0, bool ST_NT = true, bool NTL = true, bool LDT = false, bool LEAN = false>
__device__ __forceinline__ void lane_process(lane_frame &L, lane_frame *next,
                                             const rx_ft_dev &ft, uint4 *__restrict__ out,
                                             unsigned long long *__restrict__ counts,
                                             uint32_t *hist, uint32_t lds_bins,
                                             const uint2 *lt = nullptr, const uint16_t *lw = nullptr) {
    uint32_t idx;
    uint4 v;
    if (!(LEAN && LDT && (ABL & ~4) == 0 && lane_verdict_fast(L, ft, &v, &idx, lw)))
        v = lane_verdict<ABL, NTL, LDT>(L, next, ft, &idx, lt, lw);
    if (L.valid) {
        if (ABL & 4)
            asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
        else
            lane_store<ST_NT>(ft, out, L.p, v);
        lane_count(idx, counts, hist, lds_bins);
        if (ft.count_idx) put_count_idx(ft, L.p, idx);
    }
}

// PIPE = 0: load, process, repeat.  PIPE = 1: trip t+1's descriptors are
// fetched at the top of trip t and its frame bytes are issued mid-trip.
// PIPE = 2: as 1, register budget capped for 6 waves per SIMD.  PIPE = 3:
// only the descriptors are prefetched (frame bytes loaded at the top).
// LDT: the compact UDP table (ft.udpc) is copied into LDS after the histogram
// and UDP frames probe it there (PIPE 0 only)
template <int PIPE, int ABL = 0, bool ST_NT = true, bool NTL = true, bool LDT = false>
__global__ __launch_bounds__(256, PIPE == 2 ? 6 : 1) void rx_classify_lane_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t n, uint32_t unit_log2, rx_ft_dev ft,
    uint4 *__restrict__ out, unsigned long long *__restrict__ counts, uint32_t lds_bins,
    const uint32_t *__restrict__ idx, const uint32_t *__restrict__ n_dev) {
    static_assert(!LDT || PIPE == 0 || PIPE == 12 || PIPE == 14 || PIPE == 16 || PIPE == 18 ||
                      PIPE == 19 || (PIPE >= 21 && PIPE <= 25),
                  "LDS table: PIPE 0 / 12 / 14 / 16 / 18 / 19 / 21-25 only");
    constexpr bool LEAN = PIPE == 16 || PIPE == 18; // with lane_verdict_fast
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    uint2 *lt = reinterpret_cast<uint2 *>(hist + ((lds_bins + 3u) & ~3u));
    // the port window after the compact table, then (PIPE 12/14/15) the stage
    uint16_t *lw = reinterpret_cast<uint16_t *>(lt + (LDT ? ft.udpc_mask + 1u : 0u));
    const uint32_t lw_words = LDT ? ((ft.udpw_n + 7u) & ~7u) / 2u : 0u; // 16-B multiple
    if (n_dev) n = min(n, *n_dev); // index-list mode: the list length lives on the device
    const uint32_t tid = threadIdx.x;
    if constexpr (LDT) {
        const uint32_t q = (ft.udpc_mask + 1) / 2; // 16-B pieces
        for (uint32_t i = tid; i < q; i += 256)
            reinterpret_cast<uint4 *>(lt)[i] = reinterpret_cast<const uint4 *>(ft.udpc)[i];
        for (uint32_t i = tid; i < ft.udpw_n; i += 256) lw[i] = ft.udpw[i];
    }
    if (lds_bins) {
        for (uint32_t i = tid; i < lds_bins; i += 256) hist[i] = 0;
    }
    if (LDT || lds_bins) __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t p = (uint64_t)blockIdx.x * 256 + tid;
    if constexpr (PIPE == 9) {
        // issue order per trip t: frame(t) loads, descriptors(t+1), the
        // deferred verdict store of t-1, then wait for frame(t) only.  The
        // store ack and descriptor latency overlap the frame latency; the
        // probe loop's waits drain everything before the next trip.
        uint64_t base = (uint64_t)blockIdx.x * 256;
        lane_frame L;
        if (base < n) lane_desc(L, p, n, pkts, off, len, unit_log2);
        uint4 pend = make_uint4(0, 0, 0, 0);
        uint64_t pend_p = 0;
        bool pend_valid = false;
        for (; base < n; base += stride, p += stride) {
            lane_load<NTL>(L);
            const uint64_t np = p + stride;
            const bool nvalid = np < n;
            const uint64_t nq = nvalid ? np : 0;
            const uint32_t noff = off[nq];
            const uint16_t nlen = len[nq];
            if (pend_valid) lane_store<ST_NT>(ft, out, pend_p, pend);
            uint32_t idx;
            pend = lane_verdict<ABL, NTL>(L, nullptr, ft, &idx);
            pend_p = L.p;
            pend_valid = L.valid;
            lane_count(idx, counts, hist, lds_bins);
            if (ft.count_idx && L.valid) put_count_idx(ft, L.p, idx);
            L.p = np;
            L.valid = nvalid;
            L.fb = pkts + ((uint64_t)noff << unit_log2);
            L.cap = nvalid ? (int32_t)nlen : 0;
        }
        if (pend_valid) lane_store<ST_NT>(ft, out, pend_p, pend);
    } else if constexpr (PIPE == 0) {
        for (uint64_t base = (uint64_t)blockIdx.x * 256; base < n; base += stride, p += stride) {
            lane_frame L;
            lane_desc(L, p, n, pkts, off, len, unit_log2, idx);
            lane_load<NTL>(L);
            lane_process<ABL, ST_NT, NTL, LDT>(L, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
        }
    } else if constexpr (PIPE == 12) {
        // as 0, but a wave whose 64 frames fill consecutive 64-B slots loads
        // them coalesced through its LDS stage (lane_load_staged)
        uint4 *stage = reinterpret_cast<uint4 *>(hist + ((lds_bins + 3u) & ~3u) +
                                                 (LDT ? 2u * (ft.udpc_mask + 1u) + lw_words : 0u)) +
                       (tid >> 6) * 256u;
        const uint32_t lane = tid & 63u;
        for (uint64_t base = (uint64_t)blockIdx.x * 256; base < n; base += stride, p += stride) {
            lane_frame L;
            lane_desc(L, p, n, pkts, off, len, unit_log2, idx);
            const uint64_t fpos = (uint64_t)(L.fb - pkts);
            const uint64_t f0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(fpos >> 32)) << 32) |
                                __builtin_amdgcn_readfirstlane((uint32_t)fpos);
            // (the 4 KiB must lie inside the buffer: slots 0..62 end where the
            // next frame starts, slot 63 only if its frame reaches past byte 48)
            if (__ballot(L.valid && fpos == f0 + 64ull * lane && (lane != 63u || L.cap > 48)) ==
                ~0ull) // wave-uniform
                lane_load_staged(L, pkts + f0, stage, lane);
            else
                lane_load<NTL>(L);
            lane_process<ABL, ST_NT, NTL, LDT>(L, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
        }
    } else if constexpr (PIPE == 14 || PIPE == 16) {
        // 12, software-pipelined: descriptors two trips ahead, frame bytes one
        // trip ahead (issued before the current trip is staged and processed),
        // so a wave keeps its next 4 KiB in flight across its parse / probe /
        // store instead of waiting descriptor -> frame latency every trip.
        // Loads are never under a branch (the last trip's prefetch reads the
        // clamped frame 0 and is dropped): the coalesced-or-per-lane choice is
        // an address select and a staging-index select (lane_issue /
        // lane_stage), so the wait counts stay partial.  Three descriptor
        // sets x two frame-byte sets rotate with period 6, unrolled so no
        // register moves are needed (a move would wait for the load it
        // copies).
        uint4 *stage = reinterpret_cast<uint4 *>(hist + ((lds_bins + 3u) & ~3u) +
                                                 (LDT ? 2u * (ft.udpc_mask + 1u) + lw_words : 0u)) +
                       (tid >> 6) * 256u;
        const uint32_t lane = tid & 63u;
        uint64_t base = (uint64_t)blockIdx.x * 256;
        if (base < n) {
            lane_frame A, B, D;
            uint4 va[4], vb[4];
            lane_desc_nb(A, p, n, pkts, off, len, unit_log2);
            lane_desc_nb(B, p + stride, n, pkts, off, len, unit_log2);
            bool ca = lane_issue(A, pkts, lane, va), cb = false;
            for (;;) {
                // trip t = A (bytes in va), t+1 = B (descriptors), t+2 -> D
                lane_desc_nb(D, p + 2 * stride, n, pkts, off, len, unit_log2);
                cb = lane_issue(B, pkts, lane, vb);
                lane_stage(A, va, ca, stage, lane);
                lane_process<ABL, ST_NT, NTL, LDT, LEAN>(A, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                base += stride;
                p += stride;
                if (base >= n) break;
                // trip t = B (bytes in vb), t+1 = D, t+2 -> A
                lane_desc_nb(A, p + 2 * stride, n, pkts, off, len, unit_log2);
                ca = lane_issue(D, pkts, lane, va);
                lane_stage(B, vb, cb, stage, lane);
                lane_process<ABL, ST_NT, NTL, LDT, LEAN>(B, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                base += stride;
                p += stride;
                if (base >= n) break;
                // trip t = D (bytes in va), t+1 = A, t+2 -> B
                lane_desc_nb(B, p + 2 * stride, n, pkts, off, len, unit_log2);
                cb = lane_issue(A, pkts, lane, vb);
                lane_stage(D, va, ca, stage, lane);
                lane_process<ABL, ST_NT, NTL, LDT, LEAN>(D, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                base += stride;
                p += stride;
                if (base >= n) break;
                // trip t = A (bytes in vb), t+1 = B, t+2 -> D
                lane_desc_nb(D, p + 2 * stride, n, pkts, off, len, unit_log2);
                ca = lane_issue(B, pkts, lane, va);
                lane_stage(A, vb, cb, stage, lane);
                lane_process<ABL, ST_NT, NTL, LDT, LEAN>(A, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                base += stride;
                p += stride;
                if (base >= n) break;
                // trip t = B (bytes in va), t+1 = D, t+2 -> A
                lane_desc_nb(A, p + 2 * stride, n, pkts, off, len, unit_log2);
                cb = lane_issue(D, pkts, lane, vb);
                lane_stage(B, va, ca, stage, lane);
                lane_process<ABL, ST_NT, NTL, LDT, LEAN>(B, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                base += stride;
                p += stride;
                if (base >= n) break;
                // trip t = D (bytes in vb), t+1 = A, t+2 -> B
                lane_desc_nb(B, p + 2 * stride, n, pkts, off, len, unit_log2);
                ca = lane_issue(A, pkts, lane, va);
                lane_stage(D, vb, cb, stage, lane);
                lane_process<ABL, ST_NT, NTL, LDT, LEAN>(D, nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                base += stride;
                p += stride;
                if (base >= n) break;
                // back at the head's roles: A (bytes in va), B descriptors.  B's
                // descriptor loads are waited for here, where the count of later
                // loads is exact; left pending across the back edge, the loop
                // head's merged state made the compiler wait for everything
                // (vmcnt(0), draining va) once per 6 trips
                asm volatile("" ::"v"(B.cap), "v"(B.fb));
            }
        }
    } else if constexpr (PIPE == 18 || PIPE == 19 || PIPE == 21 || PIPE == 22 || PIPE == 23 ||
                         PIPE == 24 || PIPE == 25) {
        // T adjacent 256-frame tiles per trip, the shape of the byte-pattern
        // ceiling (tools/membw_cfg2, RDW U=2): every tile's frame bytes are
        // issued at the top of the trip (T x 4 KiB per wave), then the next
        // trip's descriptors; the tiles are staged, classified and stored in
        // turn.  Descriptors one trip ahead, so the frame loads never wait
        // for them.  Two descriptor sets swap roles (unrolled twice, no
        // register moves).  T = 2: 18 (with lane_verdict_fast) and 19; T = 3:
        // 21; T = 4: 22
        constexpr int T = PIPE == 21 ? 3 : (PIPE == 22 ? 4 : 2);
        // the trip's tiles: adjacent (every pipe but 25) or a grid stride apart (25)
        uint4 *stage = reinterpret_cast<uint4 *>(hist + ((lds_bins + 3u) & ~3u) +
                                                 (LDT ? 2u * (ft.udpc_mask + 1u) + lw_words : 0u)) +
                       (tid >> 6) * 256u;
        const uint32_t lane = tid & 63u;
        const uint64_t strideT = (uint64_t)T * stride;
        const uint64_t TO = PIPE == 25 ? stride : 256u;
        uint64_t base = (uint64_t)blockIdx.x * (PIPE == 25 ? 256u : 256u * T);
        uint64_t q = base + tid;
        if (base < n) {
            lane_frame A[T], B[T];
#pragma unroll
            for (int u = 0; u < T; ++u) lane_desc_nb(A[u], q + TO * u, n, pkts, off, len, unit_log2);
            auto trip = [&](lane_frame (&X)[T], lane_frame (&Y)[T]) {
                uint4 v[T][4];
                bool c[T];
                if constexpr (PIPE == 24) { // the next trip's descriptors first
#pragma unroll
                    for (int u = 0; u < T; ++u)
                        lane_desc_nb(Y[u], q + strideT + TO * u, n, pkts, off, len, unit_log2);
                }
#pragma unroll
                for (int u = 0; u < T; ++u) c[u] = lane_issue(X[u], pkts, lane, v[u]);
                if constexpr (PIPE != 24) {
#pragma unroll
                    for (int u = 0; u < T; ++u)
                        lane_desc_nb(Y[u], q + strideT + TO * u, n, pkts, off, len, unit_log2);
                }
                if constexpr (PIPE == 23) { // every tile's verdict first, the stores at the end
                    uint4 vd[T];
                    uint32_t ix[T];
#pragma unroll
                    for (int u = 0; u < T; ++u) {
                        lane_stage(X[u], v[u], c[u], stage, lane);
                        vd[u] = lane_verdict<ABL, NTL, LDT>(X[u], nullptr, ft, &ix[u], lt, lw);
                    }
#pragma unroll
                    for (int u = 0; u < T; ++u)
                        lane_finish<ABL, ST_NT>(X[u], vd[u], ix[u], ft, out, counts, hist, lds_bins);
                } else {
#pragma unroll
                    for (int u = 0; u < T; ++u) {
                        lane_stage(X[u], v[u], c[u], stage, lane);
                        lane_process<ABL, ST_NT, NTL, LDT, LEAN>(X[u], nullptr, ft, out, counts, hist, lds_bins, lt, lw);
                    }
                }
            };
            for (;;) {
                trip(A, B);
                base += strideT;
                q += strideT;
                if (base >= n) break;
                trip(B, A);
                base += strideT;
                q += strideT;
                if (base >= n) break;
                // A's descriptor loads waited for here, where the count of
                // later loads is exact (as in pipe 14)
#pragma unroll
                for (int u = 0; u < T; ++u) asm volatile("" ::"v"(A[u].cap), "v"(A[u].fb));
            }
        }
    } else if constexpr (PIPE == 3) {
        lane_frame L;
        uint64_t base = (uint64_t)blockIdx.x * 256;
        uint64_t nq = 0;
        const uint8_t *nfb = pkts;
        int32_t ncap = 0;
        if (base < n) {
            lane_desc(L, p, n, pkts, off, len, unit_log2);
            nfb = L.fb;
            ncap = L.cap;
        }
        for (; base < n; base += stride, p += stride) {
            L.p = p;
            L.valid = p < n;
            L.fb = nfb;
            L.cap = ncap;
            lane_load<NTL>(L);
            nq = p + stride; // descriptors of the next trip, in flight during this one
            const uint64_t q = nq < n ? nq : 0;
            nfb = pkts + ((uint64_t)off[q] << unit_log2);
            ncap = nq < n ? (int32_t)len[q] : 0;
            lane_process<0, ST_NT, NTL>(L, nullptr, ft, out, counts, hist, lds_bins);
        }
    } else {
        lane_frame A, B;
        uint64_t base = (uint64_t)blockIdx.x * 256;
        if (base < n) {
            lane_desc(A, p, n, pkts, off, len, unit_log2);
            lane_load<NTL>(A);
        }
        // two frames alternate roles; the loop body is unrolled twice so that
        // A and B stay in fixed registers
        while (base < n) {
            uint64_t nb = base + stride;
            lane_desc(B, p + stride, n, pkts, off, len, unit_log2);
            lane_process<0, ST_NT, NTL>(A, nb < n ? &B : nullptr, ft, out, counts, hist, lds_bins);
            base = nb;
            p += stride;
            if (base >= n) break;
            nb = base + stride;
            lane_desc(A, p + stride, n, pkts, off, len, unit_log2);
            lane_process<0, ST_NT, NTL>(B, nb < n ? &A : nullptr, ft, out, counts, hist, lds_bins);
            base = nb;
            p += stride;
        }
    }
    if (lds_bins) {
        __syncthreads();
        for (uint32_t i = tid; i < lds_bins; i += 256) {
            const uint32_t cnt = hist[i];
            if (cnt) atomicAdd(&counts[i], (unsigned long long)cnt);
        }
    }
}

template <int PIPE, int ABL = 0, bool ST_NT = true, bool NTL = true, bool LDT = false>
hipError_t launch_lane(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                       uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out,
                       unsigned long long *counts, uint32_t lds_bins, hipStream_t s,
                       const uint32_t *idx = nullptr, const uint32_t *n_dev = nullptr) {
    if ((PIPE == 14 || PIPE >= 16) && idx) return hipErrorInvalidValue; // no index-list mode
    const size_t lds = (size_t)((lds_bins + 3u) & ~3u) * 4u +
                       (LDT ? (size_t)(ft.udpc_mask + 1) * 8u + ((ft.udpw_n + 7u) & ~7u) * 2u : 0u) +
                       (PIPE == 12 || PIPE == 14 || PIPE >= 16 ? 16384u : 0u);
    int cu = 0, bpc = 0;
    hipError_t e = rx_occupancy(
        reinterpret_cast<const void *>(rx_classify_lane_kernel<PIPE, ABL, ST_NT, NTL, LDT>), 256,
        lds, &cu, &bpc);
    if (e != hipSuccess) return e;
    const uint64_t tiles = ((uint64_t)n + 255) / 256;
    uint64_t occ = (uint64_t)bpc;
    if (ft.bpc_cap && occ > ft.bpc_cap) occ = ft.bpc_cap;
    uint64_t blocks = (uint64_t)cu * occ;
    if (blocks > tiles) blocks = tiles;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL((rx_classify_lane_kernel<PIPE, ABL, ST_NT, NTL, LDT>), dim3((uint32_t)blocks), dim3(256), lds, s,
                       pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, idx, n_dev);
    return hipGetLastError();
}


// the LDS-table instantiation when the flow set has a compact UDP table
template <int PIPE, int ABL = 0, bool ST_NT = true, bool NTL = true>
hipError_t launch_lane_udpc(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                            uint32_t n, uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out,
                            unsigned long long *counts, uint32_t lds_bins, hipStream_t s,
                            const uint32_t *idx = nullptr, const uint32_t *n_dev = nullptr) {
    if (ft.udpc)
        return launch_lane<PIPE, ABL, ST_NT, NTL, true>(pkts, off, len, n, unit_log2, ft, out,
                                                         counts, lds_bins, s, idx, n_dev);
    return launch_lane<PIPE, ABL, ST_NT, NTL, false>(pkts, off, len, n, unit_log2, ft, out, counts,
                                                      lds_bins, s, idx, n_dev);
}

// ---------------------------------------------------------------------------
// Size-class binning for mixed-size bursts (IMIX): frame indices split into a
// small list (len <= thresh) and a large list, so each list runs on the
// kernel shape that suits it.  Block b owns the contiguous chunk
// [b*chunk, (b+1)*chunk): pass 1 counts its classes, one atomic per class
// per block reserves output ranges, pass 2 (len re-read from L2) writes the
// indices in order.  Lists: small at lists[0..), large at lists[n..) (2n
// slots); lens[0] = small count, lens[1] = large count.
__global__ __launch_bounds__(256) void rx_bin_kernel(const uint16_t *__restrict__ len, uint32_t n,
                                                     uint32_t chunk, uint32_t thresh,
                                                     uint32_t *__restrict__ lists,
                                                     uint32_t *__restrict__ lens) {
    __shared__ uint32_t wsum[2][4];
    __shared__ uint32_t base[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t c0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t c1 = min((uint64_t)n, c0 + chunk);
    uint32_t my_small = 0, my_large = 0;
    for (uint64_t i = c0 + tid; i < c1; i += 256) {
        const bool sm = len[i] <= thresh;
        my_small += sm;
        my_large += !sm;
    }
    // block totals
    for (int o = 32; o > 0; o >>= 1) {
        my_small += __shfl_xor(my_small, o);
        my_large += __shfl_xor(my_large, o);
    }
    if (lane == 0) {
        wsum[0][wave] = my_small;
        wsum[1][wave] = my_large;
    }
    __syncthreads();
    if (tid == 0) {
        const uint32_t ts = wsum[0][0] + wsum[0][1] + wsum[0][2] + wsum[0][3];
        const uint32_t tl = wsum[1][0] + wsum[1][1] + wsum[1][2] + wsum[1][3];
        base[0] = ts ? atomicAdd(&lens[0], ts) : 0;
        base[1] = tl ? n + atomicAdd(&lens[1], tl) : 0; // large list: lists[n ...]
    }
    __syncthreads();
    uint32_t run_s = base[0], run_l = base[1];
    for (uint64_t t0 = c0; t0 < c1; t0 += 256) {
        const uint64_t i = t0 + tid;
        const bool v = i < c1;
        const bool sm = v && len[i] <= thresh;
        const bool lg = v && !sm;
        const uint64_t ms = __ballot(sm), ml = __ballot(lg);
        const uint64_t below = (1ull << lane) - 1ull;
        if (lane == 0) {
            wsum[0][wave] = __popcll(ms);
            wsum[1][wave] = __popcll(ml);
        }
        __syncthreads();
        uint32_t ps = run_s, pl = run_l;
        for (uint32_t w = 0; w < wave; ++w) {
            ps += wsum[0][w];
            pl += wsum[1][w];
        }
        if (sm) lists[ps + __popcll(ms & below)] = (uint32_t)i;
        if (lg) lists[pl + __popcll(ml & below)] = (uint32_t)i;
        for (uint32_t w = 0; w < 4; ++w) {
            run_s += wsum[0][w];
            run_l += wsum[1][w];
        }
        __syncthreads();
    }
}

// binned path: bin, then the lane kernel over the small list and the G=8
// kernel over the large list (both read frame indices through the list)
static hipError_t launch_binned(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                                uint32_t n, uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out,
                                unsigned long long *counts, uint32_t lds_bins, hipStream_t s,
                                uint32_t *ws) {
    if (!ws) return hipErrorInvalidValue;
    uint32_t *lens = ws, *lists = ws + 4;
    hipError_t e = hipMemsetAsync(lens, 0, 16, s);
    if (e != hipSuccess) return e;
    const uint32_t chunk = 16384;
    const uint32_t blocks = (uint32_t)(((uint64_t)n + chunk - 1) / chunk);
    hipLaunchKernelGGL(rx_bin_kernel, dim3(blocks), dim3(256), 0, s, len, n, chunk, 64u, lists,
                       lens);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    rx_ft_dev fl = ft;
    if (!fl.bpc_cap) fl.bpc_cap = 6;
    e = launch_lane_udpc<0, 0, true, false>(pkts, off, len, n, unit_log2, fl, out, counts, lds_bins, s,
                                        lists, lens);
    if (e != hipSuccess) return e;
    return launch_v<8, 2, 1, 1>(pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, s,
                                lists + n, lens + 1);
}

// ---------------------------------------------------------------------------
// Stream kernel: frame heads lane-owned, frame tails streamed by the block.
//   A block takes 256 consecutive frames, one per thread.  Head phase: thread
//   t loads its descriptor and its frame's first 64 B, decodes, sums the
//   checksum words of [26, min(e, 64)) (e = checksum end) and probes the flow
//   table (speculatively for TCP: a bad checksum discards the hit, as the
//   reference never looks one up).  Tail phase: the block streams the byte span
//   that covers every frame's full tail chunks [64, e & ~15) as contiguous 16-B
//   chunks (each wave instruction loads 1 KiB of consecutive bytes whatever
//   the frame sizes), forms the exclusive prefix sum E(c) of the per-chunk word
//   sums tile by tile (DPP wave scans + 16 wave totals through LDS), and each
//   frame takes E(ce) - E(cs) from the tiles holding its boundary chunks, plus
//   its last partial chunk loaded and masked by its own thread.  Prefix
//   differences are exact mod 2^32 and a frame's tail sum is < 2^32, so bytes
//   between frames cost bandwidth only, never correctness.  A block whose span
//   is far larger than its tails (frames scattered over the buffer) falls back
//   to per-thread tail loops: correct for any layout, fast for ordered ones
//   (packed bursts, fixed slots).

// inclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true); // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true); // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true); // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true); // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1,3
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2,3
    return x;
}

// N independent inclusive scans, step-interleaved: each DPP step of one
// row reads a register the previous VALU op did not write, so the DPP
// read-after-write wait states (s_nop) of a single scan disappear
template <int N>
__device__ __forceinline__ void wave_incl_scan_n(uint32_t (&x)[N]) {
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += __builtin_amdgcn_update_dpp(0u, x[j], 0x111, 0xF, 0xF, true);
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += __builtin_amdgcn_update_dpp(0u, x[j], 0x112, 0xF, 0xF, true);
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += __builtin_amdgcn_update_dpp(0u, x[j], 0x114, 0xF, 0xF, true);
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += __builtin_amdgcn_update_dpp(0u, x[j], 0x118, 0xF, 0xF, true);
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += __builtin_amdgcn_update_dpp(0u, x[j], 0x142, 0xA, 0xF, false);
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += __builtin_amdgcn_update_dpp(0u, x[j], 0x143, 0xC, 0xF, false);
}

// One wave's share of the block span: the min of a and the max of b over the
// lanes with `has`, and the sum of b - a, reduced across the wave first so
// that one lane issues three LDS atomics.  (64 lanes of one wave atomically
// updating the same three LDS words serialise: 192 conflicting LDS atomics
// per wave, per 256-frame tile.)  Every lane of the wave must be active.
__device__ __forceinline__ void span_add(bool has, uint64_t a, uint64_t b, unsigned long long *lo,
                                         unsigned long long *hi, uint32_t *tail, uint32_t lane) {
    unsigned long long mn = has ? a : ~0ull, mx = has ? b : 0ull;
    uint32_t sm = has ? (uint32_t)(b - a) : 0u;
    const bool any = __ballot(has) != 0ull;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long omn = __shfl_xor(mn, o), omx = __shfl_xor(mx, o);
        mn = omn < mn ? omn : mn;
        mx = omx > mx ? omx : mx;
        sm += __shfl_xor(sm, o);
    }
    if (lane == 0 && any) {
        atomicMin(lo, mn);
        atomicMax(hi, mx);
        atomicAdd(tail, sm);
    }
}

__device__ __forceinline__ uint32_t chunk_sum(uint4 v) {
    return add_halves(add_halves(add_halves(add_halves(0u, v.x), v.y), v.z), v.w);
}

// Every load below is issued unconditionally (out-of-range lanes load a
// clamped, valid address and select zero) so that the compiler's wait counts
// stay partial: a lane-dependent branch around a load makes it drain every
// outstanding load (vmcnt(0)), which would serialise the tile prefetch.
// ABL (diagnostic builds only, never selected automatically): 1 = no flow
// table probe (flow id from the port: wrong verdicts by construction)
// HO (issue order of the first tile against the flow probe): 0 = probe, then
// the first tile's loads; 1 = the first tile's loads, then the probe (its
// dependent slot reads overlap the tile in flight); 2 = the probe and the
// verdict fields after the whole tail stream (the slot read's latency hides
// behind the stream; the key words stay live across it); 3 = 2 at a register
// budget for 5 resident blocks per CU instead of 6 (2 spills one VGPR at 6).
// PW (first probe window): 1 = one slot; 2 = the home slot and the next one in
// the same trip (the table keeps a mirror of slot 0 past its end), so a key
// displaced by one slot costs no dependent second read.  B1: one barrier per
// tail tile instead of two (a tile's boundary prefixes are read after the next
// tile's barrier, which already orders them after their writes; s_pre and
// s_wt are double-buffered, so the next writes to a buffer come a barrier
// after its last reads)
// FPB: frames per block (256, or 128 / 64 / 32 / 16 with the other threads
// streaming only: shorter blocks for jumbo frames, whose 256-frame blocks
// stream 2.3 MB each and leave the last round of blocks a fraction of the chip)
// L: 16-B chunks per thread per tail tile (4: 16-KiB tiles)
template <bool NTS, int ABL = 0, int HO = 0, int PW = 1, bool B1 = false, bool DS = false,
          bool HG = false, uint32_t FPB = 256, int L = 4, bool WT = false>
__global__ __launch_bounds__(256, HO == 3 ? 5 : 6) void rx_classify_stream_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t n, uint32_t unit_log2, rx_ft_dev ft,
    uint4 *__restrict__ out, unsigned long long *__restrict__ counts, uint32_t lds_bins) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    constexpr uint32_t LPT = L;          // 16-B chunks per thread per tail tile
    constexpr uint32_t TCH = 256u * LPT; // chunks per tail tile
    __shared__ __attribute__((aligned(16))) uint32_t s_pre[2][TCH];
    __shared__ __attribute__((aligned(16))) uint32_t s_wt[2][4 * LPT]; // [row j][wave w]
    __shared__ unsigned long long s_lo, s_hi;
    __shared__ uint32_t s_tail;
    // HG: heads gathered four lanes per head (head_gather_issue), transposed
    // through a 4-KiB stage per wave
    __shared__ __attribute__((aligned(16))) uint4 s_head[HG ? 4 : 1][HG ? 256 : 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t wvu = __builtin_amdgcn_readfirstlane(wv); // wave-uniform: SALU selects
    uint4 *hstage = &s_head[HG ? wv : 0][0];
    if (tid == 0) {
        s_lo = ~0ull;
        s_hi = 0;
        s_tail = 0;
    }
    for (uint32_t i = tid; i < lds_bins; i += 256) hist[i] = 0;

    // one 256-frame tile per block.  (A resident grid looping over tiles, with
    // or without the next tile's heads prefetched, measured slower: r02e,
    // r02q.  With a tile loop here the compiler kept the span re-arm constants
    // in a scratch spill written once per thread, 16 B of HBM writes per
    // frame: PMC r02g.)
    {
        const uint64_t tile = blockIdx.x;
        static_assert(FPB == 256 || FPB == 128 || FPB == 64 || FPB == 32 || FPB == 16,
                      "frames per block");
        const uint64_t p = tile * FPB + tid;
        const bool valid = tid < FPB && p < n;
        const uint64_t q = valid ? p : 0;
        const uint64_t fpos = (uint64_t)off[q] << unit_log2;
        const uint8_t *fb = pkts + fpos;
        const int32_t cp = valid ? (int32_t)len[q] : 0;

        // ---- head phase -------------------------------------------------------
        uint4 c[4];
        if constexpr (HG && !(ABL & 4)) {
            uint4 hv[4];
            head_gather_issue(pkts, fpos, cp, lane, hv);
            head_gather_stage(hstage, lane, hv, c);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                c[j] = (ABL & 4) ? make_uint4(0, 0, 0, 0) : ldg16<false>(fb + (16 * j < cp ? 16 * j : 0));
        }
        // block span of the tail chunks (below); DS: from the descriptors alone,
        // bytes [64, caplen) of every frame rounded out to 16 B (a superset of
        // the checksummed tails), so the first tiles go out while the heads are
        // still in flight instead of one HBM round trip after them
        uint64_t lo = 0, hi = 0;
        uint32_t tsum = 0, span = 0;
        bool streamed = false;
        const uint8_t *sb = fb;
        auto tile_load = [&](uint4 *v, uint32_t c0) {
#pragma unroll
            for (int j = 0; j < LPT; ++j) {
                const uint32_t k = c0 + j * 256 + tid;
                v[j] = ldg16<NTS>(sb + ((uint64_t)(k < span ? k : 0) << 4)); // masked at use
            }
        };
        auto span_of = [&]() { // a span far larger than the tails means scattered frames
            streamed = hi > lo && hi - lo <= 2ull * tsum + TCH && hi - lo < (1ull << 26);
            span = streamed ? (uint32_t)(hi - lo) : 0u;
            // (not streamed: loads of the thread's own frame head, never consumed)
            sb = streamed ? pkts + (lo << 4) : fb;
            if constexpr ((ABL & 2) != 0) { // diagnostic: no tail stream at all
                streamed = true;
                span = 0;
            }
        };
        uint4 va[LPT], vb[LPT];
        if constexpr (DS) {
            const uint64_t ds_cs = (fpos + 64) >> 4, ds_ce = (fpos + (uint32_t)cp + 15u) >> 4;
            __syncthreads(); // s_lo/s_hi/s_tail initialised
            span_add(cp > 64, ds_cs, ds_ce, &s_lo, &s_hi, &s_tail, lane);
            __syncthreads();
            lo = s_lo, hi = s_hi, tsum = s_tail;
            span_of();
            tile_load(va, 0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) c[j] = chunk_below(c[j], 16 * j, cp); // past caplen reads as 0
        const uint32_t et = c[0].w & 0xFFFFu;
        const uint32_t tl = rx_bswap16(c[1].x & 0xFFFFu);
        const uint32_t proto = c[1].y >> 24;
        const uint32_t sip = (c[1].z >> 16) | (c[1].w << 16);
        const uint32_t dip = (c[1].w >> 16) | (c[2].x << 16);
        const uint32_t sport = c[2].x >> 16;
        const uint32_t dport = c[2].y & 0xFFFFu;
        const uint32_t dgl = rx_bswap16(c[2].y >> 16);
        const uint32_t hl = ((c[2].w >> 16) & 0xFFu) >> 4;
        uint32_t cl, nd;
        if (et == 0x0608u) {
            cl = RXG_CLS_ARP;
            nd = 42;
        } else if (et != 0x0008u) {
            cl = RXG_CLS_NON_IP;
            nd = 14;
        } else if (proto == 17u) {
            cl = RXG_CLS_UDP;
            nd = 42;
        } else if (proto == 6u) {
            cl = RXG_CLS_TCP;
            nd = 54;
        } else {
            cl = RXG_CLS_IPV4_OTHER;
            nd = 24;
        }
        const bool is_udp = cl == RXG_CLS_UDP, is_tcp = cl == RXG_CLS_TCP;
        const bool l4 = is_udp || is_tcp;
        const uint32_t l4n = tl >= 20u ? tl - 20u : 0u;
        const bool do_sum = l4 && tl >= 20u;
        if (l4 && 34u + l4n > nd) nd = 34u + l4n;
        int32_t e = do_sum ? 34 + (int32_t)l4n : 0;
        if (e > cp) e = cp;
        const int32_t ef = e & ~15; // full tail chunks: [64, ef)
        const bool part = ef < e && ef >= 64;
        const bool tail = ef > 64;
        const uint64_t cs_abs = (fpos + 64) >> 4, ce_abs = (fpos + (uint32_t)ef) >> 4;
        // the last partial chunk (consumed after the stream) and the first probe slot
        const uint4 pc = (ABL & 8) ? make_uint4(0, 0, 0, 0) : ldg16<false>(fb + (part ? ef : 0));
        const bool probe = valid && l4;
        const uint32_t ka = is_udp ? dip : sip;
        const uint32_t kb = is_udp ? dport : dip;
        const uint32_t kc = is_udp ? 17u : (sport | (dport << 16));
        const uint32_t maxp = is_udp ? ft.udp_probe : ft.tcp_probe;
        const bool probe0 = probe && maxp > 0 && !(ABL & 1);
        // the port entry, loaded with the head: UDP's direct port table entry
        // (which decides most UDP keys without the hashed table), TCP's listener
        // (tcp_stream_search pass 2, used on an exact-key miss)
        const bool udp_port = is_udp && ft.udp_port != nullptr;
        const uint32_t *ptab = udp_port ? ft.udp_port : ft.listen;
        const uint32_t pe = ptab[l4 ? dport : 0u];
        // and the hashed table's home slot (not needed by a port-decided UDP key:
        // a dummy load of the frame's own head then)
        const bool hash0 = probe0 && !udp_port;
        const uint4 *sp0 = hash0 ? (is_udp ? ft.udp : ft.tcp) +
                                       (rx_hash3s(ft.hseed, ka, kb, kc) & (is_udp ? ft.udp_mask : ft.tcp_mask))
                                 : reinterpret_cast<const uint4 *>(fb);
        static_assert(PW == 1 || PW == 2 || PW == 4, "probe window");
        uint4 sw[PW];
#pragma unroll
        for (int w = 0; w < PW; ++w) sw[w] = ld_slot(sp0 + (hash0 ? w : 0));

        uint4 h1 = c[1], h2 = c[2], h3 = c[3];
        h1.x = 0;
        h1.y = 0;
        h1.z &= 0xFFFF0000u;
        if (is_udp) h2.z &= 0xFFFF0000u;
        if (is_tcp) h3.x &= 0x0000FFFFu;
        uint32_t acc = lane_chunk_sum(0u, h1, 16, e);
        acc = lane_chunk_sum(acc, h2, 32, e);
        acc = lane_chunk_sum(acc, h3, 48, e);
        if (do_sum) acc += (proto << 8) + rx_bswap16(l4n); // pseudo-header words
        const uint32_t stored = is_udp ? (c[2].z & 0xFFFFu) : (is_tcp ? (c[3].x >> 16) : 0u);

        // block span of the tail chunks; a span far larger than the tails means
        // scattered frames (per-thread fallback below)
        if constexpr (!DS) {
            __syncthreads(); // s_lo/s_hi/s_tail initialised
            span_add(tail, cs_abs, ce_abs, &s_lo, &s_hi, &s_tail, lane);
            __syncthreads();
            lo = s_lo, hi = s_hi, tsum = s_tail;
            span_of();
        }
        if (part) acc = lane_chunk_sum(acc, pc, ef, e);

        // every verdict field that does not depend on the flow: payload offset and
        // length, flags (the truncation flag for both UDP outcomes: a delivered
        // datagram extends the bytes the reference reads to 42 + payload)
        uint32_t flags = 0, poff = 0, plen = 0;
        if (is_udp) {
            poff = 42;
            plen = dgl > 8u ? dgl - 8u : 0u;
            if (dgl <= 8u) flags |= RXG_F_UDP_SHORT;
        } else if (is_tcp) {
            const int32_t pl = (int32_t)tl - 20 - 4 * (int32_t)hl;
            poff = 34u + 4u * hl;
            if (pl < 0) flags |= RXG_F_TCP_NEGLEN;
            plen = pl < 0 ? 0u : (uint32_t)pl;
        }
        const bool trunc = (int32_t)nd > cp;
        const bool trunc_ok = trunc || (is_udp && (int32_t)(42u + plen) > cp);
        const uint32_t vy = (poff & 0xFFFFu) | (plen << 16);

        // flow probe (UDP always, TCP speculatively: a bad checksum drops the hit)
        // and the return code
        uint32_t flow = RXG_FLOW_NONE;
        int32_t rc = RXG_RC_KNI;
        auto probe_flow = [&]() {
            bool hashed = probe0;
            if (probe0 && udp_port) hashed = !rx_udp_port_decide(pe, ka, ft.udp_dip, &flow);
            if (hashed) {
                // slot index and table recomputed from the keys (HO = 2 keeps only
                // the keys and the first slot live across the stream)
                const uint4 *tb = is_udp ? ft.udp : ft.tcp;
                const uint32_t mk = is_udp ? ft.udp_mask : ft.tcp_mask;
                const uint32_t mp = is_udp ? ft.udp_probe : ft.tcp_probe;
                uint32_t pj = rx_hash3s(ft.hseed, ka, kb, kc) & mk;
                uint32_t pr = 0;
                bool done = false;
                if (hash0) { // the window loaded with the head
#pragma unroll
                    for (int w = 0; w < PW; ++w) {
                        if (!done) {
                            const uint4 sl = sw[w];
                            if (sl.w == RX_SLOT_EMPTY) {
                                done = true;
                            } else if (sl.x == ka && sl.y == kb && sl.z == kc) {
                                flow = sl.w;
                                done = true;
                            } else if (++pr >= mp) {
                                done = true;
                            } else {
                                pj = (pj + 1) & mk;
                            }
                        }
                    }
                }
                while (!done) { // past the window, or a UDP key on a shared port
                    const uint4 sl = ld_slot(tb + pj);
                    if (sl.w == RX_SLOT_EMPTY) break;
                    if (sl.x == ka && sl.y == kb && sl.z == kc) {
                        flow = sl.w;
                        break;
                    }
                    if (++pr >= mp) break;
                    pj = (pj + 1) & mk;
                }
            }
            if constexpr ((ABL & 1) != 0) flow = probe ? (dport & 0x3FFu) : RXG_FLOW_NONE;
            if (is_tcp && valid && flow == RXG_FLOW_NONE) flow = pe; // listener (prefetched)
            if (is_udp)
                rc = flow == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                           : ((flags & RXG_F_UDP_SHORT) ? RXG_RC_UDP_NOMEM : RXG_RC_OK);
            if (rc == RXG_RC_OK ? trunc_ok : trunc) flags |= RXG_F_TRUNC;
        };
        if constexpr (HO == 0) probe_flow();
        // ---- tail phase -------------------------------------------------------
        if constexpr (!DS) tile_load(va, 0);
        if constexpr (HO == 1) probe_flow();
        if (streamed) {
            const uint32_t cs = tail ? (uint32_t)(cs_abs - lo) : 0xFFFFFFFFu;
            const uint32_t ce = tail ? (uint32_t)(ce_abs - lo) : 0xFFFFFFFFu;
            uint32_t es = 0, ee = 0, carry = 0;
            // one tile: chunk sums, exclusive prefix (wave scans + wave totals via
            // LDS), then each frame picks up its boundary values
            auto tile = [&](const uint4 *v, uint32_t c0, uint32_t buf) {
                uint32_t sj[LPT], xj[LPT];
#pragma unroll
                for (int j = 0; j < LPT; ++j) {
                    sj[j] = c0 + j * 256 + tid < span ? chunk_sum(v[j]) : 0u;
                    xj[j] = sj[j];
                }
                wave_incl_scan_n<LPT>(xj);
                if (lane == 63) {
#pragma unroll
                    for (int j = 0; j < LPT; ++j) s_wt[buf][j * 4 + wv] = xj[j];
                }
                __syncthreads();
                if constexpr (B1) { // the previous tile's boundaries (buffer buf ^ 1)
                    const uint32_t p0 = c0 - TCH; // wraps for c0 = 0: no frame matches
                    if (c0 != 0 && cs - p0 < TCH) es = s_pre[buf ^ 1u][cs - p0];
                    if (c0 != 0 && ce - p0 < TCH) ee = s_pre[buf ^ 1u][ce - p0];
                }
                uint32_t wt[4 * LPT]; // block-uniform: kept in SGPRs
#pragma unroll
                for (int j = 0; j < LPT; ++j) {
                    const uint4 r = *reinterpret_cast<const uint4 *>(&s_wt[buf][j * 4]);
                    wt[j * 4 + 0] = __builtin_amdgcn_readfirstlane(r.x);
                    wt[j * 4 + 1] = __builtin_amdgcn_readfirstlane(r.y);
                    wt[j * 4 + 2] = __builtin_amdgcn_readfirstlane(r.z);
                    wt[j * 4 + 3] = __builtin_amdgcn_readfirstlane(r.w);
                }
                uint32_t base = carry;
#pragma unroll
                for (int j = 0; j < LPT; ++j) {
                    uint32_t wb = 0;
#pragma unroll
                    for (int w = 0; w < 4; ++w) wb += (uint32_t)w < wvu ? wt[j * 4 + w] : 0u;
                    s_pre[buf][j * 256 + tid] = base + wb + xj[j] - sj[j];
                    base += wt[j * 4] + wt[j * 4 + 1] + wt[j * 4 + 2] + wt[j * 4 + 3];
                }
                carry = base;
                if constexpr (!B1) {
                    __syncthreads();
                    if (cs - c0 < TCH) es = s_pre[buf][cs - c0];
                    if (ce - c0 < TCH) ee = s_pre[buf][ce - c0];
                }
            };
            // unrolled twice: the A/B tiles swap roles without register moves (a
            // move would wait for the prefetch it copies); one exit per pair (a
            // trailing all-masked tile costs no bandwidth: its loads hit chunk 0)
            uint32_t c0 = 0;
            for (; c0 < span; c0 += 2 * TCH) {
                tile_load(vb, c0 + TCH);
                tile(va, c0, 0);
                tile_load(va, c0 + 2 * TCH);
                tile(vb, c0 + TCH, 1);
            }
            if constexpr (B1) { // the last tile's boundaries (buffer 1)
                __syncthreads();
                const uint32_t p0 = c0 - TCH;
                if (cs - p0 < TCH) es = s_pre[1][cs - p0];
                if (ce - p0 < TCH) ee = s_pre[1][ce - p0];
            }
            if (ce == span) ee = carry;
            if (tail) acc += ee - es;
        } else if (tail) { // scattered frames: this thread sums its own tail
            for (int32_t s = 64; s < ef; s += 64) {
                uint4 r[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) r[u] = ldg16<false>(fb + (s + 16 * u < ef ? s + 16 * u : 0));
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (s + 16 * u < ef) acc += chunk_sum(r[u]);
            }
        }

        if constexpr (HO >= 2) probe_flow();
        // ---- verdict ----------------------------------------------------------
        uint32_t ck = 0;
        if (do_sum) {
            ck = (~fold16(acc)) & 0xFFFFu;
            if (ck == 0u && proto == 17u) ck = 0xFFFFu;
        }
        const bool ok = l4 && stored == ck;
        if (is_tcp) {
            if (!ok) flow = RXG_FLOW_NONE;
            rc = !ok ? RXG_RC_TCP_BAD_CKSUM : (flow == RXG_FLOW_NONE ? RXG_RC_TCP_NO_TCB : RXG_RC_OK);
        }
        const uint32_t cidx = valid && rc == RXG_RC_OK && flow != RXG_FLOW_NONE
                                  ? (is_tcp ? ft.nu : 0u) + flow
                                  : 0xFFFFFFFFu;
        if (valid) {
            uint4 vd;
            vd.x = flow;
            vd.y = vy;
            vd.z = ck | (cl << 16) | (((uint32_t)rc & 0xFFu) << 24);
            vd.w = (ok ? 1u : 0u) | (flags << 8) | (stored << 16);
            st_verdict<WT>(ft, out, p, vd);
            lane_count(cidx, counts, hist, lds_bins);
        }
        // (FPB < 64: the first FPB lanes of wave 0; its other lanes' pieces are the next block's)
        if (FPB >= 256 || wv * 64 < FPB) put_count_idx_wave(ft, p, cidx, lane, FPB < 64 ? FPB : 64);
    } // tile
    if (lds_bins) {
        __syncthreads();
        for (uint32_t i = tid; i < lds_bins; i += 256) {
            const uint32_t cnt = hist[i];
            if (cnt) atomicAdd(&counts[i], (unsigned long long)cnt);
        }
    }
}

template <bool NTS, int ABL = 0, int HO = 0, int PW = 1, bool B1 = false, bool DS = false,
          bool HG = false, uint32_t FPB = 256, int L = 4, bool WT = false>
hipError_t launch_stream(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                         uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out,
                         unsigned long long *counts, uint32_t lds_bins, hipStream_t s,
                         const uint32_t *, const uint32_t *) {
    const uint64_t blocks = ((uint64_t)n + FPB - 1) / FPB;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((rx_classify_stream_kernel<NTS, ABL, HO, PW, B1, DS, HG, FPB, L, WT>), dim3((uint32_t)blocks),
                       dim3(256), (size_t)lds_bins * 4u, s, pkts, off, len, n, unit_log2, ft, out,
                       counts, lds_bins);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Stream kernel with the frame heads taken out of the block stream (SH, pipe
// 60).  The block span covers every captured byte of its 256 frames, known
// from the descriptors alone, so the first tile's loads go out one descriptor
// round trip after the block starts, with no head loads before them.  Each
// frame's owner marks its head chunks (the first 4 of its 16-B chunks) in an
// LDS map of the span (u8 per chunk: the owner; 0xFF is also "none") and
// publishes its first chunk; the lane that streams a chunk writes it to the
// owner's 64-B LDS head slot at k = chunk - first when k < 4 (an unmarked
// chunk reads as thread 255's, whose k is then out of range or past its
// capture, masked).  A frame's
// tail sum is the prefix difference at two chunk boundaries known from the
// descriptors: [64, caplen & ~15).  The partial last chunk of a frame (caplen
// not a multiple of 16) is captured from the stream as well: its owner marks
// it in the map, and the streaming lane writes it to slot 0 of the owner's
// head slots, whose chunk 0 is not kept (the parse needs only its ether type,
// which that lane publishes as a 2-bit class).  So nothing is loaded per frame
// at the block start (a 16-B load there fetched a line that the L2 had evicted
// again before the stream reached it: 3.6M extra L2 misses and 5% of the cfg4
// time, pipe 264 ablation, profiles/r03e).  After the stream the owner parses
// its head from LDS, sums its partial chunk, probes the flow table and writes
// the verdict.  Exact, with fallbacks that are rare in real bursts:
//  - the L4 sum ends before the capture (14 + total_length < caplen, e.g.
//    Ethernet padding): the owner re-sums [64, end) from HBM;
//  - frames sharing head or partial chunks (overlapping descriptors): the
//    losers of the map write read those from HBM after the stream (checked
//    after the map barrier), as do captures under 14 bytes (a class cannot
//    mask an ether type cut by the capture);
//  - a span of scattered frames or one larger than the map (SH_MAPC chunks):
//    per-thread head loads and tail loops.
// LDS 31.9 KiB per block (map 7.25, heads 16, prefixes 8): 5 blocks per CU.
constexpr uint32_t SH_MAPC = 7424; // span chunks the head map covers (116 KiB)

// header fields of a frame head (the first 64 B, bytes past caplen zeroed)
struct sh_head {
    uint32_t cl, nd, tl, proto, l4n, dgl, hl, ka, kb, kc, stored;
    bool is_udp, is_tcp, l4, do_sum;
    int32_t e; // end of the checksummed bytes
};

__device__ __forceinline__ sh_head sh_parse(const uint4 (&c)[4], int32_t cp) {
    sh_head h;
    const uint32_t et = c[0].w & 0xFFFFu;
    h.tl = rx_bswap16(c[1].x & 0xFFFFu);
    h.proto = c[1].y >> 24;
    const uint32_t sip = (c[1].z >> 16) | (c[1].w << 16);
    const uint32_t dip = (c[1].w >> 16) | (c[2].x << 16);
    const uint32_t sport = c[2].x >> 16;
    const uint32_t dport = c[2].y & 0xFFFFu;
    h.dgl = rx_bswap16(c[2].y >> 16);
    h.hl = ((c[2].w >> 16) & 0xFFu) >> 4;
    if (et == 0x0608u) {
        h.cl = RXG_CLS_ARP;
        h.nd = 42;
    } else if (et != 0x0008u) {
        h.cl = RXG_CLS_NON_IP;
        h.nd = 14;
    } else if (h.proto == 17u) {
        h.cl = RXG_CLS_UDP;
        h.nd = 42;
    } else if (h.proto == 6u) {
        h.cl = RXG_CLS_TCP;
        h.nd = 54;
    } else {
        h.cl = RXG_CLS_IPV4_OTHER;
        h.nd = 24;
    }
    h.is_udp = h.cl == RXG_CLS_UDP;
    h.is_tcp = h.cl == RXG_CLS_TCP;
    h.l4 = h.is_udp || h.is_tcp;
    h.l4n = h.tl >= 20u ? h.tl - 20u : 0u;
    h.do_sum = h.l4 && h.tl >= 20u;
    if (h.l4 && 34u + h.l4n > h.nd) h.nd = 34u + h.l4n;
    h.e = h.do_sum ? 34 + (int32_t)h.l4n : 0;
    if (h.e > cp) h.e = cp;
    h.ka = h.is_udp ? dip : sip;
    h.kb = h.is_udp ? dport : dip;
    h.kc = h.is_udp ? 17u : (sport | (dport << 16));
    h.stored = h.is_udp ? (c[2].z & 0xFFFFu) : (h.is_tcp ? (c[3].x >> 16) : 0u);
    return h;
}

// a parsed head in two words besides its key (EP: kept through the stream):
// a = tl | dgl << 16, b = stored | proto << 16 | cl << 24 | hl << 28
__device__ __forceinline__ uint32_t sh_pack_a(const sh_head &h) { return h.tl | (h.dgl << 16); }
__device__ __forceinline__ uint32_t sh_pack_b(const sh_head &h) {
    return h.stored | (h.proto << 16) | (h.cl << 24) | (h.hl << 28);
}
__device__ __forceinline__ sh_head sh_unpack(uint32_t ka, uint32_t kb, uint32_t kc, uint32_t a,
                                             uint32_t b, int32_t cp) {
    sh_head h;
    h.tl = a & 0xFFFFu;
    h.dgl = a >> 16;
    h.stored = b & 0xFFFFu;
    h.proto = (b >> 16) & 0xFFu;
    h.cl = (b >> 24) & 0xFu;
    h.hl = b >> 28;
    h.ka = ka;
    h.kb = kb;
    h.kc = kc;
    h.is_udp = h.cl == RXG_CLS_UDP;
    h.is_tcp = h.cl == RXG_CLS_TCP;
    h.l4 = h.is_udp || h.is_tcp;
    h.nd = h.cl == RXG_CLS_ARP ? 42u
         : h.cl == RXG_CLS_NON_IP ? 14u
         : h.is_udp ? 42u
         : h.is_tcp ? 54u
                    : 24u;
    h.l4n = h.tl >= 20u ? h.tl - 20u : 0u;
    h.do_sum = h.l4 && h.tl >= 20u;
    if (h.l4 && 34u + h.l4n > h.nd) h.nd = 34u + h.l4n;
    h.e = h.do_sum ? 34 + (int32_t)h.l4n : 0;
    if (h.e > cp) h.e = cp;
    return h;
}

// the checksum words of head chunks 1..3 (the header bytes [0, 26) and the
// L4 checksum field excluded) plus the pseudo-header's {proto, L4 length}
__device__ __forceinline__ uint32_t sh_head_sum(const uint4 (&c)[4], const sh_head &h) {
    uint4 h1 = c[1], h2 = c[2], h3 = c[3];
    h1.x = 0;
    h1.y = 0;
    h1.z &= 0xFFFF0000u;
    if (h.is_udp) h2.z &= 0xFFFF0000u;
    if (h.is_tcp) h3.x &= 0x0000FFFFu;
    uint32_t acc = lane_chunk_sum(0u, h1, 16, h.e);
    acc = lane_chunk_sum(acc, h2, 32, h.e);
    acc = lane_chunk_sum(acc, h3, 48, h.e);
    if (h.do_sum) acc += (h.proto << 8) + rx_bswap16(h.l4n); // pseudo-header words
    return acc;
}

// ABL (diagnostic builds, pipes 160 / 264): 1 = no flow-table probe (flow id
// from the port; wrong verdicts by construction), 2 = every partial last
// chunk loaded from HBM after the stream (no partial marks), 16 = no count-index
// store, 32 = the count-index store before the verdict store, 64 = no verdict
// store.  PW: slots of the first probe window
// (1, 2 or 4 consecutive slots of the hashed table loaded together; the table
// mirrors its first slots past its end), so a displaced key costs no dependent
// second round trip at the end of the block (pipes 60 / 63 / 64).
// MAPC: span chunks the head map covers.  (A map for 256 frames of 1500 B,
// 388 KiB of span at 3 blocks/CU, ran cfg3 at 1.161 vs 1.042 ms for the G=8
// group kernel: profiles/r02ac.)
// EP (pipe 65): every frame's probe is issued as soon as its head is known,
// inside the stream, instead of after it, so the block no longer ends on the
// probe round trip.  A frame whose head completes in tile t < last has it
// parsed from LDS after tile t's barrier; a frame whose head completes in the
// block's LAST tile ("early") has its four head chunks loaded at the block
// start by LDS-DMA (no VGPRs held through the stream; its head chunks are not
// marked in the map) and parsed after tile 0.  The parsed head is kept as 7
// words per lane; the probe window (PW <= 3 slots) is loaded by LDS-DMA into
// the frame's own head slots 1..3, which the parse has freed (s_hd is
// slot-major, [k][256], so one wave's slot k is the lane-linear 1 KiB an
// LDS-DMA instruction writes).  An early frame's s_rel carries bit 15, so the
// stream never takes one of its chunks for a head chunk (a chunk no frame
// marked reads as thread 255's).
// PS: the lane that streams a frame's partial last chunk sums it (masked at
// the capture, from s_cp) into s_psum instead of storing the chunk in head
// slot 0, so a head takes 48 B of LDS instead of 64 (with 8-KiB tiles the
// block fits 6 per CU: 26.1 KiB).
// FPB: frames per block (a multiple of 64; threads past it only stream), so
// that larger frames still fit the head map (1500 B: 64 frames, 96 KiB).
// TT: stream tiles in flight per thread (2, or 3 with a period-3 rotation).
// PERS: a resident grid; each block loops over block-tiles of FPB frames and
// loads the next one's descriptors during the current one's stream, so no
// block starts on a descriptor round trip (and the LDS histogram is flushed
// once per block instead of once per 256 frames).
// WT: write-through (sc1) verdict stores (the G=8 kernel's pipe 40).
template <int ABL = 0, int PW = 1, uint32_t MAPC = SH_MAPC, bool EP = false, int L = EP ? 3 : 4,
          bool PS = false, int FPB = 256, int TT = 2, bool PERS = false, bool WT = false>
__global__ __launch_bounds__(256, MAPC > SH_MAPC ? 3 : (PS && L == 2 ? 6 : 5)) void rx_classify_sh_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t n, uint32_t unit_log2, rx_ft_dev ft,
    uint4 *__restrict__ out, unsigned long long *__restrict__ counts, uint32_t lds_bins) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    // 16-B chunks per thread per tile (EP: 12-KiB tiles, so the parse inside
    // the stream fits the 96 VGPRs of 5 blocks/CU without scratch)
    constexpr uint32_t LPT = L;
    constexpr uint32_t TCH = 256u * LPT; // chunks per tile (16 KiB)
    __shared__ __attribute__((aligned(16))) uint32_t s_pre[2][TCH];
    __shared__ __attribute__((aligned(16))) uint32_t s_wt[2][4 * LPT]; // [row j][wave w]
    __shared__ __attribute__((aligned(16))) uint8_t s_map[MAPC];
    static_assert(!(EP && PS), "EP keeps chunk 0 in head slot 0");
    __shared__ __attribute__((aligned(16))) uint4 s_hd[256 * (PS ? 3 : 4)];
    __shared__ uint32_t s_psum[PS ? 256 : 1]; // PS: each frame's partial-chunk sum
    __shared__ uint16_t s_cp[PS ? 256 : 1];   // PS: each frame's capture length
    __shared__ uint16_t s_rel[256]; // each frame's first chunk in the span
    __shared__ uint32_t s_et[16];   // each frame's ether-type class, 2 bits (1 IPv4, 2 ARP)
    __shared__ unsigned long long s_lo, s_hi;
    __shared__ uint32_t s_tail, s_pk255; // thread 255's partial chunk (an unmarked chunk reads as 255)
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t wvu = __builtin_amdgcn_readfirstlane(wv);
    // head slot k of frame m
    auto hdi = [](uint32_t m, uint32_t k) -> uint32_t {
        return EP ? k * 256u + m : (PS ? (k - 1u) * 256u + m : m * 4u + k);
    };
    for (uint32_t i = tid; i < lds_bins; i += 256) hist[i] = 0;
    static_assert(FPB % 64 == 0 && FPB <= 256, "whole waves of frames");
    const uint32_t nblk = (uint32_t)(((uint64_t)n + FPB - 1) / FPB);
    // PERS: this block-tile's descriptors, loaded during the previous one
    uint32_t nx_off = 0;
    int32_t nx_len = 0;
    auto desc_load = [&](uint32_t blk) {
        const uint64_t pp = (uint64_t)blk * FPB + tid;
        const bool vv = blk < nblk && tid < (uint32_t)FPB && pp < n;
        nx_off = off[vv ? pp : 0];
        nx_len = vv ? (int32_t)len[vv ? pp : 0] : 0;
    };
    if constexpr (PERS) desc_load(blockIdx.x);
    // (without PERS the loop is one trip the compiler sees as such)
    const uint32_t bend = PERS ? nblk : blockIdx.x + 1u;
    for (uint32_t blk = blockIdx.x; blk < bend; blk += PERS ? gridDim.x : 1u) {
    if (tid == 0) {
        s_lo = ~0ull;
        s_hi = 0;
        s_tail = 0;
        s_pk255 = ~0u;
    }
    if (tid < 16) s_et[tid] = 0;
    {
        uint4 *m4 = reinterpret_cast<uint4 *>(s_map);
        for (uint32_t i = tid; i < MAPC / 16; i += 256) m4[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    const uint64_t p = (uint64_t)blk * FPB + tid;
    const bool valid = tid < (uint32_t)FPB && p < n;
    const uint64_t q = valid ? p : 0;
    uint32_t doff;
    int32_t dlen;
    if constexpr (PERS) {
        doff = nx_off;
        dlen = nx_len;
        desc_load(blk + gridDim.x); // in flight through this block-tile's stream
    } else {
        doff = off[q];
        dlen = valid ? (int32_t)len[q] : 0;
    }
    const uint64_t fpos = (uint64_t)doff << unit_log2;
    const int32_t cp = dlen;
    const uint8_t *fb = pkts + fpos;
    const uint64_t fc = fpos >> 4;                  // first chunk (absolute)
    const uint32_t nch = ((uint32_t)cp + 15u) >> 4; // chunks of the capture
    const int32_t cf = cp & ~15;                    // full chunks: [0, cf)
    const bool part = cf >= 64 && cf < cp;          // a partial last chunk past the head
    __syncthreads(); // s_lo/s_hi/s_tail and the map initialised
    span_add(cp > 0, fc, fc + nch, &s_lo, &s_hi, &s_tail, lane);
    __syncthreads();
    const uint64_t lo = s_lo, hi = s_hi;
    const uint32_t tsum = s_tail;
    const bool streamed = hi > lo && hi - lo <= MAPC && hi - lo <= 2ull * tsum + TCH;
    const uint32_t span = streamed ? (uint32_t)(hi - lo) : 0u;
    const uint8_t *sb = streamed ? pkts + (lo << 4) : fb;
    auto tile_load = [&](uint4 *v, uint32_t c0) {
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const uint32_t k = c0 + j * 256 + tid;
            v[j] = ldg16<true>(sb + ((uint64_t)(k < span ? k : 0) << 4)); // masked at use
        }
    };
    uint4 va[LPT], vb[LPT];
    tile_load(va, 0);
    const uint32_t rel = (streamed && cp > 0) ? (uint32_t)(fc - lo) : 0u;
    const uint32_t nh = nch < 4u ? nch : 4u;
    // EP: the stream's last tile, the tile that completes this frame's head
    const uint32_t tlast = span ? (span - 1u) / TCH : 0u;
    const uint32_t thead = cp > 0 ? (rel + nh - 1u) / TCH : 0u;
    // (tlast >= 2: the early parse runs after the first tile pair, which must
    // not hold the last tile, whose partial chunks land in head slot 0)
    const bool early = EP && streamed && cp >= 14 && tlast >= 2 && thead == tlast;
    const uint32_t relx = early ? 0x8000u : 0u; // (rel < MAPC < 0x8000)
    if (streamed) {
        if (!early)
            for (uint32_t k = 0; k < nh; ++k) s_map[rel + k] = (uint8_t)tid;
        s_rel[tid] = (uint16_t)(rel + relx);
        if (part && !(ABL & 2)) {
            s_map[rel + ((uint32_t)cf >> 4)] = (uint8_t)tid;
            if constexpr (PS) s_cp[tid] = (uint16_t)cp;
            if (tid == 255) s_pk255 = ((uint32_t)cf >> 4) - relx;
        }
    }
    __syncthreads(); // map complete
    const uint32_t pk255 = __builtin_amdgcn_readfirstlane(s_pk255);
    // heads from HBM after the stream: not streamed, a shared head chunk, or
    // an ether type cut by the capture; the partial chunk from HBM: not
    // streamed is summed from HBM anyway, a lost mark
    bool direct = cp > 0 && (!streamed || cp < 14);
    bool plost = false;
    if (streamed) {
        if (!early)
            for (uint32_t k = 0; k < nh; ++k)
                if (s_map[rel + k] != (uint8_t)tid) direct = true; // shared head chunk
        plost = part && ((ABL & 2) || s_map[rel + ((uint32_t)cf >> 4)] != (uint8_t)tid);
    }
    // EP: the frames whose probe goes out inside the stream (the rest, rare,
    // keep the after-stream path)
    const bool inflight = EP && streamed && cp >= 14 && !direct && tlast > 0 && (early || thead < tlast);
    if constexpr (EP) {
        if (__ballot(early) != 0ull) { // the early heads, by LDS-DMA into slots 0..3
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t dst = __builtin_amdgcn_readfirstlane(
                    rx_lds_addr(&s_hd[hdi(64u * wvu, (uint32_t)k)]));
                if (early) rx_dma16(16 * k < cp ? fb + 16 * k : fb, dst);
            }
        }
    }

    // ---- flow probe loads: the port entry (UDP: the direct port table; TCP:
    // the listener) and the hashed table's home slot, issued once per frame
    static_assert(PW == 1 || PW == 2 || PW == 4, "probe window");
    static_assert(!EP || PW <= 2, "EP: the window lives in head slots 1..2, the parsed key in 3");
    static_assert(PW - 1 <= RX_FT_MIRROR, "window past the mirrored slots");
    uint32_t pe = RXG_FLOW_NONE;
    uint4 sw[PW];
    // the probe's first loads of a parsed head: the port entry (returned) and
    // the hashed table's home window (sp0, when hash0)
    auto probe_src = [&](const sh_head &h, bool &hash0, const uint4 *&sp0) -> uint32_t {
        const bool probe0 =
            valid && h.l4 && (h.is_udp ? ft.udp_probe : ft.tcp_probe) > 0 && !(ABL & 1);
        const bool udp_port = h.is_udp && ft.udp_port != nullptr;
        const uint32_t *ptab = udp_port ? ft.udp_port : ft.listen;
        const uint32_t dport = h.is_udp ? h.kb : (h.kc >> 16);
        hash0 = probe0 && !udp_port;
        sp0 = hash0 ? (h.is_udp ? ft.udp : ft.tcp) +
                          (rx_hash3s(ft.hseed, h.ka, h.kb, h.kc) & (h.is_udp ? ft.udp_mask : ft.tcp_mask))
                    : reinterpret_cast<const uint4 *>(pkts);
        return (ABL & 1) ? RXG_FLOW_NONE : ptab[h.l4 ? dport : 0u];
    };
    auto issue_probe = [&](const uint4 (&c)[4]) {
        const sh_head h = sh_parse(c, cp);
        bool hash0;
        const uint4 *sp0;
        pe = probe_src(h, hash0, sp0);
#pragma unroll
        for (int w = 0; w < PW; ++w) sw[w] = ld_slot(sp0 + (hash0 ? w : 0));
    };
    // chunk 0 stands in by its ether type (the class the stream published);
    // slot 0 holds the partial last chunk
    auto head_of = [&](uint4 (&c)[4]) {
        const uint32_t ec = (s_et[tid >> 4] >> (2u * (tid & 15u))) & 3u;
        c[0] = make_uint4(0, 0, 0, ec == 1u ? 0x0008u : (ec == 2u ? 0x0608u : 0u));
#pragma unroll
        for (int k = 1; k < 4; ++k) c[k] = chunk_below(s_hd[hdi(tid, (uint32_t)k)], 16 * k, cp);
    };

    // ---- stream: tile prefixes, head capture, boundary pickup ---------------
    const bool tailf = cf > 64; // full chunks past the head: [4, cf / 16)
    const uint32_t cs = tailf ? rel + 4u : 0xFFFFFFFFu;
    const uint32_t ce = tailf ? rel + ((uint32_t)cf >> 4) : 0xFFFFFFFFu;
    uint32_t es = 0, ee = 0, carry = 0;
    auto stile = [&](const uint4 *v, uint32_t c0, uint32_t buf) {
        uint32_t sj[LPT], xj[LPT];
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const uint32_t k = c0 + j * 256 + tid;
            sj[j] = k < span ? chunk_sum(v[j]) : 0u;
            xj[j] = sj[j];
            if (k < span) { // (0xFF is thread 255 or no mark: the k range tells)
                const uint32_t m = s_map[k], hk = k - s_rel[m];
                if (hk == 0u) { // chunk 0: its ether type, as a class
                    const uint32_t et = v[j].w & 0xFFFFu;
                    const uint32_t ec = et == 0x0008u ? 1u : (et == 0x0608u ? 2u : 0u);
                    if (ec) atomicOr(&s_et[m >> 4], ec << (2u * (m & 15u)));
                } else if (hk < 4u || m != 255u || hk == pk255) {
                    // head chunks 1..3, or the owner's partial chunk (the only
                    // other chunk it marks) into slot 0
                    if (!PS || hk < 4u)
                        s_hd[hdi(m, hk < 4u ? hk : 0u)] = v[j];
                    else
                        s_psum[m] = lane_chunk_sum(0u, v[j], 16 * (int32_t)hk, (int32_t)s_cp[m]);
                }
            }
        }
        wave_incl_scan_n<LPT>(xj);
        if (lane == 63) {
#pragma unroll
            for (int j = 0; j < LPT; ++j) s_wt[buf][j * 4 + wv] = xj[j];
        }
        __syncthreads();
        { // the previous tile's boundaries (buffer buf ^ 1)
            const uint32_t p0 = c0 - TCH; // wraps for c0 = 0: no frame matches
            if (c0 != 0 && cs - p0 < TCH) es = s_pre[buf ^ 1u][cs - p0];
            if (c0 != 0 && ce - p0 < TCH) ee = s_pre[buf ^ 1u][ce - p0];
        }
        uint32_t wt[4 * LPT]; // block-uniform: kept in SGPRs
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            const uint4 r = *reinterpret_cast<const uint4 *>(&s_wt[buf][j * 4]);
            wt[j * 4 + 0] = __builtin_amdgcn_readfirstlane(r.x);
            wt[j * 4 + 1] = __builtin_amdgcn_readfirstlane(r.y);
            wt[j * 4 + 2] = __builtin_amdgcn_readfirstlane(r.z);
            wt[j * 4 + 3] = __builtin_amdgcn_readfirstlane(r.w);
        }
        uint32_t base = carry;
#pragma unroll
        for (int j = 0; j < LPT; ++j) {
            uint32_t wb = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) wb += (uint32_t)w < wvu ? wt[j * 4 + w] : 0u;
            s_pre[buf][j * 256 + tid] = base + wb + xj[j] - sj[j];
            base += wt[j * 4] + wt[j * 4 + 1] + wt[j * 4 + 2] + wt[j * 4 + 3];
        }
        carry = base;
    };
    // EP: after tile c0's barrier, the frames whose head is now known parse it,
    // keep it packed, load the port entry and send the window's LDS-DMA
    uint32_t spa = 0, spb = 0;
    auto ep_issue = [&](uint32_t c0) {
        if constexpr (EP) {
            const bool due = inflight && (early ? c0 == 0u : (thead >> 1) * (2u * TCH) == c0);
            if (__ballot(due) == 0ull) return;
            // the early heads' LDS-DMA went out before the next tile's LPT
            // loads (the counter retires in order; the stream waited as far)
            if (c0 == 0u) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
            if (due) {
                uint4 c[4];
                head_of(c);
                if (early) c[0] = s_hd[hdi(tid, 0u)]; // (only its ether type is parsed)
                const sh_head h = sh_parse(c, cp);
                spa = sh_pack_a(h);
                spb = sh_pack_b(h);
                // slots 1..3 were read above: the key and the head sum to slot 3
                s_hd[hdi(tid, 3u)] = make_uint4(h.ka, h.kb, h.kc, sh_head_sum(c, h));
                bool hash0;
                const uint4 *sp0;
                pe = probe_src(h, hash0, sp0);
                if (hash0) // the window to slots 1..PW
#pragma unroll
                    for (int w = 0; w < PW; ++w)
                        rx_dma16(sp0 + w, __builtin_amdgcn_readfirstlane(
                                              rx_lds_addr(&s_hd[hdi(64u * wvu, 1u + w)])));
            }
        }
    };
    static_assert(TT == 2 || (TT == 3 && !EP), "tiles in flight");
    uint32_t c0 = 0;
    if constexpr (TT == 3) { // tile t in buffer t & 1, three tiles of loads in flight
        uint4 vc[LPT];
        tile_load(vb, TCH);
        for (; c0 < span; c0 += 3 * TCH) {
            const uint32_t t0 = c0 / TCH;
            tile_load(vc, c0 + 2 * TCH);
            stile(va, c0, t0 & 1u);
            tile_load(va, c0 + 3 * TCH);
            stile(vb, c0 + TCH, (t0 + 1u) & 1u);
            tile_load(vb, c0 + 4 * TCH);
            stile(vc, c0 + 2 * TCH, t0 & 1u);
        }
    } else {
        for (; c0 < span; c0 += 2 * TCH) {
            tile_load(vb, c0 + TCH);
            stile(va, c0, 0);
            tile_load(va, c0 + 2 * TCH);
            stile(vb, c0 + TCH, 1);
            ep_issue(c0); // the heads completed in this pair of tiles
        }
    }
    __syncthreads(); // the last tile's prefixes and every head slot written
    if constexpr (EP) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the windows landed
    if (streamed) {
        const uint32_t p0 = c0 - TCH, lb = (p0 / TCH) & 1u; // the last tile, its buffer
        if (cs - p0 < TCH) es = s_pre[lb][cs - p0];
        if (ce - p0 < TCH) ee = s_pre[lb][ce - p0];
        if (ce == span) ee = carry;
    }

    // ---- head: parse, checksum, probe, verdict ------------------------------------
    uint4 c[4];
    head_of(c);
    if (__ballot(direct) != 0ull) { // rare (wave-uniform branch): heads from HBM
        uint4 hd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) hd[k] = ldg16<false>(direct && 16 * k < cp ? fb + 16 * k : pkts);
        if (direct)
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = chunk_below(hd[k], 16 * k, cp);
    }
    sh_head h;
    uint32_t acc;
    if (EP && inflight) { // parsed inside the stream; the window in slots 1..PW
        const uint4 k3 = s_hd[hdi(tid, 3u)];
        h = sh_unpack(k3.x, k3.y, k3.z, spa, spb, cp);
        acc = k3.w;
#pragma unroll
        for (int w = 0; w < PW; ++w) sw[w] = s_hd[hdi(tid, 1u + w)];
    } else {
        issue_probe(c);
        h = sh_parse(c, cp);
        acc = sh_head_sum(c, h);
    }
    const int32_t e = h.e;
    // the sum ends where the capture does (the common case): tail from the
    // stream prefixes, the partial chunk from its slot; otherwise re-sum from HBM
    if (h.do_sum && e > 64) {
        if (streamed && e == cp) {
            if (tailf) acc += ee - es;
            if (part) {
                if constexpr (PS) {
                    uint32_t ps = plost ? 0u : s_psum[tid];
                    if (__ballot(plost) != 0ull) { // rare (wave-uniform branch): lost mark
                        const uint4 ph = ldg16<false>(plost ? fb + cf : pkts);
                        if (plost) ps = lane_chunk_sum(0u, ph, cf, e);
                    }
                    acc += ps;
                } else {
                    uint4 pv = s_hd[hdi(tid, 0u)];
                    if (__ballot(plost) != 0ull) { // rare (wave-uniform branch): lost mark
                        const uint4 ph = ldg16<false>(plost ? fb + cf : pkts);
                        if (plost) pv = ph;
                    }
                    acc = lane_chunk_sum(acc, pv, cf, e);
                }
            }
        } else {
            for (int32_t s = 64; s < e; s += 16) acc = lane_chunk_sum(acc, ldg16<false>(fb + s), s, e);
        }
    }
    uint32_t ck = 0;
    if (h.do_sum) {
        ck = (~fold16(acc)) & 0xFFFFu;
        if (ck == 0u && h.proto == 17u) ck = 0xFFFFu;
    }
    const bool probe = valid && h.l4;
    const uint32_t maxp = h.is_udp ? ft.udp_probe : ft.tcp_probe;
    const bool probe0 = probe && maxp > 0 && !(ABL & 1);
    const bool udp_port = h.is_udp && ft.udp_port != nullptr;
    const bool hash0 = probe0 && !udp_port;
    uint32_t flags = 0, poff = 0, plen = 0;
    if (h.is_udp) {
        poff = 42;
        plen = h.dgl > 8u ? h.dgl - 8u : 0u;
        if (h.dgl <= 8u) flags |= RXG_F_UDP_SHORT;
    } else if (h.is_tcp) {
        const int32_t pl = (int32_t)h.tl - 20 - 4 * (int32_t)h.hl;
        poff = 34u + 4u * h.hl;
        if (pl < 0) flags |= RXG_F_TCP_NEGLEN;
        plen = pl < 0 ? 0u : (uint32_t)pl;
    }
    const bool trunc = (int32_t)h.nd > cp;
    const bool trunc_ok = trunc || (h.is_udp && (int32_t)(42u + plen) > cp);
    uint32_t flow = RXG_FLOW_NONE;
    int32_t rc = RXG_RC_KNI;
    bool hashed = probe0;
    if (probe0 && udp_port) hashed = !rx_udp_port_decide(pe, h.ka, ft.udp_dip, &flow);
    if (hashed) {
        const uint4 *tb = h.is_udp ? ft.udp : ft.tcp;
        const uint32_t mk = h.is_udp ? ft.udp_mask : ft.tcp_mask;
        uint32_t pj = rx_hash3s(ft.hseed, h.ka, h.kb, h.kc) & mk;
        uint32_t pr = 0;
        bool done = false;
        if (hash0) { // the window loaded with the head
#pragma unroll
            for (int w = 0; w < PW; ++w) {
                if (!done) {
                    const uint4 sl = sw[w];
                    if (sl.w == RX_SLOT_EMPTY) {
                        done = true;
                    } else if (sl.x == h.ka && sl.y == h.kb && sl.z == h.kc) {
                        flow = sl.w;
                        done = true;
                    } else if (++pr >= maxp) {
                        done = true;
                    } else {
                        pj = (pj + 1) & mk;
                    }
                }
            }
        }
        while (!done) { // past the window, or a UDP key on a shared port
            const uint4 sl = ld_slot(tb + pj);
            if (sl.w == RX_SLOT_EMPTY) break;
            if (sl.x == h.ka && sl.y == h.kb && sl.z == h.kc) {
                flow = sl.w;
                break;
            }
            if (++pr >= maxp) break;
            pj = (pj + 1) & mk;
        }
    }
    if constexpr ((ABL & 1) != 0) flow = probe ? (h.kb & 0x3FFu) : RXG_FLOW_NONE;
    if (h.is_tcp && valid && flow == RXG_FLOW_NONE) flow = pe; // listener (prefetched)
    if (h.is_udp)
        rc = flow == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                   : ((flags & RXG_F_UDP_SHORT) ? RXG_RC_UDP_NOMEM : RXG_RC_OK);
    if (rc == RXG_RC_OK ? trunc_ok : trunc) flags |= RXG_F_TRUNC;
    const bool ok = h.l4 && h.stored == ck;
    if (h.is_tcp) {
        if (!ok) flow = RXG_FLOW_NONE;
        rc = !ok ? RXG_RC_TCP_BAD_CKSUM : (flow == RXG_FLOW_NONE ? RXG_RC_TCP_NO_TCB : RXG_RC_OK);
    }
    const uint32_t cidx = valid && rc == RXG_RC_OK && flow != RXG_FLOW_NONE
                              ? (h.is_tcp ? ft.nu : 0u) + flow
                              : 0xFFFFFFFFu;
    if (valid) {
        uint4 vd;
        vd.x = flow;
        vd.y = (poff & 0xFFFFu) | (plen << 16);
        vd.z = ck | (h.cl << 16) | (((uint32_t)rc & 0xFFu) << 24);
        vd.w = (ok ? 1u : 0u) | (flags << 8) | (h.stored << 16);
        if constexpr ((ABL & 32) != 0)
            if (wvu * 64u < (uint32_t)FPB) put_count_idx_wave(ft, p, cidx, lane); // (diagnostic order)
        if constexpr ((ABL & 64) != 0) // diagnostic: no verdict store
            asm volatile("" ::"v"(vd.x), "v"(vd.y), "v"(vd.z), "v"(vd.w));
        else
            st_verdict<WT>(ft, out, p, vd);
        lane_count(cidx, counts, hist, lds_bins);
    }
    if constexpr ((ABL & 48) == 0)
        if (wvu * 64u < (uint32_t)FPB) put_count_idx_wave(ft, p, cidx, lane); // (waves of frames)
    if constexpr (PERS) __syncthreads(); // every LDS read of this block-tile done
    } // block-tiles
    if (lds_bins) {
        __syncthreads();
        for (uint32_t i = tid; i < lds_bins; i += 256) {
            const uint32_t cnt = hist[i];
            if (cnt) atomicAdd(&counts[i], (unsigned long long)cnt);
        }
    }
}

template <int ABL = 0, int PW = 1, uint32_t MAPC = SH_MAPC, bool EP = false, int L = EP ? 3 : 4,
          bool PS = false, int FPB = 256, int TT = 2, bool PERS = false, bool WT = false>
hipError_t launch_sh(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                     uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out,
                     unsigned long long *counts, uint32_t lds_bins, hipStream_t s,
                     const uint32_t *, const uint32_t *) {
    uint64_t blocks = ((uint64_t)n + FPB - 1) / FPB;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (PERS) { // one resident wave of blocks
        int cu = 0, bpc = 0;
        hipError_t e = rx_occupancy(
            reinterpret_cast<const void *>(rx_classify_sh_kernel<ABL, PW, MAPC, EP, L, PS, FPB, TT, PERS, WT>),
            256, (size_t)lds_bins * 4u, &cu, &bpc);
        if (e != hipSuccess) return e;
        const uint64_t res = (uint64_t)cu * (uint64_t)(bpc > 0 ? bpc : 1);
        if (blocks > res) blocks = res;
    }
    if (EP && ((uintptr_t)pkts & 15u)) // LDS-DMA needs 16-B aligned frames: pipe 64 instead
        return launch_sh<ABL, 4, MAPC, false>(pkts, off, len, n, unit_log2, ft, out, counts,
                                              lds_bins, s, nullptr, nullptr);
    hipLaunchKernelGGL((rx_classify_sh_kernel<ABL, PW, MAPC, EP, L, PS, FPB, TT, PERS, WT>), dim3((uint32_t)blocks),
                       dim3(256),
                       (size_t)lds_bins * 4u, s, pkts, off, len, n, unit_log2, ft, out, counts,
                       lds_bins);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// WC kernel (RX_DIAG pipes 80-83; the access-shape experiment of VERDICT r4
// next #7, tools/membw_cfg3.hip): a wave owns F consecutive frames per trip
// and reads their byte span as contiguous 1-KiB wave-instructions (lane l
// loads chunk 64 j + l of the span), where the G=8 group kernel's
// instructions touch 8 frames x 128 B.  Each lane adds its chunks past a
// frame's head (chunks 4.., the last masked at the capture) into that frame's
// partial; a wave reduce per frame gives the tail sums; the frames' head
// chunks 0..3 go through LDS to the frame's owner lane (lane f), which
// parses them, adds the head sum and, as the SH kernel's end of block,
// probes, checks and writes the verdict.  The next trip's span is loaded
// while the probes are in flight (PIPE).  A trip whose frames are not dense
// (out of order, overlapping, a span over 64 * NL chunks), and a frame whose
// checksummed bytes end before its capture, take the generic paths (the whole
// wave per frame; the tail re-summed from HBM by its owner).
template <int F, int NL, bool PIPE>
__global__ __launch_bounds__(256) void rx_classify_wc_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t n, uint32_t unit_log2, rx_ft_dev ft,
    uint4 *__restrict__ out, unsigned long long *__restrict__ counts, uint32_t lds_bins) {
    static_assert(F >= 1 && F <= 8 && NL >= 1 && NL <= 12, "wave tile");
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    __shared__ __attribute__((aligned(16))) uint4 s_hd[4][F][4]; // per wave: head chunks
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    for (uint32_t i = tid; i < lds_bins; i += 256) hist[i] = 0;
    if (lds_bins) __syncthreads();
    const uint64_t ntile = ((uint64_t)n + F - 1) / F;
    const uint64_t nw = (uint64_t)gridDim.x * 4u;
    // a trip's frames, wave-uniform after readlane: frame t*F + f at byte fo[f]
    // (relative to fo[0]), capture cp[f]; dense: the span fits the loads
    struct trip {
        uint64_t t, base;
        uint32_t fo[F];
        int32_t cp[F];
        uint32_t span; // chunks
        bool dense;
    };
    auto desc = [&](uint64_t t, uint32_t &o, int32_t &c) {
        const uint64_t p = t * F + (lane < (uint32_t)F ? lane : 0u);
        const bool v = t < ntile && lane < (uint32_t)F && p < n;
        o = off[v ? p : 0];
        c = v ? (int32_t)len[v ? p : 0] : 0;
    };
    auto geometry = [&](trip &T, uint64_t t, uint32_t o, int32_t c) {
        T.t = t;
        uint64_t pos[F];
        bool ok = t < ntile;
#pragma unroll
        for (int f = 0; f < F; ++f) {
            pos[f] = (uint64_t)__builtin_amdgcn_readlane((int)o, f) << unit_log2;
            T.cp[f] = __builtin_amdgcn_readlane(c, f);
        }
        T.base = pos[0];
        uint64_t end = pos[0];
#pragma unroll
        for (int f = 0; f < F; ++f) {
            const uint64_t e = pos[f] + (uint64_t)((T.cp[f] + 15) & ~15);
            if (T.cp[f] > 0) {
                ok = ok && pos[f] >= end; // in order, no overlap
                end = e;
            }
            T.fo[f] = (uint32_t)((pos[f] - T.base) >> 4);
        }
        const uint64_t sp = (end - T.base) >> 4;
        T.dense = ok && sp <= 64u * NL;
        T.span = T.dense ? (uint32_t)sp : 0u;
    };
    auto load = [&](uint4 (&v)[NL], const trip &T) {
        const uint8_t *b = pkts + T.base;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const uint32_t k = 64u * j + lane;
            v[j] = ldg16<true>(b + ((uint64_t)(k < T.span ? k : 0u) << 4)); // masked at use
        }
    };

    uint64_t t = (uint64_t)blockIdx.x * 4u + wv;
    trip T, N;
    uint4 v[NL], nv[NL];
    {
        uint32_t o;
        int32_t c;
        desc(t, o, c);
        geometry(T, t, o, c);
        load(v, T);
    }
    for (; t < ntile; t += nw) {
        uint32_t no;
        int32_t nc;
        desc(t + nw, no, nc); // the next trip's descriptors, in flight through this one
        // ---- the frames' partial sums (chunks 4..) and head chunks to LDS
        uint32_t ps[F];
#pragma unroll
        for (int f = 0; f < F; ++f) ps[f] = 0;
        if (T.dense) {
            // per chunk: one sum, F range tests; the head chunks (4 of every
            // frame) go to LDS and the one partial last chunk of a frame is
            // masked in a wave-uniform branch, so the common chunk costs
            // about a dozen VALU (an earlier wave-owns-frames kernel masked
            // every chunk and became issue-bound)
#pragma unroll
            for (int j = 0; j < NL; ++j) {
                const uint32_t k = 64u * j + lane;
                const uint32_t cs = k < T.span ? chunk_sum(v[j]) : 0u;
                bool part = false;
#pragma unroll
                for (int f = 0; f < F; ++f) {
                    const uint32_t r = k - T.fo[f]; // chunk of frame f (wraps below it)
                    const uint32_t nfull = (uint32_t)T.cp[f] >> 4;
                    ps[f] += (r - 4u < nfull - 4u && nfull > 4u) ? cs : 0u; // r in [4, nfull)
                    if (r < 4u && r < (((uint32_t)T.cp[f] + 15u) >> 4)) s_hd[wv][f][r] = v[j];
                    part = part || (r == nfull && r >= 4u && (T.cp[f] & 15));
                }
                if (__ballot(part) != 0ull) { // (wave-uniform) a frame's partial last chunk
#pragma unroll
                    for (int f = 0; f < F; ++f) {
                        const uint32_t r = k - T.fo[f];
                        const uint32_t nfull = (uint32_t)T.cp[f] >> 4;
                        if (r == nfull && r >= 4u && (T.cp[f] & 15))
                            ps[f] = lane_chunk_sum(ps[f], v[j], 16 * (int32_t)r, T.cp[f]);
                    }
                }
            }
        }
#pragma unroll
        for (int f = 0; f < F; ++f) ps[f] = gsum<64>(ps[f]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- owner lane f: parse, sums, probe loads
        const uint32_t fl = lane < (uint32_t)F ? lane : 0u;
        int32_t cp = 0;
        uint32_t tail = 0;
#pragma unroll
        for (int f = 0; f < F; ++f)
            if (fl == (uint32_t)f) cp = T.cp[f], tail = ps[f];
        const uint64_t p = t * F + fl;
        const bool valid = lane < (uint32_t)F && t < ntile && p < n;
        const uint8_t *fb = pkts + ((uint64_t)off[valid ? p : 0] << unit_log2);
        uint4 c[4];
        if (T.dense) {
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = chunk_below(s_hd[wv][fl][k], 16 * k, cp);
        }
        if (!T.dense) { // (wave-uniform) heads from HBM
#pragma unroll
            for (int k = 0; k < 4; ++k)
                c[k] = chunk_below(ldg16<false>(valid && 16 * k < cp ? fb + 16 * k : pkts), 16 * k, cp);
        }
        const sh_head h = sh_parse(c, cp);
        uint32_t acc = sh_head_sum(c, h);
        const int32_t e = h.e;
        const bool resum = h.do_sum && e > 64 && (!T.dense || e != cp);
        if (h.do_sum && e > 64 && !resum) acc += tail;
        if (__ballot(valid && resum) != 0ull) { // rare (wave-uniform branch): the tail from HBM
            if (valid && resum)
                for (int32_t s = 64; s < e; s += 16) acc = lane_chunk_sum(acc, ldg16<false>(fb + s), s, e);
        }
        // probe loads: the port entry and the hashed table's 4-slot window
        const bool probe = valid && h.l4;
        const uint32_t maxp = h.is_udp ? ft.udp_probe : ft.tcp_probe;
        const bool probe0 = probe && maxp > 0;
        const bool udp_port = h.is_udp && ft.udp_port != nullptr;
        const bool hash0 = probe0 && !udp_port;
        const uint32_t *ptab = udp_port ? ft.udp_port : ft.listen;
        const uint32_t dport = h.is_udp ? h.kb : (h.kc >> 16);
        const uint32_t pe = probe ? ptab[dport] : RXG_FLOW_NONE;
        constexpr int PW = 4;
        uint32_t pj = rx_hash3s(ft.hseed, h.ka, h.kb, h.kc) & (h.is_udp ? ft.udp_mask : ft.tcp_mask);
        const uint4 *tb = h.is_udp ? ft.udp : ft.tcp;
        uint4 sw[PW];
#pragma unroll
        for (int w = 0; w < PW; ++w) sw[w] = ld_slot(hash0 ? tb + pj + w : reinterpret_cast<const uint4 *>(pkts));
        // the next trip's span, in flight while the probes return
        if constexpr (PIPE) {
            geometry(N, t + nw, no, nc);
            load(nv, N);
        }
        // ---- verdict
        uint32_t ck = 0;
        if (h.do_sum) {
            ck = (~fold16(acc)) & 0xFFFFu;
            if (ck == 0u && h.proto == 17u) ck = 0xFFFFu;
        }
        uint32_t flags = 0, poff = 0, plen = 0;
        if (h.is_udp) {
            poff = 42;
            plen = h.dgl > 8u ? h.dgl - 8u : 0u;
            if (h.dgl <= 8u) flags |= RXG_F_UDP_SHORT;
        } else if (h.is_tcp) {
            const int32_t pl = (int32_t)h.tl - 20 - 4 * (int32_t)h.hl;
            poff = 34u + 4u * h.hl;
            if (pl < 0) flags |= RXG_F_TCP_NEGLEN;
            plen = pl < 0 ? 0u : (uint32_t)pl;
        }
        const bool trunc = (int32_t)h.nd > cp;
        const bool trunc_ok = trunc || (h.is_udp && (int32_t)(42u + plen) > cp);
        uint32_t flow = RXG_FLOW_NONE;
        int32_t rc = RXG_RC_KNI;
        bool hashed = probe0;
        if (probe0 && udp_port) hashed = !rx_udp_port_decide(pe, h.ka, ft.udp_dip, &flow);
        if (hashed) {
            const uint32_t mk = h.is_udp ? ft.udp_mask : ft.tcp_mask;
            uint32_t pr = 0;
            bool done = false;
            if (hash0) {
#pragma unroll
                for (int w = 0; w < PW; ++w) {
                    if (!done) {
                        const uint4 sl = sw[w];
                        if (sl.w == RX_SLOT_EMPTY) {
                            done = true;
                        } else if (sl.x == h.ka && sl.y == h.kb && sl.z == h.kc) {
                            flow = sl.w;
                            done = true;
                        } else if (++pr >= maxp) {
                            done = true;
                        } else {
                            pj = (pj + 1) & mk;
                        }
                    }
                }
            }
            while (!done) { // past the window, or a UDP key on a shared port
                const uint4 sl = ld_slot(tb + pj);
                if (sl.w == RX_SLOT_EMPTY) break;
                if (sl.x == h.ka && sl.y == h.kb && sl.z == h.kc) {
                    flow = sl.w;
                    break;
                }
                if (++pr >= maxp) break;
                pj = (pj + 1) & mk;
            }
        }
        if (h.is_tcp && valid && flow == RXG_FLOW_NONE) flow = pe; // listener
        if (h.is_udp)
            rc = flow == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                       : ((flags & RXG_F_UDP_SHORT) ? RXG_RC_UDP_NOMEM : RXG_RC_OK);
        if (rc == RXG_RC_OK ? trunc_ok : trunc) flags |= RXG_F_TRUNC;
        const bool ok = h.l4 && h.stored == ck;
        if (h.is_tcp) {
            if (!ok) flow = RXG_FLOW_NONE;
            rc = !ok ? RXG_RC_TCP_BAD_CKSUM : (flow == RXG_FLOW_NONE ? RXG_RC_TCP_NO_TCB : RXG_RC_OK);
        }
        if (valid) {
            const uint32_t cidx =
                rc == RXG_RC_OK && flow != RXG_FLOW_NONE ? (h.is_tcp ? ft.nu : 0u) + flow : 0xFFFFFFFFu;
            uint4 vd;
            vd.x = flow;
            vd.y = (poff & 0xFFFFu) | (plen << 16);
            vd.z = ck | (h.cl << 16) | (((uint32_t)rc & 0xFFu) << 24);
            vd.w = (ok ? 1u : 0u) | (flags << 8) | (h.stored << 16);
            st_verdict(ft, out, p, vd);
            lane_count(cidx, counts, hist, lds_bins);
            if (ft.count_idx) put_count_idx(ft, p, cidx);
        }
        if constexpr (PIPE) {
            T = N;
#pragma unroll
            for (int j = 0; j < NL; ++j) v[j] = nv[j];
        } else {
            geometry(T, t + nw, no, nc);
            load(v, T);
        }
        // (the next trip's LDS head writes follow this trip's reads in the wave's order)
        __builtin_amdgcn_wave_barrier();
    }
    if (lds_bins) {
        __syncthreads();
        for (uint32_t i = tid; i < lds_bins; i += 256) {
            const uint32_t cnt = hist[i];
            if (cnt) atomicAdd(&counts[i], (unsigned long long)cnt);
        }
    }
}

template <int F, int NL, bool PIPE>
hipError_t launch_wc(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                     uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out, unsigned long long *counts,
                     uint32_t lds_bins, hipStream_t s, const uint32_t *, const uint32_t *) {
    const size_t lds = (size_t)lds_bins * 4u;
    int cu = 0, bpc = 0;
    hipError_t e = rx_occupancy(reinterpret_cast<const void *>(rx_classify_wc_kernel<F, NL, PIPE>), 256,
                                lds, &cu, &bpc);
    if (e != hipSuccess) return e;
    uint64_t occ = (uint64_t)bpc;
    if (ft.bpc_cap && occ > ft.bpc_cap) occ = ft.bpc_cap;
    const uint64_t waves = ((uint64_t)n + F - 1) / F;
    uint64_t blocks = (uint64_t)cu * occ;
    if (blocks * 4 > waves) blocks = (waves + 3) / 4;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL((rx_classify_wc_kernel<F, NL, PIPE>), dim3((uint32_t)blocks), dim3(256), lds, s,
                       pkts, off, len, n, unit_log2, ft, out, counts, lds_bins);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-flow counts for 8192 < flows <= 2M (too many for a per-block LDS
// histogram at full occupancy, and scattered 8-B global atomics each cost one
// memory-side request): the classify kernel writes one count index per frame
// (ft.count_idx: 2 B when the flows fit one 65536-flow range, else 4 B), and
// a slab histogram sums them.  A 2-B index of all ones is a frame not counted
// (flow 65535 of exactly 65536 is counted by the classify kernel itself,
// rx_ft_dev::count_ffff).  Pass 1: block b (1024 threads, one per CU: 128
// KiB of LDS) adds the indices of its share of the frames that fall in its
// 65536-flow range (blockIdx.y) into 16-bit LDS bins, two per dword (lo =
// even flow, hi = odd), and writes the bins out as slab b.  A bin overflows
// only when more than 65535 of the block's frames are one flow: the sum of the
// bins then differs from the block's exact tally of counted frames (each wrap
// loses 65535 or 65536), and the block zeroes its slab and adds its frames
// with global atomics instead (pathological traffic only).  Pass 2: a thread
// per 4 bin pairs sums that column over the slabs (16-B loads) and adds it to
// counts.
constexpr uint32_t SLAB_MAX_FLOWS = 65536;
constexpr uint32_t SLAB_MIN_FLOWS = 8193;   // below: LDS histogram in the classify kernel

template <typename T> // count index: uint16_t (one range, <= 65536 flows) or uint32_t
__global__ __launch_bounds__(1024) void rx_count_slab_kernel(const T *__restrict__ cidx,
                                                              uint32_t n, uint32_t per,
                                                              uint32_t words, uint32_t nflows,
                                                              uint32_t *__restrict__ slab,
                                                              unsigned long long *__restrict__ counts) {
    constexpr uint32_t E = 16 / sizeof(T); // indices per 16-B load
    // blockIdx.y = flow range: flows [y * 65536, y * 65536 + lim)
    __shared__ uint32_t bins[SLAB_MAX_FLOWS / 2];
    __shared__ uint32_t tally, sum;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < words; i += 1024) bins[i] = 0;
    if (tid == 0) tally = sum = 0;
    __syncthreads();
    const uint32_t f0 = blockIdx.y * SLAB_MAX_FLOWS;
    const uint32_t lim = min(nflows - f0, SLAB_MAX_FLOWS);
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = min((uint64_t)n, b0 + per);
    uint32_t mine = 0;
    auto count = [&](uint32_t x) {
        const uint32_t f = x - f0; // not counted (all ones) and other ranges: f >= lim
        if (f < lim) {
            atomicAdd(&bins[f >> 1], 1u << (16u * (f & 1u)));
            ++mine;
        }
    };
    // a 2-B all-ones index is never counted here: with fewer than 65536 flows
    // it is no flow, and with exactly 65536 flow 65535 was counted by the
    // classify kernel (rx_ft_dev::count_ffff)
    auto index_of = [&](uint32_t x) -> uint32_t {
        if constexpr (sizeof(T) == 2)
            if (x == 0xFFFFu) return ~0u;
        return x;
    };
    // 4E indices per thread per trip (four 16-B loads in flight); b0 is a
    // multiple of 8 (per is), so the vector loads are aligned
    uint64_t i = b0 + (uint64_t)E * tid;
    for (; i + (uint64_t)E * 3 * 1024 + E - 1 < b1; i += (uint64_t)E * 4 * 1024) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = ldg16<true>(reinterpret_cast<const uint8_t *>(cidx + i + (uint64_t)u * E * 1024));
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if constexpr (sizeof(T) == 2) {
                    count(index_of(w[j] & 0xFFFFu));
                    count(index_of(w[j] >> 16));
                } else {
                    count(w[j]);
                }
            }
        }
    }
    for (; i < b1; i += (uint64_t)E * 1024)
        for (uint64_t k = i; k < i + E && k < b1; ++k) count(index_of(cidx[k]));
    if (mine) atomicAdd(&tally, mine);
    __syncthreads();
    uint32_t part = 0;
    for (uint32_t k = tid; k < words; k += 1024) part += (bins[k] & 0xFFFFu) + (bins[k] >> 16);
    if (part) atomicAdd(&sum, part);
    __syncthreads();
    const bool wrapped = sum != tally; // block-uniform
    uint32_t *dst = slab + ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * words;
    // non-temporal: 32 MiB of slabs through the L2 would evict the flow tables
    // the next burst's classify probes
    for (uint32_t k = tid; k < words; k += 1024) __builtin_nontemporal_store(wrapped ? 0u : bins[k], &dst[k]);
    if (wrapped)
        for (uint64_t k = b0 + tid; k < b1; k += 1024) {
            const uint32_t f = index_of(cidx[k]) - f0;
            if (f < lim) atomicAdd(&counts[(uint64_t)f0 + f], 1ull);
        }
}

// block = 64 lanes x 4 bin pairs (one 16-B column piece per lane) x 16 waves,
// wave w summing slabs w, w + 16, ... with 4 loads in flight; the 16 partial
// sums meet in LDS.  words is a multiple of 4 (slab_words).  (Splitting the
// slabs over 4x the blocks, adding with u64 atomics, was 7 us slower at cfg4:
// profiles/r02f/ab_count_paths.txt.)
__global__ __launch_bounds__(1024) void rx_count_reduce_kernel(const uint32_t *__restrict__ slab,
                                                                uint32_t nslabs, uint32_t words,
                                                                uint32_t nflows,
                                                                unsigned long long *__restrict__ counts) {
    __shared__ uint4 part[2][16][64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    // blockIdx.y = flow range (its slabs, its 65536 counts)
    slab += (uint64_t)blockIdx.y * nslabs * words;
    counts += (uint64_t)blockIdx.y * SLAB_MAX_FLOWS;
    nflows -= blockIdx.y * SLAB_MAX_FLOWS;
    const uint32_t w = (blockIdx.x * 64 + lane) * 4; // first of this lane's 4 words
    const uint32_t wc = w < words ? w : 0;
    uint4 lo = make_uint4(0, 0, 0, 0), hi = lo;
    auto add = [&](uint4 x) {
        lo.x += x.x & 0xFFFFu, hi.x += x.x >> 16;
        lo.y += x.y & 0xFFFFu, hi.y += x.y >> 16;
        lo.z += x.z & 0xFFFFu, hi.z += x.z >> 16;
        lo.w += x.w & 0xFFFFu, hi.w += x.w >> 16;
    };
    uint32_t b = wv;
    for (; b + 16 * 3 < nslabs; b += 16 * 4) {
        uint4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            x[u] = ldg16<true>(reinterpret_cast<const uint8_t *>(slab + (uint64_t)(b + 16 * u) * words + wc));
#pragma unroll
        for (int u = 0; u < 4; ++u) add(x[u]);
    }
    for (; b < nslabs; b += 16)
        add(ldg16<true>(reinterpret_cast<const uint8_t *>(slab + (uint64_t)b * words + wc)));
    part[0][wv][lane] = lo;
    part[1][wv][lane] = hi;
    __syncthreads();
    if (wv == 0 && w < words) {
        lo = hi = make_uint4(0, 0, 0, 0);
#pragma unroll 4 // (fully unrolled it spilled 8 VGPRs at the 1024-thread budget)
        for (int k = 0; k < 16; ++k) {
            const uint4 a = part[0][k][lane], c = part[1][k][lane];
            lo.x += a.x, lo.y += a.y, lo.z += a.z, lo.w += a.w;
            hi.x += c.x, hi.y += c.y, hi.z += c.z, hi.w += c.w;
        }
        const uint32_t l[4] = {lo.x, lo.y, lo.z, lo.w}, h[4] = {hi.x, hi.y, hi.z, hi.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t f = 2 * (w + k);
            if (l[k] && f < nflows) counts[f] += l[k];
            if (h[k] && f + 1 < nflows) counts[f + 1] += h[k];
        }
    }
}

// few slabs (the multi-range geometry): one thread per 4 bin pairs sums every
// slab of its range, 8 loads in flight; 256-thread blocks of 1024 pairs
__global__ __launch_bounds__(256) void rx_count_reduce_few_kernel(
    const uint32_t *__restrict__ slab, uint32_t nslabs, uint32_t words, uint32_t nflows,
    unsigned long long *__restrict__ counts) {
    slab += (uint64_t)blockIdx.y * nslabs * words;
    counts += (uint64_t)blockIdx.y * SLAB_MAX_FLOWS;
    nflows -= blockIdx.y * SLAB_MAX_FLOWS;
    const uint32_t w = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (w >= words) return;
    uint32_t l[4] = {0, 0, 0, 0}, h[4] = {0, 0, 0, 0};
    uint32_t b = 0;
    for (; b + 8 <= nslabs; b += 8) {
        uint4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            x[u] = ldg16<true>(reinterpret_cast<const uint8_t *>(slab + (uint64_t)(b + u) * words + w));
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            l[0] += x[u].x & 0xFFFFu, h[0] += x[u].x >> 16;
            l[1] += x[u].y & 0xFFFFu, h[1] += x[u].y >> 16;
            l[2] += x[u].z & 0xFFFFu, h[2] += x[u].z >> 16;
            l[3] += x[u].w & 0xFFFFu, h[3] += x[u].w >> 16;
        }
    }
    for (; b < nslabs; ++b) {
        const uint4 x = ldg16<true>(reinterpret_cast<const uint8_t *>(slab + (uint64_t)b * words + w));
        l[0] += x.x & 0xFFFFu, h[0] += x.x >> 16;
        l[1] += x.y & 0xFFFFu, h[1] += x.y >> 16;
        l[2] += x.z & 0xFFFFu, h[2] += x.z >> 16;
        l[3] += x.w & 0xFFFFu, h[3] += x.w >> 16;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t f = 2 * (w + k);
        if (l[k] && f < nflows) counts[f] += l[k];
        if (h[k] && f + 1 < nflows) counts[f + 1] += h[k];
    }
}

// Flows above 65536: the count is split into ranges of 65536 flows
// (blockIdx.y), each range's blocks scanning every index; up to
// SLAB_MAX_RANGES ranges, beyond that global atomics in the classify kernel.
constexpr uint32_t SLAB_MAX_RANGES = 32;

static uint32_t slab_ranges(const rx_ft_dev &ft) {
    return (ft.nu + ft.nt + SLAB_MAX_FLOWS - 1) / SLAB_MAX_FLOWS;
}

// 16-bit bin pairs per slab (a multiple of 4): all flows for one range, a
// whole range otherwise
static uint32_t slab_words(const rx_ft_dev &ft) {
    return slab_ranges(ft) > 1 ? SLAB_MAX_FLOWS / 2 : (((ft.nu + ft.nt + 1) / 2 + 3) & ~3u);
}

// slab geometry: about one 1024-thread block per CU in all (256 blocks over
// the ranges), >= 16384 frames per slab so the slabs stay small beside the
// indices, a multiple of 4 frames (aligned 16-B index loads)
static void slab_geometry(uint32_t n, uint32_t nranges, uint32_t *nslabs, uint32_t *per,
                          uint32_t div_log2 = 0) {
    const uint64_t want = std::max<uint64_t>(1, (256u >> div_log2) / nranges);
    uint64_t pr = std::max<uint64_t>(((uint64_t)n + want - 1) / want, 16384);
    pr = (pr + 7) & ~7ull;
    const uint64_t nb = ((uint64_t)n + pr - 1) / pr;
    *nslabs = (uint32_t)(nb ? nb : 1);
    *per = (uint32_t)pr;
}

static bool use_slab(const rx_ft_dev &ft, bool counts) {
    const uint32_t nf = ft.nu + ft.nt;
    return counts && nf >= SLAB_MIN_FLOWS && nf <= SLAB_MAX_FLOWS * SLAB_MAX_RANGES;
}

// u16 count indices: the flows fit one range
static bool cidx16(const rx_ft_dev &ft) { return ft.nu + ft.nt <= SLAB_MAX_FLOWS; }

static hipError_t launch_count_slab(const void *cidx, uint32_t n, const rx_ft_dev &ft,
                                    unsigned long long *counts, uint32_t *slab, hipStream_t s) {
    const uint32_t nr = slab_ranges(ft), words = slab_words(ft), nf = ft.nu + ft.nt;
    uint32_t nslabs, per;
    slab_geometry(n, nr, &nslabs, &per, ft.slab_div_log2);
    if (ft.cidx16)
        hipLaunchKernelGGL(rx_count_slab_kernel<uint16_t>, dim3(nslabs, nr), dim3(1024), 0, s,
                           static_cast<const uint16_t *>(cidx), n, per, words, nf,
                           slab, counts);
    else
        hipLaunchKernelGGL(rx_count_slab_kernel<uint32_t>, dim3(nslabs, nr), dim3(1024), 0, s,
                           static_cast<const uint32_t *>(cidx), n, per, words, nf,
                           slab, counts);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (nslabs <= 64)
        hipLaunchKernelGGL(rx_count_reduce_few_kernel, dim3((words / 4 + 255) / 256, nr), dim3(256),
                           0, s, slab, nslabs, words, nf, counts);
    else
        hipLaunchKernelGGL(rx_count_reduce_kernel, dim3((words / 4 + 63) / 64, nr), dim3(1024), 0,
                           s, slab, nslabs, words, nf, counts);
    return hipGetLastError();
}

typedef hipError_t (*launch_fn)(const uint8_t *, const uint32_t *, const uint16_t *, uint32_t,
                                uint32_t, const rx_ft_dev &, uint4 *, unsigned long long *,
                                uint32_t, hipStream_t, const uint32_t *, const uint32_t *);
struct variant_entry {
    uint32_t g, p, fpg, pipe;
    launch_fn fn;
    uint32_t bpc; // default resident blocks per CU (0 = occupancy), from measurement
};
// every compiled variant; the first entry per lanes-per-frame g is its default.
// g = 1 (one frame per lane): p = 4 chunks up front, pipe = prefetch mode
// (0 none, 1 descriptors + frame one trip ahead, 2 = 1 capped at 6 waves/SIMD,
// 3 descriptors only, 4 = 0 with plain verdict stores, 5/6 = 0/4 with plain
// frame loads, 7/8 = 1/2 with plain frame loads, 9/10 = ordered one-trip
// descriptor prefetch + deferred store, nt / plain store); g >= 4: pipe 0/1 = no /
// one-trip pipeline, 2/3 = 0/1 with plain frame loads; pipe >= 100 are
// diagnostic ablations (wrong verdicts by construction, tuning only).
static const variant_entry k_variants[] = {
    // The product table: the four defaults (rx_pick_variant) and the measured
    // alternatives next to them, every one parity-tested (tests/
    // test_gpu_parity.py runs each).  Experiment variants whose sweeps are
    // recorded in profiles/ and DESIGN.md were removed from the code;
    // diagnostic ablations (wrong verdicts or counts by construction) and the
    // shapes kept for tuning compile only into the RX_DIAG build
    // (librxgpu_diag.so, Makefile), so no public call on the product library
    // can return a verdict that differs from the reference's (common.c:97-108,
    // tcp.c:345-371: the contract every entry keeps).
    // pipe 12 at 4 blocks/CU: with per-flow counts its LDS (stage + UDP table +
    // histogram) allows 4 anyway; without counts 5 fit and ran 36% slower
    // (r01g: 0.255 vs 0.346 ms on cfg2, profiles/r01g/sweep_lane_bpc_counts.txt)
    {1, 4, 1, 12, launch_lane_udpc<12, 0, true, false>, 4},
    // 5: per-lane head loads, LDS UDP table (the binned path's small-frame kernel)
    {1, 4, 1, 5, launch_lane_udpc<0, 0, true, false>, 6},
    // 14 (the 64-B default): 12 software-pipelined (descriptors two trips,
    // frame bytes one trip ahead)
    {1, 4, 1, 14, launch_lane_udpc<14, 0, true, false>, 2},
    // 19: two adjacent 256-frame tiles per trip, both tiles' frame bytes
    // issued at the top of the trip, descriptors one trip ahead (the
    // byte-pattern ceiling's shape); 25 (the 64-B default from round 6): the
    // same with the trip's two tiles a grid stride apart, 0.2242-0.2248 vs
    // 0.2263-0.2268 ms per step for 19 (profiles/r06az)
    {1, 4, 1, 19, launch_lane_udpc<19, 0, true, false>, 2},
    {1, 4, 1, 25, launch_lane_udpc<25, 0, true, false>, 2},
    // 16 (the 64-B default for 8-B verdicts): 14 with lane_verdict_fast, 18%
    // fewer vector and half the scalar instructions; with 16-B verdicts the
    // same time as 14 (the stores bound it: profiles/r06ab, r06ac), with
    // 8-B verdicts 79.0-79.5 vs 76.2-77.4 Gpps for 14 (profiles/r06ak)
    {1, 4, 1, 16, launch_lane_udpc<16, 0, true, false>, 2},
    {1, 4, 1, 0, launch_lane<0>},
    // group kernels, one per G (the first entry per g is its default)
    {4, 1, 1, 1, launch_v<4, 1, 1, 1>},
    {8, 2, 2, 0, launch_v<8, 2, 2, 0>},
    // 40 (the 1500-B default): G=8 with write-through verdict stores (sc1:
    // the lines leave the L2 instead of staying in it)
    {8, 2, 2, 40, launch_v<8, 2, 2, 0, true, 0, 1, true>},
    // 41 / 42: 40 write-batched (WB): each block owns contiguous tiles and
    // writes the verdicts of 16 / 32 of them (16 / 32 KiB) at once (sc1)
    {8, 2, 2, 41, launch_v<8, 2, 2, 0, true, 0, 1, true, 16>},
    {8, 2, 2, 42, launch_v<8, 2, 2, 0, true, 0, 1, true, 32>},
    // 48 (the 1500-B default): 24 tiles per batch with the per-block histogram
    // in 16-bit bin pairs (32 KiB of LDS at 4097 flows, as 41's), the 32-bit
    // histogram when a block's share reaches 65536 frames
    {8, 2, 2, 48, launch_v<8, 2, 2, 0, true, 0, 1, true, 24, true>},
    {8, 2, 1, 0, launch_v<8, 2, 1, 0>},
    {16, 2, 2, 0, launch_v<16, 2, 2, 0>},
    {32, 3, 2, 0, launch_v<32, 3, 2, 0>},
    {64, 4, 1, 0, launch_v<64, 4, 1, 0>},
    // g = 0: stream kernel (head per lane, tails streamed per block); 30: nt
    // tail loads; 38: probe after the stream, one barrier per tail tile (B1);
    // 738 / 938 (the jumbo default): 38 with 32 / 16 frames per block
    {0, 1, 1, 30, launch_stream<true>},
    {0, 1, 1, 38, launch_stream<true, 0, 3, 1, true>},
    {0, 1, 1, 738, launch_stream<true, 0, 3, 1, true, false, false, 32>},
    {0, 1, 1, 938, launch_stream<true, 0, 3, 1, true, false, false, 16>},
    // SH kernel (heads taken out of the block stream): 60; 64: a four-slot
    // first probe window; 67 (the IMIX default): 64 with 8-KiB tiles
    {0, 1, 1, 60, launch_sh<0>},
    {0, 1, 1, 64, launch_sh<0, 4>},
    {0, 1, 1, 67, launch_sh<0, 4, SH_MAPC, false, 2>},
#if RX_DIAG
    // ---- tuning shapes (correct verdicts; sweeps in profiles/) ----
    {1, 4, 1, 13, launch_lane<12, 0, true, false>, 6}, // 12 without the LDS UDP table
    // two adjacent tiles per trip (19, the 64-B default) with
    // lane_verdict_fast: 0.2326 vs 0.2240 ms for 19 (profiles/r06ad)
    {1, 4, 1, 18, launch_lane_udpc<18, 0, true, false>, 2},
    {1, 4, 1, 23, launch_lane_udpc<23, 0, true, false>, 2}, // 19, both tiles' stores at the trip's end
    {1, 4, 1, 24, launch_lane_udpc<24, 0, true, false>, 2}, // 19, next descriptors before the frames
    {1, 4, 1, 21, launch_lane_udpc<21, 0, true, false>, 2}, // three tiles per trip
    {1, 4, 1, 22, launch_lane_udpc<22, 0, true, false>, 2}, // four
    {8, 2, 2, 1, launch_v<8, 2, 2, 1>},
    {16, 2, 1, 0, launch_v<16, 2, 1, 0>},
    // write-batched G=8 around pipe 41 (WB 16, sc1): WB 8 / 12 / 24 (sc1), 16 (nt)
    {8, 2, 2, 43, launch_v<8, 2, 2, 0, true, 0, 1, true, 8>},
    {8, 2, 2, 44, launch_v<8, 2, 2, 0, true, 0, 1, true, 12>},
    {8, 2, 2, 45, launch_v<8, 2, 2, 0, true, 0, 1, false, 16>},
    {8, 2, 2, 46, launch_v<8, 2, 2, 0, true, 0, 1, true, 24>},
    // ... with a 16-bit histogram (half its LDS): WB 16 / 32 (24: pipe 48, the default)
    {8, 2, 2, 47, launch_v<8, 2, 2, 0, true, 0, 1, true, 16, true>},
    {8, 2, 2, 49, launch_v<8, 2, 2, 0, true, 0, 1, true, 32, true>},
    // ... five blocks per CU: pipe 48 needs 103 VGPRs and 32,784 B of LDS at
    // 4097 flows (both just above a fifth of the CU), so it runs 4 per CU.
    // WB 23 / 20 with the register budget of 5 blocks (MINW 5: <= 96 VGPRs)
    // fit 5; WB 23 at 4 blocks isolates the batch depth
    {8, 2, 2, 50, launch_v<8, 2, 2, 0, true, 0, 5, true, 23, true>},
    {8, 2, 2, 51, launch_v<8, 2, 2, 0, true, 0, 5, true, 20, true>},
    {8, 2, 2, 52, launch_v<8, 2, 2, 0, true, 0, 1, true, 23, true>},
    {8, 2, 2, 53, launch_v<8, 2, 2, 0, true, 0, 5, true, 16, true>},
    // pipe 48 with the remaining passes of both frames loaded together, 2 / 4
    // / 10 per frame per batch (RI)
    {8, 2, 2, 54, launch_v<8, 2, 2, 0, true, 2, 1, true, 24, true>},
    {8, 2, 2, 55, launch_v<8, 2, 2, 0, true, 4, 1, true, 24, true>},
    {8, 2, 2, 56, launch_v<8, 2, 2, 0, true, 10, 1, true, 24, true>},
    {0, 1, 1, 54, launch_stream<true, 0, 3, 1, true, false, true>}, // heads gathered 4 lanes/head
    {0, 1, 1, 66, launch_sh<0, 4, SH_MAPC, false, 3>},              // 12-KiB tiles
    {0, 1, 1, 68, launch_sh<0, 4, SH_MAPC, false, 2, true>},        // partial sums in the stream
    {0, 1, 1, 75, launch_sh<0, 2, SH_MAPC, false, 2>},              // two-slot window
    {0, 1, 1, 65, launch_sh<0, 2, SH_MAPC, true>},                  // probes inside the stream
    // ---- ablations: wrong verdicts (or counts) by construction ----
    // lane kernel (ABL bits: 1 = no bucket probe, 4 = no verdict store, 8 = no
    // checksum arithmetic): 101, 104, 108, 113 = 1|4|8; 2xx: the same with
    // plain frame loads at 6 blocks/CU
    {1, 4, 1, 101, launch_lane<0, 1>},     {1, 4, 1, 104, launch_lane<0, 4>},
    {1, 4, 1, 108, launch_lane<0, 8>},     {1, 4, 1, 113, launch_lane<0, 13>},
    {1, 4, 1, 201, launch_lane<0, 1, true, false>, 6}, {1, 4, 1, 204, launch_lane<0, 4, true, false>, 6},
    {1, 4, 1, 213, launch_lane<0, 13, true, false>, 6},
    // the 64-B default (pipe 14) with the same ablations (round 6): 1401 no
    // probe, 1404 no verdict store, 1408 no checksum arithmetic, 1413 = all three
    {1, 4, 1, 1401, launch_lane_udpc<14, 1, true, false>, 2},
    {1, 4, 1, 1404, launch_lane_udpc<14, 4, true, false>, 2},
    {1, 4, 1, 1408, launch_lane_udpc<14, 8, true, false>, 2},
    {1, 4, 1, 1413, launch_lane_udpc<14, 13, true, false>, 2},
    {1, 4, 1, 1604, launch_lane_udpc<16, 4, true, false>, 2}, // pipe 16, no verdict store
    // stream kernel: no flow probe (130); pipe 46 (span from the descriptors)
    // and its ablations: no probe (146), no tail stream (246), no head loads
    // (446), neither heads nor stream (646); pipe 38: no head loads (438), no
    // partial-chunk load (838), neither (1238)
    {0, 1, 1, 130, launch_stream<true, 1>},
    {0, 1, 1, 46, launch_stream<true, 0, 3, 1, true, true>},
    {0, 1, 1, 146, launch_stream<true, 1, 3, 1, true, true>},
    {0, 1, 1, 246, launch_stream<true, 2, 3, 1, true, true>},
    {0, 1, 1, 446, launch_stream<true, 4, 3, 1, true, true>},
    {0, 1, 1, 646, launch_stream<true, 6, 3, 1, true, true>},
    {0, 1, 1, 438, launch_stream<true, 4, 3, 1, true>}, {0, 1, 1, 838, launch_stream<true, 8, 3, 1, true>},
    {0, 1, 1, 1238, launch_stream<true, 12, 3, 1, true>},
    // SH kernel: no flow probe (160); every partial last chunk from HBM after
    // the stream (264); no count-index store (1064: counts wrong); the count
    // index stored before the verdict (2064)
    {0, 1, 1, 160, launch_sh<1>}, {0, 1, 1, 264, launch_sh<2, 4>},
    {0, 1, 1, 1064, launch_sh<16, 4>}, {0, 1, 1, 2064, launch_sh<32, 4>},
    // 167: 67 without the flow probe
    {0, 1, 1, 167, launch_sh<1, 4, SH_MAPC, false, 2>},
    // pipe 67 without the count-index store (1667) / the verdict store (6467)
    {0, 1, 1, 1667, launch_sh<16, 4, SH_MAPC, false, 2>},
    {0, 1, 1, 6467, launch_sh<64, 4, SH_MAPC, false, 2>},
    // ---- the wave-contiguous shape (WC kernel): F frames per wave trip, NL
    // loads per lane; 80 / 81: F = 2, NL = 3 (1.5-KiB slots) with / without
    // the next trip's span in flight; 82 / 83: F = 4, NL = 6
    {0, 1, 1, 80, launch_wc<2, 3, true>}, {0, 1, 1, 81, launch_wc<2, 3, false>},
    {0, 1, 1, 82, launch_wc<4, 6, true>}, {0, 1, 1, 83, launch_wc<4, 6, false>},
#endif
};

} // namespace

// Default variant per typical frame length (measured on MI355X with
// bench.py --sweep, interleaved rounds).  Any frame length works
// with any variant (frames longer than P passes take the remainder loop); the
// choice only moves speed.
#if !RX_V8
void rx_pick_variant(uint32_t len_hint, uint32_t *g, uint32_t *p, uint32_t *fpg, uint32_t *pipe,
                     bool v8) {
    if (len_hint == 0) len_hint = 1518;
    if (len_hint <= 64) { // cfg2: 64 B; LDS-staged coalesced loads (0.258 vs 0.280 ms, r01b),
        // software-pipelined one trip ahead (pipe 14: 0.2487-0.2506 vs 0.2641-0.2660 ms for
        // pipe 12 at 3 blocks/CU, r02i); with the LDS port window the two tie within 1%
        // and pipe 14 is best at 2 blocks/CU (0.2328-0.2343 vs 0.2346-0.2352 for pipe 12 at
        // 4-6, r02m, r02o); two adjacent tiles per trip with both tiles' bytes issued at the
        // top (pipe 19): 0.2271 vs 0.2346 ms in an interleaved sweep, 0.2270-0.2277 vs
        // 0.2355-0.2361 per step across alternating processes (profiles/r06ae); 3 / 4
        // tiles per trip 0.2364 / 0.2396, 19 at 3 blocks/CU 0.2393.  With 8-B verdicts
        // (rxg_classify_dev8) the one-tile pipeline stays ahead, 14 at 77.6-77.7 vs
        // 72.9-73.2 Gpps for 19 (profiles/r06ai), and 14 with the straight-line verdict
        // (16) at 79.0-79.5 vs 76.2-77.4 (profiles/r06ak)
        // The trip's two tiles a grid stride apart instead of adjacent (pipe 25): 0.2242-
        // 0.2248 vs 0.2263-0.2268 ms per step in alternating processes (profiles/r06az)
        *g = 1, *p = 4, *fpg = 1, *pipe = v8 ? 16 : 25;
    } else if (len_hint <= 600) { // IMIX-like mixes (cfg4): stream kernel with the heads taken
        // out of the block stream and a four-slot first probe window (SH): 1.2704 vs 1.3417 ms
        // for pipe 54 (heads gathered before the stream) on one box, 1.1401 vs 1.1716 on
        // another (counts on, interleaved sweeps, profiles/r02ab); 8-KiB stream tiles (pipe 67)
        // instead of 16: 1.0586 vs 1.1364 and 1.1590 vs 1.1997 ms (profiles/r04b)
        *g = 0, *p = 0, *fpg = 0, *pipe = 67;
    } else if (len_hint <= 1536) { // cfg3: 1500 B.  Write-through verdict stores (pipe 40):
        // 1.0191 vs 1.0322 ms for pipe 0 (interleaved sweep, profiles/r03c/sweep_cfg3_wt.txt),
        // 0.9919 vs 1.0002 across processes (profiles/r03b/ab_store_policy_sc1.txt); written
        // in batches of 16 tiles per block (pipe 41): 0.9992-1.0046 vs 1.0243-1.0280 ms for
        // 40 on two boxes (WB 8 / 12 / 24: 1.038 / 1.024 / 1.054; WB 16 nt 1.013;
        // profiles/r06e, r06f); batches of 24 with a 16-bit histogram (pipe 48, the
        // same 32 KiB of LDS): 0.9881 / 0.9901 vs 0.9927 / 0.9951 ms for 41 (profiles/r06l)
        *g = 8, *p = 2, *fpg = 2, *pipe = 48;
    } else { // jumbo (cfg5: 9000 B): stream kernel (1.72 ms vs 1.77 for G=16, r01b sweep), pipe 38
        // (vs 30: 1.7275 vs 1.7309 and 1.7578 vs 1.7626 ms, r01g, r01j) with 16 frames per block:
        // 32 frames 1.6746 vs 1.7833 ms for 256 (64: 1.6810, 128: 1.7139; profiles/r03f/sweep_cfg5_fpb.txt),
        // 16 frames 1.6521-1.6595 vs 1.6735-1.6805 for 32 (8: 1.7300; profiles/r03j)
        *g = 0, *p = 0, *fpg = 0, *pipe = 938;
    }
}

// the kernel a variant launches, as rocprofv3 names it (without the template
// arguments): rxg_kernel_variant, so a bench line names the dispatch that a
// kernel trace of the same run shows
const char *rx_variant_kernel(uint32_t g, uint32_t pipe) {
    if (g == 1) return "rx_classify_lane_kernel";
    if (g >= 4) return "rx_classify_kernel";
    if (pipe == 20) return "rx_bin_kernel+rx_classify_lane_kernel+rx_classify_kernel";
    switch (pipe % 1000u % 100u) {
    case 60: case 61: case 62: case 63: case 64: case 65: case 66: case 67: case 68: case 69:
    case 70: case 71: case 72: case 73: case 74: case 75: case 76: case 77: case 78:
        return "rx_classify_sh_kernel";
    case 80: case 81: case 82: case 83:
        return "rx_classify_wc_kernel";
    default:
        return "rx_classify_stream_kernel";
    }
}

#endif


#if !RX_V8

// a compiled variant matching (g, p, fpg, pipe) as rx_classify_launch
// matches it (p, fpg = 0: any; pipe = ~0: any) (rxg_tune)
bool rx_variant_exists(uint32_t g, uint32_t p, uint32_t fpg, uint32_t pipe) {
    if (g == 0 && pipe == 20) return true; // size-class binned path
    for (const variant_entry &v : k_variants)
        if (v.g == g && (p == 0 || v.p == p) && (fpg == 0 || v.fpg == fpg) &&
            (pipe == 0xFFFFFFFFu || v.pipe == pipe))
            return true;
    return false;
}
#endif


// workspace bytes one launch needs: the binned path's lists (16 B + 8 B per
// frame), then nbuf count-index buffers (room for 4 B per frame each: two when
// the counts of one burst run on a second stream while the next burst is
// classified, rxg_classify_dev_cs) and the count slabs
static size_t ws_lists_bytes(uint32_t n, uint32_t g, uint32_t pipe) {
    return (g == 0 && pipe == 20) ? ((16 + 8ull * n + 255) & ~(size_t)255) : 0;
}
static size_t ws_cidx_bytes(uint32_t n) { return ((size_t)n * 4 + 255) & ~(size_t)255; }

#if !RX_V8
bool rx_count_uses_slabs(const rx_ft_dev &ft, bool counts) { return use_slab(ft, counts); }

size_t rx_classify_ws_bytes(uint32_t n, uint32_t g, uint32_t pipe, const rx_ft_dev &ft,
                            bool counts, uint32_t nbuf) {
    size_t b = ws_lists_bytes(n, g, pipe);
    if (use_slab(ft, counts)) {
        uint32_t nslabs, per;
        slab_geometry(n, slab_ranges(ft), &nslabs, &per, ft.slab_div_log2);
        b += ws_cidx_bytes(n) * std::max(nbuf, 1u) +
             (size_t)nslabs * slab_ranges(ft) * slab_words(ft) * 4;
    }
    return b;
}

// phase: RX_PH_ALL = classify then (slab path) count, both on s; RX_PH_CLASSIFY
// = the classify kernel only, writing count indices into index buffer `buf`;
// RX_PH_COUNT = the slab + reduce passes over index buffer `buf` only (the
// caller orders it after the RX_PH_CLASSIFY launch that filled the buffer).
// Without the slab path (few flows, or no counts) RX_PH_COUNT does nothing and
// the other two count inside the classify kernel.
#endif

hipError_t RX_K1_NAME(rx_classify_launch)(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                              uint32_t n, uint32_t unit_log2, uint32_t g, uint32_t p, uint32_t fpg,
                              uint32_t pipe, const rx_ft_dev &ft_in, uint4 *out,
                              unsigned long long *counts, hipStream_t s, uint32_t *ws,
                              uint32_t phase, uint32_t buf, uint32_t nbuf) {
    if (n == 0) return hipSuccess;
    const uint32_t nflows = ft_in.nu + ft_in.nt;
    const bool slab = use_slab(ft_in, counts != nullptr);
    if (slab && !ws) return hipErrorInvalidValue;
    if (buf >= std::max(nbuf, 1u)) return hipErrorInvalidValue;
    // workspace: [binned lists][count indices x nbuf][slabs]
    const size_t lists = ws_lists_bytes(n, g, pipe);
    uint8_t *cidx = slab ? reinterpret_cast<uint8_t *>(ws) + lists + ws_cidx_bytes(n) * buf : nullptr;
    rx_ft_dev ft = ft_in;
    ft.count_idx = cidx;
    ft.cidx16 = slab && cidx16(ft_in) && !ft_in.count_4b;
    ft.count_ffff = (ft.cidx16 && nflows == SLAB_MAX_FLOWS) ? counts + 0xFFFFu : nullptr;
    if (phase != RX_PH_COUNT) {
        unsigned long long *kcounts = slab ? nullptr : counts; // slab: counted after classify
        const uint32_t lds_bins = (kcounts && nflows > 0 && nflows <= 8192u) ? nflows : 0u;
        hipError_t e = hipErrorInvalidValue;
        if (g == 0 && pipe == 20) { // size-class binned (workspace: 16 B + 8 B per frame)
            e = launch_binned(pkts, off, len, n, unit_log2, ft, out, kcounts, lds_bins, s, ws);
        } else {
            for (const variant_entry &v : k_variants)
                if (v.g == g && (p == 0 || v.p == p) && (fpg == 0 || v.fpg == fpg) &&
                    (pipe == 0xFFFFFFFFu || v.pipe == pipe)) {
                    rx_ft_dev fv = ft;
                    if (!fv.bpc_cap) fv.bpc_cap = v.bpc; // (rxg_tune_grid's cap, else the variant's)
                    e = v.fn(pkts, off, len, n, unit_log2, fv, out, kcounts, lds_bins, s, nullptr,
                             nullptr);
                    break;
                }
        }
        if (e != hipSuccess) return e;
    }
    if (!slab || phase == RX_PH_CLASSIFY) return hipSuccess;
    uint32_t *slabs = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(ws) + lists +
                                                   ws_cidx_bytes(n) * std::max(nbuf, 1u));
    return launch_count_slab(cidx, n, ft, counts, slabs, s);
}
