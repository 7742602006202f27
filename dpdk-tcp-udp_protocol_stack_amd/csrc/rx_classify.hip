// rx_classify.hip — K1: fused parse + L4 checksum + flow classify (gfx950).
//
// One frame is owned by a lane GROUP of G lanes (G = 4..64, a power of two,
// chosen per burst from the typical frame length).  Lane k of the group reads
// the 16-B chunks k, k+G, k+2G, ... of the frame, so one wave-instruction
// loads 64 x 16 B = 1 KiB of contiguous frame bytes (frames are packed in
// HBM), and a 64-B frame is exactly one load per lane at G = 4.
//
// What each frame goes through (reference behaviour, see ../../include/rxgpu.h):
//   pkt_process demux           netfamily.c:152-200
//   udp_process front           udp.c:11-19, 37-46
//   tcp_process front           tcp.c:345-371 (checksum with field zeroed)
//   rte_ipv4_udptcp_cksum       rte_ip.h:325-349 (DPDK 19.11.12, IHL ignored)
//   get_hostinfo_fromip_port    common.c:97-108   -> UDP bucket probe
//   tcp_stream_search           common.c:31-55    -> TCP bucket probe, then listener table
//
// Checksum: the one's-complement sum is order-independent as long as the
// total is formed without losing carries; a u32 holds the plain sum of up to
// 65535 bytes of 16-bit words (< 2^31), so every lane accumulates a plain u32,
// the group adds the lane sums with a shuffle butterfly, and the fold happens
// once.  Words are little-endian 16-bit words at even frame offsets, exactly
// the reference's native-word view (frame starts are 16-B aligned).
//
// Flow probe: the 4 lowest lanes of the group load one 64-B bucket (4 slots)
// and __ballot the compare; the matching lane's value is shuffled to the group.
#include <hip/hip_runtime.h>

#include "rx_common.h"

namespace {

// bytes [lo, hi) of the 4-byte little-endian word that starts at `pos`
__device__ __forceinline__ uint32_t keep_mask(int32_t pos, int32_t lo, int32_t hi) {
    int32_t a = lo - pos;
    int32_t b = hi - pos;
    a = a < 0 ? 0 : (a > 4 ? 4 : a);
    b = b < 0 ? 0 : (b > 4 ? 4 : b);
    uint64_t m = ((1ull << (8 * b)) - 1ull) & ~((1ull << (8 * a)) - 1ull);
    return (uint32_t)m;
}

// sum of the LE 16-bit words of chunk c (frame bytes [s, s+16)) restricted to
// [lo, hi), with the 2-byte field at `hole` (even; -64 = none) taken as zero
__device__ __forceinline__ uint32_t chunk_sum(uint4 c, int32_t s, int32_t lo, int32_t hi,
                                              int32_t hole) {
    uint32_t x[4] = {c.x, c.y, c.z, c.w};
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int32_t pos = s + 4 * j;
        uint32_t m = keep_mask(pos, lo, hi);
        // hole bytes [hole, hole+2) inside this word?
        int32_t hd = hole - pos; // 0 or 2 when inside (hole is even)
        if (hd == 0) m &= 0xFFFF0000u;
        if (hd == 2) m &= 0x0000FFFFu;
        uint32_t v = x[j] & m;
        acc += (v & 0xFFFFu) + (v >> 16);
    }
    return acc;
}

__device__ __forceinline__ uint4 mask_chunk(uint4 c, int32_t s, int32_t cap) {
    c.x &= keep_mask(s + 0, 0, cap);
    c.y &= keep_mask(s + 4, 0, cap);
    c.z &= keep_mask(s + 8, 0, cap);
    c.w &= keep_mask(s + 12, 0, cap);
    return c;
}

template <int G>
__global__ __launch_bounds__(256) void rx_classify_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t n, uint32_t unit_log2, rx_ft_dev ft,
    uint4 *__restrict__ out, unsigned long long *__restrict__ counts, uint32_t lds_bins) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    static_assert(G >= 4 && G <= 64 && (G & (G - 1)) == 0, "G must be a power of two in [4,64]");
    constexpr uint32_t GPB = 256 / G;  // frame groups per block
    constexpr int32_t STEP = 16 * G;   // bytes one group pass covers

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint32_t gl = lane & (G - 1);
    const uint32_t gbase = lane & ~(uint32_t)(G - 1);
    const uint32_t grp = tid / G;

    if (lds_bins) {
        for (uint32_t i = tid; i < lds_bins; i += 256) hist[i] = 0;
        __syncthreads();
    }

    const uint64_t stride = (uint64_t)gridDim.x * GPB;
    for (uint64_t p = (uint64_t)blockIdx.x * GPB + grp; p < n; p += stride) {
        const uint8_t *f = pkts + ((uint64_t)off[p] << unit_log2);
        const int32_t cap = (int32_t)len[p];

        // ---- pass 0: chunk gl, header fields broadcast from lanes 0..3
        const int32_t s0 = 16 * (int32_t)gl;
        uint4 c0 = make_uint4(0, 0, 0, 0);
        if (s0 < cap) c0 = mask_chunk(*reinterpret_cast<const uint4 *>(f + s0), s0, cap);

        const uint32_t h03 = __shfl(c0.w, gbase + 0); // bytes 12..15
        const uint32_t h10 = __shfl(c0.x, gbase + 1); // 16..19
        const uint32_t h11 = __shfl(c0.y, gbase + 1); // 20..23
        const uint32_t h12 = __shfl(c0.z, gbase + 1); // 24..27
        const uint32_t h13 = __shfl(c0.w, gbase + 1); // 28..31
        const uint32_t h20 = __shfl(c0.x, gbase + 2); // 32..35
        const uint32_t h21 = __shfl(c0.y, gbase + 2); // 36..39
        const uint32_t h22 = __shfl(c0.z, gbase + 2); // 40..43
        const uint32_t h23 = __shfl(c0.w, gbase + 2); // 44..47
        const uint32_t h30 = __shfl(c0.x, gbase + 3); // 48..51

        const uint32_t et = h03 & 0xFFFFu; // LE view of bytes 12,13
        const uint32_t tl = rx_bswap16(h10 & 0xFFFFu);
        const uint32_t proto = h11 >> 24;
        const uint32_t sip = (h12 >> 16) | (h13 << 16);
        const uint32_t dip = (h13 >> 16) | (h20 << 16);
        const uint32_t sport = h20 >> 16;
        const uint32_t dport = h21 & 0xFFFFu;
        const uint32_t dgram_len = rx_bswap16(h21 >> 16);

        uint32_t cls, need;
        int32_t hole = -64;
        if (et == 0x0608u) {
            cls = RXG_CLS_ARP;
            need = 42;
        } else if (et != 0x0008u) {
            cls = RXG_CLS_NON_IP;
            need = 14;
        } else if (proto == 17u) {
            cls = RXG_CLS_UDP;
            hole = 40;
            need = 42;
        } else if (proto == 6u) {
            cls = RXG_CLS_TCP;
            hole = 50;
            need = 54;
        } else {
            cls = RXG_CLS_IPV4_OTHER;
            need = 24;
        }
        const bool l4 = cls == RXG_CLS_UDP || cls == RXG_CLS_TCP;
        const uint32_t l4n = tl >= 20u ? tl - 20u : 0u;
        const bool do_sum = l4 && tl >= 20u;
        if (l4 && 34u + l4n > need) need = 34u + l4n;

        // ---- checksum over [26, 34 + l4n) ∩ [0, cap) (pseudo src/dst + L4)
        const int32_t lo = 26;
        int32_t hi = do_sum ? 34 + (int32_t)l4n : 0;
        if (hi > cap) hi = cap;
        uint32_t sum = do_sum ? chunk_sum(c0, s0, lo, hi, hole) : 0u;
        for (int32_t sb = STEP; sb < hi; sb += 4 * STEP) { // group-uniform trip count
            uint4 c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int32_t s = s0 + sb + u * STEP;
                c[u] = make_uint4(0, 0, 0, 0);
                if (s < hi) c[u] = *reinterpret_cast<const uint4 *>(f + s);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) sum += chunk_sum(c[u], s0 + sb + u * STEP, lo, hi, hole);
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) sum += __shfl_xor(sum, o);

        uint32_t ck = 0;
        if (do_sum) {
            sum += proto << 8;          // psd {zero, proto}
            sum += rx_bswap16(l4n);     // psd be16(l4_len)
            ck = (~rx_fold(sum)) & 0xFFFFu;
            if (ck == 0u && proto == 17u) ck = 0xFFFFu;
        }
        const uint32_t stored = cls == RXG_CLS_UDP ? (h22 & 0xFFFFu)
                                                   : (cls == RXG_CLS_TCP ? (h30 >> 16) : 0u);
        const bool ok = l4 && stored == ck;

        // ---- flow probe
        const bool do_udp = cls == RXG_CLS_UDP;
        const bool do_tcp = cls == RXG_CLS_TCP && ok;
        uint32_t flow = RXG_FLOW_NONE;
        if (do_udp || do_tcp) {
            const uint4 *tbl = do_udp ? ft.udp : ft.tcp;
            const uint32_t mask = do_udp ? ft.udp_mask : ft.tcp_mask;
            const uint32_t maxp = do_udp ? ft.udp_probe : ft.tcp_probe;
            const uint32_t ka = do_udp ? dip : sip;
            const uint32_t kb = do_udp ? dport : dip;
            const uint32_t kc = do_udp ? 17u : (sport | (dport << 16));
            uint32_t b = rx_hash3(ka, kb, kc) & mask;
            for (uint32_t pr = 0; pr < maxp; ++pr) {
                uint4 sl = make_uint4(0, 0, 0, RX_SLOT_EMPTY);
                if (gl < RX_BUCKET_SLOTS) sl = tbl[(b << 2) + gl];
                const bool hit = gl < RX_BUCKET_SLOTS && sl.w != RX_SLOT_EMPTY && sl.x == ka &&
                                 sl.y == kb && sl.z == kc;
                const bool emp = gl < RX_BUCKET_SLOTS && sl.w == RX_SLOT_EMPTY;
                const uint32_t gh = (uint32_t)(__ballot(hit) >> gbase) & 0xFu;
                const uint32_t ge = (uint32_t)(__ballot(emp) >> gbase) & 0xFu;
                const uint32_t v = __shfl(sl.w, gbase + (gh ? (uint32_t)(__ffs(gh) - 1) : 0u));
                if (gh) {
                    flow = v;
                    break;
                }
                if (ge) break;
                b = (b + 1) & mask;
            }
            if (do_tcp && flow == RXG_FLOW_NONE) flow = ft.listen[dport];
        }

        // ---- verdict (reference return codes)
        int32_t rc;
        uint32_t poff = 0, plen = 0, flags = 0;
        if (cls == RXG_CLS_UDP) {
            rc = flow == RXG_FLOW_NONE ? RXG_RC_UDP_NO_SOCKET
                                       : (dgram_len <= 8u ? RXG_RC_UDP_NOMEM : RXG_RC_OK);
            poff = 42;
            plen = dgram_len > 8u ? dgram_len - 8u : 0u;
            if (dgram_len <= 8u) flags |= RXG_F_UDP_SHORT;
            if (rc == RXG_RC_OK && 42u + plen > need) need = 42u + plen;
        } else if (cls == RXG_CLS_TCP) {
            const uint32_t hl = ((h23 >> 16) & 0xFFu) >> 4;
            const int32_t pl = (int32_t)tl - 20 - 4 * (int32_t)hl;
            poff = 34u + 4u * hl;
            if (pl < 0) flags |= RXG_F_TCP_NEGLEN;
            plen = pl < 0 ? 0u : (uint32_t)pl;
            rc = !ok ? RXG_RC_TCP_BAD_CKSUM
                     : (flow == RXG_FLOW_NONE ? RXG_RC_TCP_NO_TCB : RXG_RC_OK);
        } else {
            rc = RXG_RC_KNI;
        }
        if ((int32_t)need > cap) flags |= RXG_F_TRUNC;

        if (gl == 0) {
            uint4 v;
            v.x = flow;
            v.y = (poff & 0xFFFFu) | (plen << 16);
            v.z = ck | (cls << 16) | (((uint32_t)rc & 0xFFu) << 24);
            v.w = (ok ? 1u : 0u) | (flags << 8) | (stored << 16);
            out[p] = v;
            if (counts && rc == RXG_RC_OK && flow != RXG_FLOW_NONE) {
                const uint32_t idx = (cls == RXG_CLS_TCP ? ft.nu : 0u) + flow;
                if (lds_bins)
                    atomicAdd(&hist[idx], 1u);
                else
                    atomicAdd(&counts[idx], 1ull);
            }
        }
    }

    if (lds_bins) {
        __syncthreads();
        for (uint32_t i = tid; i < lds_bins; i += 256) {
            const uint32_t c = hist[i];
            if (c) atomicAdd(&counts[i], (unsigned long long)c);
        }
    }
}

template <int G>
hipError_t launch_g(const uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                    uint32_t unit_log2, const rx_ft_dev &ft, uint4 *out, unsigned long long *counts,
                    uint32_t lds_bins, uint32_t max_blocks, hipStream_t s) {
    constexpr uint32_t GPB = 256 / G;
    uint64_t blocks = (n + GPB - 1) / GPB;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks == 0) blocks = 1;
    size_t lds = (size_t)lds_bins * 4u;
    hipLaunchKernelGGL((rx_classify_kernel<G>), dim3((uint32_t)blocks), dim3(256), lds, s, pkts, off,
                       len, n, unit_log2, ft, out, counts, lds_bins);
    return hipGetLastError();
}

} // namespace

// Lanes per frame from a typical frame length: about two to three group
// passes per frame, at least 4 lanes (the 64-B header spans 4 chunks).
uint32_t rx_pick_group(uint32_t len_hint) {
    if (len_hint == 0) len_hint = 1518;
    uint32_t chunks = (len_hint + 15) / 16;
    uint32_t g = 4;
    while (g < 64 && g * 2 <= chunks / 2) g *= 2;
    return g;
}

// LDS histogram when the flow count fits comfortably (<= 8192 bins = 32 KiB).
hipError_t rx_classify_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                              uint32_t n, uint32_t unit_log2, uint32_t group, const rx_ft_dev &ft,
                              uint4 *out, unsigned long long *counts, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t nflows = ft.nu + ft.nt;
    const uint32_t lds_bins = (counts && nflows > 0 && nflows <= 8192u) ? nflows : 0u;
    const uint32_t max_blocks = 256u * 8u; // 256 CUs x 8 resident 256-thread blocks
    switch (group) {
    case 4:
        return launch_g<4>(pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, max_blocks, s);
    case 8:
        return launch_g<8>(pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, max_blocks, s);
    case 16:
        return launch_g<16>(pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, max_blocks, s);
    case 32:
        return launch_g<32>(pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, max_blocks, s);
    case 64:
        return launch_g<64>(pkts, off, len, n, unit_log2, ft, out, counts, lds_bins, max_blocks, s);
    default:
        return hipErrorInvalidValue;
    }
}
