// tx_cksum.hip — K2: TX checksum generation for a burst of outgoing frames
// (gfx950).  The reference builds every frame it sends on the protocol lcore
// and checksums it there, one frame at a time:
//   ng_encode_udp_apppkt   udp.c:84-95   hdr_checksum = rte_ipv4_cksum,
//                                        dgram_cksum = rte_ipv4_udptcp_cksum
//   ng_encode_tcp_apppkt   tcp.c:444-463 hdr_checksum = rte_ipv4_cksum,
//                                        cksum       = rte_ipv4_udptcp_cksum
// (DPDK 19.11.12 rte_ip.h:255-265 and :325-349; each computed with its own
// field taken as 0).  Here a burst of frames in the rx burst layout is
// checksummed in place: IPv4 frames get the header checksum, IPv4 UDP/TCP
// frames the L4 checksum as well; other frames are not touched.
//
// Work decomposition: a group of G lanes per frame, lane k reading chunks
// k, k+G, ... (1 KiB per wave instruction); lanes 0..2 of pass 0 hold the
// IPv4 header; both sums are exact integer partial sums added over the group
// with DPP, so the result is the reference's whatever the split (see
// rx_classify.hip).  One frame per group, one launch-wide grid.
#include <hip/hip_runtime.h>

#include "rx_common.h"
#include "rx_device.h"

namespace {

template <int G>
__global__ __launch_bounds__(256) void tx_cksum_kernel(uint8_t *__restrict__ pkts,
                                                       const uint32_t *__restrict__ off,
                                                       const uint16_t *__restrict__ len, uint32_t n,
                                                       uint32_t unit_log2) {
    constexpr uint32_t GPB = 256 / G;
    constexpr int32_t STEP = 16 * G;
    const uint32_t tid = threadIdx.x, gl = tid & (G - 1);
    const uint64_t f = (uint64_t)blockIdx.x * GPB + tid / G;
    if (f >= n) return; // group-uniform: every lane of a group has the same f
    uint8_t *fb = pkts + ((uint64_t)off[f] << unit_log2);
    const int32_t cp = (int32_t)len[f];
    const int32_t s0 = 16 * (int32_t)gl;
    uint4 x0 = make_uint4(0, 0, 0, 0);
    if (s0 < cp) x0 = chunk_below(ldg16<false>(fb + s0), s0, cp); // past caplen reads 0
    const uint32_t et = gbcast<G, 0>(x0.w) & 0xFFFFu;           // bytes 12,13
    const uint32_t h10 = gbcast<G, 1>(x0.x), h11 = gbcast<G, 1>(x0.y);
    const bool ipv4 = et == 0x0008u;
    const uint32_t tl = rx_bswap16(h10 & 0xFFFFu), proto = h11 >> 24;
    const bool l4 = ipv4 && (proto == 17u || proto == 6u);
    const bool do_sum = l4 && tl >= 20u; // rte_ip.h:330-331: tl < 20 -> checksum 0
    const uint32_t l4n = tl >= 20u ? tl - 20u : 0u;
    const int32_t hole = proto == 17u ? 40 : 50;

    // IPv4 header words [14, 34), the header checksum field (24, 25) as 0
    uint32_t ip = 0;
    if (gl == 0) ip = x0.w >> 16;
    if (gl == 1) ip = add_halves(add_halves(add_halves(0u, x0.x), x0.y), x0.w) + (x0.z >> 16);
    if (gl == 2) ip = x0.x & 0xFFFFu;
    // L4 words [26, e), e = min(34 + l4n, caplen), the L4 field as 0
    int32_t e = do_sum ? 34 + (int32_t)l4n : 0;
    if (e > cp) e = cp;
    uint32_t acc = 0;
    {
        uint4 v = x0;
        if (s0 + 16 > e) v = chunk_below(v, s0, e);
        if (gl == 0) v = make_uint4(0, 0, 0, 0);
        if (gl == 1) v.x = v.y = 0, v.z &= 0xFFFF0000u;
        if (gl == 2 && hole == 40) v.z &= 0xFFFF0000u;
        if (gl == 3 && hole == 50) v.x &= 0x0000FFFFu;
        acc = add_halves(add_halves(add_halves(add_halves(acc, v.x), v.y), v.z), v.w);
    }
    for (int32_t sb = STEP; sb < e; sb += 4 * STEP) { // group-uniform
        uint4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int32_t s = s0 + sb + u * STEP;
            r[u] = ldg16<true>(fb + (s < e ? s : 0)); // unconditional: partial wait counts
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int32_t s = s0 + sb + u * STEP;
            const uint4 v = chunk_below(r[u], s, e); // zero past e (and past the frame)
            acc = add_halves(add_halves(add_halves(add_halves(acc, v.x), v.y), v.z), v.w);
        }
    }
    ip = gsum<G>(ip);
    acc = gsum<G>(acc);
    if (gl != 0 || !ipv4) return;
    if (cp >= 26) { // rte_ipv4_cksum, rte_ip.h:255-265
        const uint32_t c = fold16(ip);
        *reinterpret_cast<uint16_t *>(fb + 24) = (uint16_t)(c == 0xFFFFu ? c : (~c & 0xFFFFu));
    }
    if (l4 && cp >= hole + 2) { // rte_ipv4_udptcp_cksum, rte_ip.h:325-349
        acc += (proto << 8) + rx_bswap16(l4n); // pseudo-header {0, proto}, be16(l4 len)
        uint32_t c = (~fold16(acc)) & 0xFFFFu;
        if (c == 0u && proto == 17u) c = 0xFFFFu;
        if (!do_sum) c = 0u;
        *reinterpret_cast<uint16_t *>(fb + hole) = (uint16_t)c;
    }
}

template <int G>
hipError_t launch_tx(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                     uint32_t unit_log2, hipStream_t s) {
    const uint64_t blocks = ((uint64_t)n + 256 / G - 1) / (256 / G);
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tx_cksum_kernel<G>, dim3((uint32_t)blocks), dim3(256), 0, s, pkts, off, len,
                       n, unit_log2);
    return hipGetLastError();
}

} // namespace

// lanes per frame from the typical frame length: a pass of 16*G bytes per group
hipError_t tx_cksum_launch(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                           uint32_t unit_log2, uint32_t len_hint, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (len_hint == 0) len_hint = 1518;
    if (len_hint <= 128) return launch_tx<4>(pkts, off, len, n, unit_log2, s);
    if (len_hint <= 1536) return launch_tx<8>(pkts, off, len, n, unit_log2, s);
    return launch_tx<16>(pkts, off, len, n, unit_log2, s);
}
