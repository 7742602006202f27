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
// k, k+G, ... of the frame; lanes 0..2 of pass 0 hold the IPv4 header; both
// sums are exact integer partial sums added over the group with DPP, so the
// result is the reference's whatever the split (see rx_classify.hip).  A
// group takes FPG frames per trip and issues the first P passes of all of
// them before consuming any (FPG*P loads of a lane in flight); longer frames
// finish in batches of 4 passes.  The grid is the resident block count and
// blocks stride over tiles, as for the RX kernels (or one block per tile:
// TX_FULL_GRID, the round-1 shape, kept as a tuning alternative).
#include <hip/hip_runtime.h>

#include "rx_common.h"
#include "rx_device.h"

namespace {

// WB (how the two checksum fields reach memory): 0 = two 2-B stores by the
// group's lane 0; 1 = the lanes holding the fields store their whole 16-B
// header chunk, patched; 2 = lanes 0..3 store all four header chunks
// [0, 64), patched (one full 64-B sector per frame).  Unchanged bytes are
// written back as read, and only chunks that start inside the frame (the
// buffer owns every frame's bytes up to its next 16-B boundary).
template <int G, int P, int WB>
__device__ __forceinline__ void tx_frame(uint8_t *fb, int32_t cp, bool valid, const uint4 (&c)[P],
                                         uint32_t gl) {
    constexpr int32_t STEP = 16 * G;
    const int32_t s0 = 16 * (int32_t)gl;
    uint4 x0 = c[0];
    if (s0 + 16 > cp) x0 = chunk_below(x0, s0, cp);   // past caplen reads 0
    const uint32_t et = gbcast<G, 0>(x0.w) & 0xFFFFu; // bytes 12,13
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
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const int32_t s = s0 + q * STEP;
        uint4 v = q == 0 ? x0 : c[q];
        if (s + 16 > e) v = chunk_below(v, s, e);
        if (q == 0) {
            if (gl == 0) v = make_uint4(0, 0, 0, 0);
            if (gl == 1) v.x = v.y = 0, v.z &= 0xFFFF0000u;
            if (gl == 2 && hole == 40) v.z &= 0xFFFF0000u;
            if (gl == 3 && hole == 50) v.x &= 0x0000FFFFu;
        }
        acc = add_halves(add_halves(add_halves(add_halves(acc, v.x), v.y), v.z), v.w);
    }
    for (int32_t sb = P * STEP; sb < e; sb += 4 * STEP) { // group-uniform
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
    ip = gsum<G>(ip); // group totals in every lane of the group
    acc = gsum<G>(acc);
    if (!valid || !ipv4) return;
    const uint32_t kip = fold16(ip); // rte_ipv4_cksum, rte_ip.h:255-265
    const uint32_t hip = kip == 0xFFFFu ? kip : (~kip & 0xFFFFu);
    acc += (proto << 8) + rx_bswap16(l4n); // pseudo-header {0, proto}, be16(l4 len)
    uint32_t kl4 = (~fold16(acc)) & 0xFFFFu; // rte_ipv4_udptcp_cksum, rte_ip.h:325-349
    if (kl4 == 0u && proto == 17u) kl4 = 0xFFFFu;
    if (!do_sum) kl4 = 0u;
    const bool w_ip = cp >= 26, w_l4 = l4 && cp >= hole + 2;
    if constexpr (WB == 0) {
        if (gl != 0) return;
        if (w_ip) *reinterpret_cast<uint16_t *>(fb + 24) = (uint16_t)hip;
        if (w_l4) *reinterpret_cast<uint16_t *>(fb + hole) = (uint16_t)kl4;
    } else {
        uint4 v = c[0]; // as read (bytes past caplen included)
        bool mine = WB == 2 ? (gl < 4 && s0 < cp) : false;
        if (gl == 1 && w_ip) v.z = (v.z & 0xFFFF0000u) | hip, mine = true;         // bytes 24,25
        if (gl == 2 && w_l4 && hole == 40) v.z = (v.z & 0xFFFF0000u) | kl4, mine = true; // 40,41
        if (gl == 3 && w_l4 && hole == 50) v.x = (v.x & 0x0000FFFFu) | (kl4 << 16), mine = true; // 50,51
        if (mine) *reinterpret_cast<uint4 *>(fb + s0) = v;
    }
}

template <int G, int P, int FPG, int WB>
__global__ __launch_bounds__(256) void tx_cksum_kernel(uint8_t *__restrict__ pkts,
                                                       const uint32_t *__restrict__ off,
                                                       const uint16_t *__restrict__ len, uint32_t n,
                                                       uint32_t unit_log2) {
    constexpr uint32_t GPB = 256 / G, TILE = GPB * FPG;
    constexpr int32_t STEP = 16 * G;
    const uint32_t tid = threadIdx.x, gl = tid & (G - 1), grp = tid / G;
    const int32_t s0 = 16 * (int32_t)gl;
    for (uint64_t tile = blockIdx.x; tile * TILE < n; tile += gridDim.x) {
        uint8_t *fb[FPG];
        int32_t cp[FPG];
        bool valid[FPG];
        uint4 c[FPG][P];
#pragma unroll
        for (int f = 0; f < FPG; ++f) {
            const uint64_t pos = tile * TILE + (uint64_t)f * GPB + grp;
            valid[f] = pos < n;
            const uint64_t q = valid[f] ? pos : 0;
            fb[f] = pkts + ((uint64_t)off[q] << unit_log2);
            cp[f] = valid[f] ? (int32_t)len[q] : 0;
        }
        // every pass of every frame in flight before the first is consumed;
        // unconditional with clamped addresses (bytes past caplen are masked)
#pragma unroll
        for (int f = 0; f < FPG; ++f)
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const int32_t s = s0 + q * STEP;
                c[f][q] = q == 0 ? ldg16<false>(fb[f] + (s < cp[f] ? s : 0))
                                 : ldg16<true>(fb[f] + (s < cp[f] ? s : 0));
            }
#pragma unroll
        for (int f = 0; f < FPG; ++f) tx_frame<G, P, WB>(fb[f], cp[f], valid[f], c[f], gl);
    }
}

// bpc_cap: resident blocks per CU (0 = occupancy); TX_FULL_GRID = one block
// per tile instead of a resident grid
constexpr uint32_t TX_FULL_GRID = 1000;
template <int G, int P, int FPG, int WB = 0>
hipError_t launch_tx(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                     uint32_t unit_log2, uint32_t bpc_cap, hipStream_t s) {
    constexpr uint32_t TILE = (256 / G) * FPG;
    int cu = 0, occ = 0;
    hipError_t e = rx_occupancy(reinterpret_cast<const void *>(tx_cksum_kernel<G, P, FPG, WB>),
                                256, 0, &cu, &occ);
    if (e != hipSuccess) return e;
    const uint64_t tiles = ((uint64_t)n + TILE - 1) / TILE;
    uint64_t bpc = (uint64_t)occ;
    if (bpc_cap && bpc > bpc_cap) bpc = bpc_cap;
    uint64_t blocks = (uint64_t)cu * bpc;
    if (blocks > tiles || bpc_cap == TX_FULL_GRID) blocks = tiles;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((tx_cksum_kernel<G, P, FPG, WB>), dim3((uint32_t)blocks), dim3(256), 0, s, pkts,
                       off, len, n, unit_log2);
    return hipGetLastError();
}

typedef hipError_t (*tx_launch_fn)(uint8_t *, const uint32_t *, const uint16_t *, uint32_t,
                                   uint32_t, uint32_t, hipStream_t);
struct tx_variant {
    tx_launch_fn fn;
    uint32_t bpc; // resident blocks per CU cap (0 = occupancy)
};
// 10: the default for <= 64 B frames and for mixed sizes; 1..3 for <= 128,
// <= 1536 and longer frames; the rest are tuning alternatives (rxg_tune_tx).
// At 64 B one block per 64-frame tile (10) ran 0.3945-0.3962 ms against
// 0.4468-0.4478 for the resident grid with 4 frames per group (0), and 4 /
// 1 block per tile with 2 / 4 frames per group 0.4084 / 0.4109; the next
// trip's descriptors loaded one trip ahead (resident grid) 0.4523-0.4533
// (interleaved sweeps, profiles/r06ag).  Round 1 had measured 10 behind 0
// (0.4538 vs 0.4460, r01d).
// Measured (tools/tx_sweep.py, profiles/r01d/tx_sweep.txt): the write mode and
// the schedule move these by only 2-4%.  Changing 4 bytes in a frame's first
// 64 B dirties its first 128-B line, and the line goes back to HBM whole, so
// every TX launch also writes 128 B per frame (64 B per 64-B frame) that the
// algorithmic byte count (frame + 6 + 4) does not include.
static const tx_variant k_tx[] = {
    {launch_tx<4, 1, 4, 2>, 0},              {launch_tx<4, 2, 2, 2>, 0},
    {launch_tx<8, 12, 1, 2>, 0},             {launch_tx<16, 8, 1, 2>, 0},
    {launch_tx<4, 1, 1>, TX_FULL_GRID},      {launch_tx<8, 1, 1>, TX_FULL_GRID},
    {launch_tx<4, 1, 4, 1>, 0},              {launch_tx<4, 1, 4>, 0},
    {launch_tx<8, 12, 1, 1>, 0},             {launch_tx<8, 12, 1>, 0},
    {launch_tx<4, 1, 1, 2>, TX_FULL_GRID},   {launch_tx<8, 1, 1, 2>, TX_FULL_GRID},
    {launch_tx<16, 8, 1>, 0},
};

} // namespace

uint32_t tx_num_variants() { return (uint32_t)(sizeof(k_tx) / sizeof(k_tx[0])); }

// lanes per frame and passes in flight from the typical frame length, unless
// `variant` (< tx_num_variants()) forces one; bpc_cap 0 = the variant's own
hipError_t tx_cksum_launch(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                           uint32_t unit_log2, uint32_t len_hint, uint32_t variant,
                           uint32_t bpc_cap, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (len_hint == 0) len_hint = 1518;
    // (mixed sizes, e.g. IMIX at 354 B average: G=4, one frame per group and
    // block per tile, 1.88 ms vs 2.30 for G=8 on cfg4, profiles/r01d + r01e)
    uint32_t v = len_hint <= 64 ? 10 : (len_hint <= 128 ? 1 : (len_hint <= 600 ? 10 : (len_hint <= 1536 ? 2 : 3)));
    if (variant < tx_num_variants()) v = variant;
    return k_tx[v].fn(pkts, off, len, n, unit_log2, bpc_cap ? bpc_cap : k_tx[v].bpc, s);
}
