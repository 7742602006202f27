// rx_compact.hip — K3: per-socket payload compaction of a classified burst,
// the device half of UDP delivery (udp_process after its lookup, udp.c:25-52).
//
// The reference, for every datagram that found its socket (rc 0), mallocs an
// offload and a payload buffer, copies dgram_len - 8 payload bytes from udp+1
// (udp.c:37-46) and enqueues the offload on that socket's receive ring
// (udp.c:48), one frame at a time.  Here one pass over the burst's verdicts
// groups the delivered datagrams by socket (a stable counting sort: inside a
// socket they keep burst order, the order the ring would have) and gathers
// their payloads into one buffer, socket after socket, each payload at a
// 16-B aligned offset; the host then hands each socket one contiguous slice
// (one memcpy per socket per burst, host/nstack.c).
//
// Three kernels, all for <= RX_CP_MAX_FLOWS UDP ids (the reference's socket
// layer has at most D_MAX_FD_COUNT = 1024 descriptors, common.h:34):
//   1. per 1024-frame tile: each wave groups its 64 frames by socket (ballot
//      per distinct socket), the groups' datagram and byte counts add into an
//      LDS histogram, written out per tile;
//   2. one block: per socket, the exclusive prefix over tiles, then the
//      exclusive scan over sockets (datagram ranks and byte offsets);
//   3. per tile again: the waves add their groups into the tile histogram in
//      wave order (one barrier per wave), which gives every datagram its rank
//      and byte offset; it writes its record and copies its payload.
// Bytes past a frame's capture read as 0 (the delivery oracle's rule).
#include <hip/hip_runtime.h>

#include "rx_common.h"

#define RX_CP_MAX_FLOWS 1024u
#define RX_CP_WAVES 16u
#define RX_CP_TILE (64u * RX_CP_WAVES)

namespace {

__device__ __forceinline__ uint32_t cp_scan(uint32_t x) { // inclusive, 64 lanes, all active
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false);
    return x;
}

// one frame as delivery sees it: delivered (UDP, rc 0, a socket id < nflows),
// its socket, its payload length (dgram_len - 8, udp.c:38), the captured part
// of it (the rest reads as zeros: only the captured bytes are gathered) and
// that rounded up to 16 B
struct cp_frame {
    bool deliv;
    uint32_t flow, plen, ncopy, padded;
};

__device__ __forceinline__ cp_frame cp_decode(const uint4 *__restrict__ v,
                                              const uint16_t *__restrict__ len, uint64_t i,
                                              uint64_t n, uint32_t nflows) {
    cp_frame f{false, 0u, 0u, 0u, 0u};
    if (i < n) {
        const uint4 x = v[i];
        const uint32_t cls = (x.z >> 16) & 0xFFu;
        const int32_t rc = (int8_t)(x.z >> 24);
        f.deliv = cls == RXG_CLS_UDP && rc == RXG_RC_OK && x.x < nflows;
        f.flow = f.deliv ? x.x : 0u;
        f.plen = f.deliv ? (x.y >> 16) : 0u;
        const uint32_t cap = f.deliv ? len[i] : 0u;
        const uint32_t avail = cap > 42u ? cap - 42u : 0u;
        f.ncopy = f.plen < avail ? f.plen : avail;
        f.padded = (f.ncopy + 15u) & ~15u;
    }
    return f;
}

// this lane's place in its wave: the datagrams of one socket form a group;
// rank / bpre = datagrams / bytes of the group in lower lanes; the group's
// leader (lowest lane) also gets the group's totals and every lane its
// leader's lane
struct cp_group {
    uint32_t rank, bpre, lead, gcnt, gbytes;
};

__device__ __forceinline__ cp_group cp_groups(const cp_frame &f, uint32_t lane) {
    cp_group g{0u, 0u, lane, 0u, 0u};
    uint64_t rem = __ballot(f.deliv);
    while (rem) {
        const uint32_t l = (uint32_t)__builtin_ctzll(rem);
        const uint32_t fl = __shfl(f.flow, (int)l);
        const uint64_t m = __ballot(f.deliv && f.flow == fl);
        const bool in = (m >> lane) & 1ull;
        const uint32_t x = in ? f.padded : 0u;
        const uint32_t inc = cp_scan(x);
        const uint32_t tot = __shfl(inc, 63);
        if (in) {
            g.rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            g.bpre = inc - x;
            g.lead = l;
            if (lane == l) g.gcnt = (uint32_t)__popcll(m), g.gbytes = tot;
        }
        rem &= ~m;
    }
    return g;
}

__global__ __launch_bounds__(1024) void rx_cp_count_kernel(const uint4 *__restrict__ v,
                                                           const uint16_t *__restrict__ len, uint32_t n,
                                                           uint32_t nflows, uint2 *__restrict__ tiles) {
    __shared__ uint32_t cnt[RX_CP_MAX_FLOWS], byt[RX_CP_MAX_FLOWS];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t k = tid; k < nflows; k += 1024u) cnt[k] = byt[k] = 0u;
    __syncthreads();
    const cp_frame f = cp_decode(v, len, (uint64_t)blockIdx.x * RX_CP_TILE + tid, n, nflows);
    const cp_group g = cp_groups(f, lane);
    if (g.gcnt) {
        atomicAdd(&cnt[f.flow], g.gcnt);
        atomicAdd(&byt[f.flow], g.gbytes);
    }
    __syncthreads();
    uint2 *t = tiles + (uint64_t)blockIdx.x * nflows;
    for (uint32_t k = tid; k < nflows; k += 1024u) t[k] = make_uint2(cnt[k], byt[k]);
}

// one block, a thread per socket: exclusive prefixes over the tiles, then over
// the sockets; tiles[t][f] becomes (first rank, first byte) of socket f's
// datagrams in tile t; first[f] = socket f's first rank (first[nflows] = all),
// totals = {datagrams, bytes}
__global__ __launch_bounds__(1024) void rx_cp_scan_kernel(uint2 *__restrict__ tiles, uint32_t ntiles,
                                                          uint32_t nflows, uint32_t *__restrict__ first,
                                                          uint32_t *__restrict__ totals) {
    __shared__ uint32_t wc[16], wb[16];
    const uint32_t f = threadIdx.x, lane = f & 63u, wv = f >> 6;
    uint32_t c = 0u, b = 0u;
    if (f < nflows)
        for (uint32_t t = 0; t < ntiles; ++t) {
            const uint2 x = tiles[(uint64_t)t * nflows + f];
            tiles[(uint64_t)t * nflows + f] = make_uint2(c, b);
            c += x.x;
            b += x.y;
        }
    const uint32_t ic = cp_scan(c), ib = cp_scan(b);
    if (lane == 63u) wc[wv] = ic, wb[wv] = ib;
    __syncthreads();
    uint32_t oc = 0u, ob = 0u;
    for (uint32_t w = 0; w < wv; ++w) oc += wc[w], ob += wb[w];
    const uint32_t ec = oc + ic - c, eb = ob + ib - b; // exclusive over the sockets
    if (f < nflows) {
        first[f] = ec;
        for (uint32_t t = 0; t < ntiles; ++t) {
            uint2 &x = tiles[(uint64_t)t * nflows + f];
            x = make_uint2(x.x + ec, x.y + eb);
        }
    }
    if (f == 1023u) { // the last thread holds the grand totals
        first[nflows] = ec + c;
        totals[0] = ec + c;
        totals[1] = eb + b;
    }
}

// payload bytes [0, ncopy) of a datagram from frame + 42 (udp + 1, udp.c:46),
// zero to its 16-B padded end; sources read as dwords below the capture only
__device__ __forceinline__ void cp_copy(const uint8_t *__restrict__ fr, uint32_t cap, uint32_t ncopy,
                                        uint4 *__restrict__ dst) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(fr + 40); // 4-B aligned (frames are 16-B)
    auto word = [&](uint32_t k) -> uint32_t { return 40u + 4u * k < cap ? w[k] : 0u; };
    uint32_t prev = word(0);
    for (uint32_t j = 0; 16u * j < ncopy; ++j) {
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t nx = word(4u * j + (uint32_t)q + 1u);
            o[q] = (prev >> 16) | (nx << 16); // bytes 42 + 16j + 4q .. +4
            prev = nx;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) { // mask bytes past the copied ones
            const uint32_t b0 = 16u * j + 4u * (uint32_t)q;
            const uint32_t keep = ncopy > b0 ? ncopy - b0 : 0u;
            if (keep < 4u) o[q] &= keep ? ((1u << (8u * keep)) - 1u) : 0u;
        }
        dst[j] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

__global__ __launch_bounds__(1024) void rx_cp_place_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t unit_log2, const uint4 *__restrict__ v, uint32_t n,
    uint32_t nflows, const uint2 *__restrict__ tiles, rxg_dgram *__restrict__ dg,
    uint8_t *__restrict__ payload, uint64_t cap, uint32_t *__restrict__ totals) {
    __shared__ uint32_t cnt[RX_CP_MAX_FLOWS], byt[RX_CP_MAX_FLOWS];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    for (uint32_t k = tid; k < nflows; k += 1024u) cnt[k] = byt[k] = 0u;
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * RX_CP_TILE + tid;
    const cp_frame f = cp_decode(v, len, i, n, nflows);
    const cp_group g = cp_groups(f, lane);
    // the waves' groups join the tile histogram in wave order: a lower wave's
    // datagrams of a socket precede a higher wave's (burst order)
    uint32_t oc = 0u, ob = 0u;
    for (uint32_t w = 0; w < RX_CP_WAVES; ++w) {
        if (w == wv && g.gcnt) {
            oc = atomicAdd(&cnt[f.flow], g.gcnt);
            ob = atomicAdd(&byt[f.flow], g.gbytes);
        }
        __syncthreads();
    }
    oc = __shfl(oc, (int)g.lead);
    ob = __shfl(ob, (int)g.lead);
    if (!f.deliv) return;
    const uint2 base = tiles[(uint64_t)blockIdx.x * nflows + f.flow];
    const uint32_t rank = base.x + oc + g.rank;
    const uint64_t boff = (uint64_t)base.y + ob + g.bpre;
    const uint8_t *fr = pkts + ((uint64_t)off[i] << unit_log2);
    const uint32_t cp = len[i];
    auto rd = [&](uint32_t k) -> uint32_t { return k < cp ? fr[k] : 0u; };
    rxg_dgram d;
    d.frame = (uint32_t)i;
    d.offset = (uint32_t)boff;
    d.sip = rd(26) | (rd(27) << 8) | (rd(28) << 16) | (rd(29) << 24);
    d.sport = (uint16_t)(rd(34) | (rd(35) << 8));
    d.len = (uint16_t)f.plen;
    dg[rank] = d;
    if (boff + f.padded <= cap)
        cp_copy(fr, cp, f.ncopy, reinterpret_cast<uint4 *>(payload + boff));
    else
        atomicOr(&totals[2], 1u); // payload buffer too small
}

} // namespace

size_t rx_compact_ws_bytes(uint32_t n, uint32_t nflows) {
    const uint64_t ntiles = ((uint64_t)n + RX_CP_TILE - 1) / RX_CP_TILE;
    return (size_t)(ntiles ? ntiles : 1) * nflows * sizeof(uint2);
}

// d_first: nflows + 1 entries; d_totals: 3 (datagrams, bytes, overflow flag)
hipError_t rx_compact_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                             uint32_t n, uint32_t unit_log2, const uint4 *verd, uint32_t nflows,
                             rxg_dgram *dg, uint32_t *first, uint8_t *payload, uint64_t cap,
                             uint32_t *totals, void *ws, hipStream_t s) {
    if (nflows == 0 || nflows > RX_CP_MAX_FLOWS) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(totals, 0, 3 * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t ntiles = (uint32_t)(((uint64_t)n + RX_CP_TILE - 1) / RX_CP_TILE);
    uint2 *tiles = static_cast<uint2 *>(ws);
    if (ntiles) {
        hipLaunchKernelGGL(rx_cp_count_kernel, dim3(ntiles), dim3(1024), 0, s, verd, len, n, nflows,
                           tiles);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(rx_cp_scan_kernel, dim3(1), dim3(1024), 0, s, tiles, ntiles, nflows, first,
                       totals);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (ntiles)
        hipLaunchKernelGGL(rx_cp_place_kernel, dim3(ntiles), dim3(1024), 0, s, pkts, off, len,
                           unit_log2, verd, n, nflows, tiles, dg, payload, cap, totals);
    return hipGetLastError();
}
