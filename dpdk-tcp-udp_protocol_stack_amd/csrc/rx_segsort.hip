// rx_segsort.hip — K4: per-connection segment sort and payload gather of a
// classified burst, the device half of TCP delivery.
//
// The reference hands every segment that found a tcb (tcp_process rc 0) to
// the state machine one frame at a time (tcp.c:373-415); an ESTABLISHED
// segment with PSH gets a malloc'd tcp_fragment holding a copy of its
// payload, queued on the tcb's receive ring (ng_tcp_enqueue_recvbuffer,
// tcp.c:133-185), and an ACK (tcp_handle_established, tcp.c:218-297).  A
// connection's segments must reach its state machine in burst order; segments
// of different connections are independent.  So one device pass here:
//   1. sorts the burst's rc-0 TCP segments by tcb id with a stable LSD radix
//      sort (8-bit digits, as many passes as the id space needs: 2 at 4096
//      tcbs, 3 at 1M), keys read straight from the verdicts in the first pass;
//   2. decodes, per sorted segment, the header fields the state machine reads
//      (flags, data offset, total length, seq / ack, ports) into a 32-B
//      record, and the payload length it will copy (PSH segments only);
//   3. gathers those payloads into one buffer in sorted order (16-B aligned
//      slots, a wave per segment), so each connection's payloads are one
//      contiguous slice: one allocation and one copy per connection per
//      burst on the host (host/nstack.c).
// Bytes past a frame's capture read as 0 (the delivery oracle's rule).
#include <hip/hip_runtime.h>

#include "rx_common.h"

#define SS_THREADS 256u
#define SS_ITEMS 8u
#define SS_TILE (SS_THREADS * SS_ITEMS) // keys per radix tile
#define SS_DIGITS 256u

namespace {

// inclusive scan over the 64 lanes of a wave (all lanes active): DPP row
// shifts inside each row of 16, then the row broadcasts across rows
__device__ __forceinline__ uint32_t ss_wave_scan(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xC, 0xF, false);
    return x;
}

// sort key of frame i in the first pass: its tcb id for a delivered TCP
// segment (class TCP, rc 0, id inside the id space), else the sentinel nt,
// which sorts after every id
__device__ __forceinline__ uint32_t ss_key0(const uint4 *__restrict__ v, uint64_t i, uint32_t nt) {
    const uint4 x = v[i];
    const uint32_t cls = (x.z >> 16) & 0xFFu;
    const int32_t rc = (int8_t)(x.z >> 24);
    return (cls == RXG_CLS_TCP && rc == RXG_RC_OK && x.x < nt) ? x.x : nt;
}

// digit histogram of one tile, digit-major (hist[d * ntiles + tile]), so one
// exclusive scan over the whole array gives every (digit, tile) its first
// output position; the first pass also counts the delivered segments
template <bool FIRST>
__global__ __launch_bounds__(SS_THREADS) void ss_hist_kernel(const uint4 *__restrict__ v,
                                                             const uint32_t *__restrict__ keys,
                                                             uint32_t n, uint32_t nt, uint32_t shift,
                                                             uint32_t ntiles, uint32_t *__restrict__ hist,
                                                             uint32_t *__restrict__ totals) {
    __shared__ uint32_t h[SS_DIGITS];
    const uint32_t t = threadIdx.x;
    h[t] = 0u;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * SS_TILE;
    uint32_t elig = 0u;
#pragma unroll
    for (uint32_t r = 0; r < SS_ITEMS; ++r) {
        const uint64_t i = base + r * SS_THREADS + t;
        if (i < n) {
            const uint32_t k = FIRST ? ss_key0(v, i, nt) : keys[i];
            elig += k < nt;
            atomicAdd(&h[(k >> shift) & 0xFFu], 1u);
        }
    }
    __syncthreads();
    hist[(uint64_t)t * ntiles + blockIdx.x] = h[t];
    if (FIRST) {
        for (int o = 32; o > 0; o >>= 1) elig += __shfl_xor(elig, o);
        if ((t & 63u) == 0u && elig) atomicAdd(&totals[0], elig);
    }
}

// exclusive scan of a[0..m) in place, one block (a thread per contiguous
// chunk); *total (nullable) = the sum
__global__ __launch_bounds__(1024) void ss_scan_kernel(uint32_t *__restrict__ a, uint32_t m,
                                                       uint32_t *__restrict__ total) {
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t per = (m + 1023u) / 1024u;
    const uint32_t b0 = min(m, t * per), b1 = min(m, b0 + per);
    uint32_t s = 0u;
    for (uint32_t k = b0; k < b1; ++k) s += a[k];
    const uint32_t inc = ss_wave_scan(s);
    if (lane == 63u) ws[w] = inc;
    __syncthreads();
    uint32_t run = inc - s;
    for (uint32_t q = 0; q < w; ++q) run += ws[q];
    if (t == 1023u && total) *total = run + s;
    for (uint32_t k = b0; k < b1; ++k) {
        const uint32_t x = a[k];
        a[k] = run;
        run += x;
    }
}

// stable scatter of one tile by digit: the tile's keys are taken in index
// order, 256 at a time; a wave ranks its lanes among those with the same
// digit (8 ballots: the lanes agreeing on every digit bit), the waves' digit
// counts meet in LDS in wave order, and every key lands after the tile's
// earlier keys of its digit and after every earlier tile's (the scanned
// histogram)
template <bool FIRST>
__global__ __launch_bounds__(SS_THREADS) void ss_scatter_kernel(
    const uint4 *__restrict__ v, const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
    uint32_t n, uint32_t nt, uint32_t shift, uint32_t ntiles, const uint32_t *__restrict__ hist,
    uint32_t *__restrict__ kout, uint32_t *__restrict__ vout) {
    __shared__ uint32_t base[SS_DIGITS];
    __shared__ uint32_t cnt[SS_THREADS / 64u][SS_DIGITS];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    base[t] = hist[(uint64_t)t * ntiles + blockIdx.x];
    const uint64_t tile0 = (uint64_t)blockIdx.x * SS_TILE;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t r = 0; r < SS_ITEMS; ++r) {
        const uint64_t i = tile0 + r * SS_THREADS + t;
        const bool ok = i < n;
        uint32_t key = 0u, val = 0u;
        if (ok) {
            key = FIRST ? ss_key0(v, i, nt) : kin[i];
            val = FIRST ? (uint32_t)i : vin[i];
        }
        const uint32_t d = (key >> shift) & 0xFFu;
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (uint32_t b = 0; b < 8u; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & below);
#pragma unroll
        for (uint32_t q = 0; q < SS_THREADS / 64u; ++q) cnt[q][t] = 0u;
        __syncthreads();
        if (ok && rank == 0u) cnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (ok) {
            uint32_t pos = base[d] + rank;
            for (uint32_t q = 0; q < w; ++q) pos += cnt[q][d];
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
        uint32_t add = 0u;
#pragma unroll
        for (uint32_t q = 0; q < SS_THREADS / 64u; ++q) add += cnt[q][t];
        base[t] += add;
    }
}

// one record per sorted segment (j < the delivered count): the header fields
// the state machine reads, and the payload it keeps (PSH and plen > 0:
// tcp.c:153-166; the captured part); the block's exclusive scan of the
// 16-B-padded payload sizes gives each its offset inside the block's slice,
// tsum[block] the slice's size (0 for blocks past the count)
template <bool INPLACE>
__global__ __launch_bounds__(SS_THREADS) void ss_record_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t unit_log2, const uint32_t *__restrict__ keys,
    const uint32_t *__restrict__ vals, const uint32_t *__restrict__ totals,
    rxg_segment *__restrict__ seg, uint32_t *__restrict__ tsum) {
    __shared__ uint32_t ws[SS_THREADS / 64u];
    const uint32_t nseg = totals[0];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t j = blockIdx.x * SS_THREADS + t;
    if (blockIdx.x * SS_THREADS >= nseg) { // (uniform)
        if (t == 0u && !INPLACE) tsum[blockIdx.x] = 0u;
        return;
    }
    rxg_segment s;
    uint32_t padded = 0u;
    if (j < nseg) {
        const uint32_t i = vals[j];
        const uint8_t *f = pkts + ((uint64_t)off[i] << unit_log2);
        const uint32_t cap = len[i];
        auto b = [&](uint32_t k) -> uint32_t { return k < cap ? (uint32_t)f[k] : 0u; };
        const uint32_t tl = (b(16) << 8) | b(17); // ip total_length (tcp.c:391)
        s.frame = i;
        s.flow = keys[j];
        s.seq = (b(38) << 24) | (b(39) << 16) | (b(40) << 8) | b(41);
        s.ack = (b(42) << 24) | (b(43) << 16) | (b(44) << 8) | b(45);
        s.hl = (uint8_t)(b(46) >> 4);
        s.flags = (uint8_t)b(47);
        s.plen = (int32_t)tl - 20 - 4 * (int32_t)s.hl; // tcp.c:145-146 with iTcplen = tl - 20
        s.sport = (uint16_t)(b(34) | (b(35) << 8));
        s.dport = (uint16_t)(b(36) | (b(37) << 8));
        const uint32_t from = 34u + 4u * s.hl;
        const uint32_t avail = cap > from ? cap - from : 0u;
        const uint32_t keep = ((s.flags & 0x08u) && s.plen > 0) ? min((uint32_t)s.plen, avail) : 0u;
        s.ncopy = (uint16_t)keep;
        padded = (keep + 15u) & ~15u;
    }
    if constexpr (INPLACE) { // the payload stays in the frame: bytes [34 + 4*hl, + ncopy)
        if (j < nseg) {
            s.offset = 34u + 4u * s.hl;
            seg[j] = s;
        }
        return;
    }
    const uint32_t inc = ss_wave_scan(padded);
    if (lane == 63u) ws[w] = inc;
    __syncthreads();
    uint32_t o = inc - padded;
    for (uint32_t q = 0; q < w; ++q) o += ws[q];
    if (t == SS_THREADS - 1u) tsum[blockIdx.x] = o + padded;
    if (j < nseg) {
        s.offset = o; // + the block's base (ss_copy_kernel)
        seg[j] = s;
    }
}

// a wave per segment: its final offset (block base added), then its payload,
// bytes [34 + 4*hl, + ncopy) of the frame, as 16-B chunks (dword loads below
// the capture, realigned with v_alignbyte), zero to the 16-B padded end
__global__ __launch_bounds__(SS_THREADS) void ss_copy_kernel(
    const uint8_t *__restrict__ pkts, const uint32_t *__restrict__ off,
    const uint16_t *__restrict__ len, uint32_t unit_log2, const uint32_t *__restrict__ tbase,
    rxg_segment *__restrict__ seg, uint8_t *__restrict__ payload, uint64_t cap,
    uint32_t *__restrict__ totals) {
    const uint32_t nseg = totals[0];
    const uint32_t j = blockIdx.x * (SS_THREADS / 64u) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (j >= nseg) return;
    const rxg_segment s = seg[j];
    const uint64_t o = (uint64_t)s.offset + tbase[j / SS_THREADS];
    if (lane == 0u) seg[j].offset = (uint32_t)o;
    if (!s.ncopy) return;
    const uint32_t ncopy = s.ncopy;
    if (o + ((ncopy + 15u) & ~15u) > cap) {
        if (lane == 0u) atomicOr(&totals[2], 1u); // payload buffer too small
        return;
    }
    const uint8_t *f = pkts + ((uint64_t)off[s.frame] << unit_log2);
    const uint32_t fcap = len[s.frame];
    const uint32_t src = 34u + 4u * s.hl;
    for (uint32_t c = lane; 16u * c < ncopy; c += 64u) {
        const uint32_t a = src + 16u * c, a0 = a & ~3u, sh = a & 3u;
        uint32_t wv[5];
#pragma unroll
        for (uint32_t q = 0; q < 5u; ++q) {
            const uint32_t p = a0 + 4u * q;
            wv[q] = p < fcap ? *reinterpret_cast<const uint32_t *>(f + p) : 0u;
        }
        uint32_t o4[4];
#pragma unroll
        for (uint32_t q = 0; q < 4u; ++q) {
            o4[q] = sh ? __builtin_amdgcn_alignbyte(wv[q + 1], wv[q], sh) : wv[q];
            const uint32_t b0 = 16u * c + 4u * q;
            const uint32_t keep = ncopy > b0 ? ncopy - b0 : 0u;
            if (keep < 4u) o4[q] &= keep ? ((1u << (8u * keep)) - 1u) : 0u;
        }
        *reinterpret_cast<uint4 *>(payload + o + 16u * c) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
    }
}

inline uint32_t ss_tiles(uint32_t n) { return (uint32_t)(((uint64_t)n + SS_TILE - 1) / SS_TILE); }
inline uint32_t ss_blocks(uint32_t n) { return (uint32_t)(((uint64_t)n + SS_THREADS - 1) / SS_THREADS); }
inline size_t ss_align(size_t x) { return (x + 255) & ~(size_t)255; }

} // namespace

// workspace: keys and values twice (ping-pong), the digit histograms, the
// record blocks' payload sizes
size_t rx_segsort_ws_bytes(uint32_t n) {
    const size_t nn = n ? n : 1;
    return 4 * ss_align(nn * 4) + ss_align((size_t)SS_DIGITS * (ss_tiles(n) ? ss_tiles(n) : 1) * 4) +
           ss_align((size_t)(ss_blocks(n) ? ss_blocks(n) : 1) * 4);
}

// d_totals: 3 (segments, payload bytes, overflow flag)
hipError_t rx_segsort_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                             uint32_t n, uint32_t unit_log2, const uint4 *verd, uint32_t nt,
                             rxg_segment *seg, uint8_t *payload, uint64_t cap, uint32_t *totals,
                             void *ws, hipStream_t s) {
    hipError_t e = hipMemsetAsync(totals, 0, 3 * sizeof(uint32_t), s);
    if (e != hipSuccess || n == 0 || nt == 0) return e;
    const size_t nn = ss_align((size_t)n * 4);
    uint8_t *w8 = static_cast<uint8_t *>(ws);
    uint32_t *ka = reinterpret_cast<uint32_t *>(w8), *va = reinterpret_cast<uint32_t *>(w8 + nn);
    uint32_t *kb = reinterpret_cast<uint32_t *>(w8 + 2 * nn), *vb = reinterpret_cast<uint32_t *>(w8 + 3 * nn);
    const uint32_t ntiles = ss_tiles(n), nblk = ss_blocks(n);
    uint32_t *hist = reinterpret_cast<uint32_t *>(w8 + 4 * nn);
    uint32_t *tsum = reinterpret_cast<uint32_t *>(w8 + 4 * nn + ss_align((size_t)SS_DIGITS * ntiles * 4));
    // key bits: ids 0..nt-1 and the sentinel nt
    const uint32_t bits = 32u - (uint32_t)__builtin_clz(nt);
    const uint32_t passes = (bits + 7u) / 8u;
    const uint32_t *kin = nullptr, *vin = nullptr;
    uint32_t *kout = ka, *vout = va;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t shift = 8u * p;
        if (p == 0)
            hipLaunchKernelGGL(ss_hist_kernel<true>, dim3(ntiles), dim3(SS_THREADS), 0, s, verd,
                               nullptr, n, nt, shift, ntiles, hist, totals);
        else
            hipLaunchKernelGGL(ss_hist_kernel<false>, dim3(ntiles), dim3(SS_THREADS), 0, s, verd,
                               kin, n, nt, shift, ntiles, hist, totals);
        hipLaunchKernelGGL(ss_scan_kernel, dim3(1), dim3(1024), 0, s, hist, SS_DIGITS * ntiles,
                           nullptr);
        if (p == 0)
            hipLaunchKernelGGL(ss_scatter_kernel<true>, dim3(ntiles), dim3(SS_THREADS), 0, s, verd,
                               nullptr, nullptr, n, nt, shift, ntiles, hist, kout, vout);
        else
            hipLaunchKernelGGL(ss_scatter_kernel<false>, dim3(ntiles), dim3(SS_THREADS), 0, s, verd,
                               kin, vin, n, nt, shift, ntiles, hist, kout, vout);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        kin = kout, vin = vout;
        kout = (kout == ka) ? kb : ka;
        vout = (vout == va) ? vb : va;
    }
    if (!payload) { // in place: records only, offset = the payload's offset in its frame
        hipLaunchKernelGGL(ss_record_kernel<true>, dim3(nblk), dim3(SS_THREADS), 0, s, pkts, off,
                           len, unit_log2, kin, vin, totals, seg, tsum);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(ss_record_kernel<false>, dim3(nblk), dim3(SS_THREADS), 0, s, pkts, off, len,
                       unit_log2, kin, vin, totals, seg, tsum);
    hipLaunchKernelGGL(ss_scan_kernel, dim3(1), dim3(1024), 0, s, tsum, nblk, totals + 1);
    hipLaunchKernelGGL(ss_copy_kernel, dim3((uint32_t)(((uint64_t)n + 3) / 4)), dim3(SS_THREADS), 0,
                       s, pkts, off, len, unit_log2, tsum, seg, payload, cap, totals);
    return hipGetLastError();
}
