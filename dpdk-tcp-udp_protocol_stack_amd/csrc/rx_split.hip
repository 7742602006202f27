// rx_split.hip — RSS split and shard gather (gfx950): the multi-GPU ingest of
// the rx path.
//
// The reference configures ONE rx queue (ng_init_port, netfamily.c:38-39) and
// dequeues one burst of it at a time (netfamily.c:147); the multi-queue NIC
// its README assumes (README.md:13) would spread flows over queues by an RSS
// hash.  Here a burst is split over n_shards ranks (GPUs) the same way: shard
// of a frame = rx_rss_frame (Toeplitz over the IP/port tuple, rx_common.h)
// mod n_shards.  The split keeps a permutation back to the burst index, so
// per-shard verdicts re-ordered by it equal the one-GPU verdicts (SURVEY.md
// §8(e)), and a gather packs one shard's frames into a contiguous burst (the
// NIC's DMA into that queue's ring) for the GPU that owns the shard.
//
// Kernels (all stable: frames keep their burst order inside a shard):
//   split_count   one block per 4096-frame chunk: shard of every frame (one
//                 byte per frame into the workspace), per-chunk shard counts
//   scan_u64      one block: exclusive prefix sum of a count array in place
//   split_scatter one block per chunk: frame indices to perm[] at the scanned
//                 chunk/shard base plus the frame's rank among same-shard
//                 frames of the chunk before it (wave ballots, in order)
//   gather_units / gather_offsets / gather_copy: 64-B units per frame, their
//                 exclusive scan (packed destination offsets), the copy by
//                 lane groups of 16 (16-B chunks)
#include <hip/hip_runtime.h>
#include <string.h>

#include <new>

#include "rx_common.h"
#include "rx_device.h"

namespace {

constexpr uint32_t SPLIT_CHUNK = 4096; // frames per split / gather block
constexpr uint32_t SPLIT_PER_THREAD = SPLIT_CHUNK / 256;

__device__ __forceinline__ uint32_t frame_shard(const uint8_t *__restrict__ pkts, uint32_t off,
                                                uint32_t cap, uint32_t unit_log2, uint32_t nsh) {
    const uint8_t *fb = pkts + ((uint64_t)off << unit_log2);
    uint32_t w[12];
#pragma unroll
    for (int j = 0; j < 3; ++j) { // bytes [0, 48): the buffer extends to each frame's 16-B end
        uint4 c = ldg16<false>(fb + (16 * j < (int32_t)cap ? 16 * j : 0));
        c = chunk_below(c, 16 * j, (int32_t)cap);
        w[4 * j] = c.x, w[4 * j + 1] = c.y, w[4 * j + 2] = c.z, w[4 * j + 3] = c.w;
    }
    return rx_rss_frame(w) % nsh;
}

// counts[s * nchunks + chunk] = frames of `chunk` in shard s; shard ids to sh[]
__global__ __launch_bounds__(256) void split_count_kernel(const uint8_t *__restrict__ pkts,
                                                          const uint32_t *__restrict__ off,
                                                          const uint16_t *__restrict__ len,
                                                          uint32_t n, uint32_t unit_log2,
                                                          uint32_t nsh, uint8_t *__restrict__ sh,
                                                          unsigned long long *__restrict__ counts) {
    __shared__ uint32_t cnt[RX_MAX_SHARDS];
    const uint32_t tid = threadIdx.x, chunk = blockIdx.x;
    if (tid < RX_MAX_SHARDS) cnt[tid] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)chunk * SPLIT_CHUNK;
#pragma unroll 4
    for (uint32_t k = 0; k < SPLIT_PER_THREAD; ++k) {
        const uint64_t i = base + (uint64_t)k * 256 + tid;
        if (i < n) {
            const uint32_t s = frame_shard(pkts, off[i], len[i], unit_log2, nsh);
            sh[i] = (uint8_t)s;
            atomicAdd(&cnt[s], 1u);
        }
    }
    __syncthreads();
    if (tid < nsh) counts[(uint64_t)tid * gridDim.x + chunk] = cnt[tid];
}

// exclusive prefix sum of v[0..m) in place, one 1024-thread block; *total = sum
__global__ __launch_bounds__(1024) void scan_u64_kernel(unsigned long long *__restrict__ v,
                                                        uint64_t m,
                                                        unsigned long long *__restrict__ total) {
    __shared__ unsigned long long part[1024];
    const uint32_t tid = threadIdx.x;
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t b = tid * per, e = b + per < m ? b + per : m;
    unsigned long long s = 0;
    for (uint64_t i = b; i < e; ++i) s += v[i];
    part[tid] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) { // Hillis-Steele over the 1024 segment sums
        const unsigned long long x = tid >= o ? part[tid - o] : 0ull;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    unsigned long long run = part[tid] - s; // exclusive
    for (uint64_t i = b; i < e; ++i) {
        const unsigned long long x = v[i];
        v[i] = run;
        run += x;
    }
    if (tid == 1023 && total) *total = part[1023];
}

// perm[base(s, chunk) + rank] = i, in burst order inside each shard
__global__ __launch_bounds__(256) void split_scatter_kernel(const uint8_t *__restrict__ sh,
                                                            uint32_t n, uint32_t nsh,
                                                            const unsigned long long *__restrict__ base,
                                                            uint32_t *__restrict__ perm) {
    __shared__ uint32_t run[RX_MAX_SHARDS];       // next slot of each shard (chunk-relative)
    __shared__ uint32_t wcnt[4][RX_MAX_SHARDS];   // per-wave counts of one 256-frame step
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6, chunk = blockIdx.x;
    if (tid < RX_MAX_SHARDS) run[tid] = 0;
    const uint64_t c0 = (uint64_t)chunk * SPLIT_CHUNK;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t k = 0; k < SPLIT_PER_THREAD; ++k) {
        const uint64_t i = c0 + (uint64_t)k * 256 + tid;
        const bool valid = i < n;
        const uint32_t s = valid ? sh[i] : 0xFFu;
        if (tid < 4 * RX_MAX_SHARDS) (&wcnt[0][0])[tid] = 0;
        __syncthreads();
        // rank among this wave's lanes below with the same shard: one ballot
        // per distinct shard present in the wave
        uint32_t rank = 0;
        uint64_t todo = __ballot(valid);
        while (todo) { // wave-uniform
            const uint32_t leader = (uint32_t)__builtin_ctzll(todo);
            const uint32_t ls = __shfl(s, leader);
            const uint64_t m = __ballot(valid && s == ls);
            if (valid && s == ls) rank = (uint32_t)__popcll(m & below);
            if (lane == leader) wcnt[wv][ls] = (uint32_t)__popcll(m);
            todo &= ~m;
        }
        __syncthreads();
        if (valid) {
            uint32_t pos = run[s] + rank;
            for (uint32_t w = 0; w < wv; ++w) pos += wcnt[w][s];
            perm[base[(uint64_t)s * gridDim.x + chunk] + pos] = (uint32_t)i;
        }
        __syncthreads();
        if (tid < nsh) run[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
        __syncthreads(); // before the next step resets wcnt
    }
}

// first[s] = scanned base of (shard s, chunk 0); first[nsh] = n
__global__ void split_first_kernel(const unsigned long long *__restrict__ base, uint32_t nchunks,
                                   uint32_t nsh, uint32_t n, uint32_t *__restrict__ first) {
    const uint32_t k = threadIdx.x;
    if (k < nsh) first[k] = nchunks ? (uint32_t)base[(uint64_t)k * nchunks] : 0u;
    if (k == nsh) first[k] = n;
}

__device__ __forceinline__ uint32_t frame_units(uint32_t l) { // 64-B units, >= 1
    return l ? (l + 63u) >> 6 : 1u;
}

// per-chunk sums of the destination units of frames idx[0..count)
__global__ __launch_bounds__(256) void gather_units_kernel(const uint16_t *__restrict__ len,
                                                           const uint32_t *__restrict__ idx,
                                                           uint32_t count,
                                                           unsigned long long *__restrict__ sums) {
    __shared__ uint32_t part[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t c0 = (uint64_t)blockIdx.x * SPLIT_CHUNK;
    uint32_t s = 0;
    for (uint32_t k = 0; k < SPLIT_PER_THREAD; ++k) {
        const uint64_t q = c0 + (uint64_t)k * 256 + tid;
        if (q < count) s += frame_units(len[idx[q]]);
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((tid & 63u) == 0) part[tid >> 6] = s;
    __syncthreads();
    if (tid == 0) sums[blockIdx.x] = (unsigned long long)part[0] + part[1] + part[2] + part[3];
}

// destination offsets (64-B units) and lengths, in order inside each chunk
__global__ __launch_bounds__(256) void gather_offsets_kernel(const uint16_t *__restrict__ len,
                                                             const uint32_t *__restrict__ idx,
                                                             uint32_t count,
                                                             const unsigned long long *__restrict__ base,
                                                             uint32_t *__restrict__ dst_off,
                                                             uint16_t *__restrict__ dst_len) {
    __shared__ unsigned long long run;
    __shared__ uint32_t wsum[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (tid == 0) run = base[blockIdx.x];
    const uint64_t c0 = (uint64_t)blockIdx.x * SPLIT_CHUNK;
    for (uint32_t k = 0; k < SPLIT_PER_THREAD; ++k) {
        const uint64_t q = c0 + (uint64_t)k * 256 + tid;
        const uint32_t l = q < count ? len[idx[q]] : 0u;
        const uint32_t u = q < count ? frame_units(l) : 0u;
        uint32_t x = u; // inclusive wave scan
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        unsigned long long p = run + x - u;
        for (uint32_t w = 0; w < wv; ++w) p += wsum[w];
        if (q < count) {
            dst_off[q] = (uint32_t)p;
            dst_len[q] = (uint16_t)l;
        }
        __syncthreads();
        if (tid == 0) run += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

// copy: 16 lanes per frame (4 frames per wave), 16-B chunks up to the
// frame's 16-B end; a frame whose destination ends past cap is not copied
__global__ __launch_bounds__(256) void gather_copy_kernel(const uint8_t *__restrict__ pkts,
                                                          const uint32_t *__restrict__ off,
                                                          uint32_t unit_log2,
                                                          const uint32_t *__restrict__ idx,
                                                          uint32_t count,
                                                          const uint32_t *__restrict__ dst_off,
                                                          const uint16_t *__restrict__ dst_len,
                                                          uint8_t *__restrict__ dst, uint64_t cap) {
    const uint64_t q = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const uint32_t gl = threadIdx.x & 15u;
    if (q >= count) return;
    const uint32_t l = dst_len[q];
    const uint64_t d = (uint64_t)dst_off[q] << 6;
    const uint64_t nb = (uint64_t)frame_units(l) << 6; // whole 64-B units (zero tail)
    if (d + nb > cap) return;
    const uint8_t *src = pkts + ((uint64_t)off[idx[q]] << unit_log2);
    const uint32_t l16 = (l + 15u) & ~15u; // the source owns bytes up to its 16-B end
    for (uint32_t s = 16 * gl; s < nb; s += 256) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (s < l16) v = chunk_below(ldg16<true>(src + s), (int32_t)s, (int32_t)l);
        *reinterpret_cast<uint4 *>(dst + d + s) = v;
    }
}

} // namespace

// ---- launchers (called by rx_api.hip's C ABI) -------------------------------

size_t rx_split_ws_bytes(uint32_t n, uint32_t nsh) {
    const uint64_t nchunks = ((uint64_t)n + SPLIT_CHUNK - 1) / SPLIT_CHUNK;
    return (((uint64_t)n + 255) & ~255ull) + nchunks * nsh * 8 + 8;
}

// first[s] (s <= nsh) = start of shard s in perm; first[nsh] = n
hipError_t rx_split_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                           uint32_t n, uint32_t unit_log2, uint32_t nsh, uint32_t *first,
                           uint32_t *perm, void *ws, hipStream_t s) {
    const uint32_t nchunks = (uint32_t)(((uint64_t)n + SPLIT_CHUNK - 1) / SPLIT_CHUNK);
    uint8_t *sh = reinterpret_cast<uint8_t *>(ws);
    unsigned long long *cnt =
        reinterpret_cast<unsigned long long *>(sh + (((uint64_t)n + 255) & ~255ull));
    hipError_t e = hipSuccess;
    if (nchunks) {
        hipLaunchKernelGGL(split_count_kernel, dim3(nchunks), dim3(256), 0, s, pkts, off, len, n,
                           unit_log2, nsh, sh, cnt);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(scan_u64_kernel, dim3(1), dim3(1024), 0, s, cnt,
                           (uint64_t)nchunks * nsh, (unsigned long long *)nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(split_scatter_kernel, dim3(nchunks), dim3(256), 0, s, sh, n, nsh, cnt,
                           perm);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(split_first_kernel, dim3(1), dim3(RX_MAX_SHARDS + 1), 0, s, cnt, nchunks, nsh,
                       n, first);
    return hipGetLastError();
}

size_t rx_gather_ws_bytes(uint32_t count) {
    const uint64_t nchunks = ((uint64_t)count + SPLIT_CHUNK - 1) / SPLIT_CHUNK;
    return nchunks * 8 + 8;
}

// *d_total (device) = 64-B units the packed shard occupies
hipError_t rx_gather_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                            uint32_t unit_log2, const uint32_t *idx, uint32_t count, uint8_t *dst,
                            uint64_t cap, uint32_t *dst_off, uint16_t *dst_len, void *ws,
                            hipStream_t s) {
    const uint32_t nchunks = (uint32_t)(((uint64_t)count + SPLIT_CHUNK - 1) / SPLIT_CHUNK);
    unsigned long long *sums = reinterpret_cast<unsigned long long *>(ws);
    unsigned long long *total = sums + nchunks;
    hipLaunchKernelGGL(gather_units_kernel, dim3(nchunks), dim3(256), 0, s, len, idx, count, sums);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(scan_u64_kernel, dim3(1), dim3(1024), 0, s, sums, (uint64_t)nchunks, total);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(gather_offsets_kernel, dim3(nchunks), dim3(256), 0, s, len, idx, count, sums,
                       dst_off, dst_len);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint64_t threads = (uint64_t)count * 16;
    hipLaunchKernelGGL(gather_copy_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s,
                       pkts, off, unit_log2, idx, count, dst_off, dst_len, dst, cap);
    return hipGetLastError();
}

// host split: the same shard function and the same stable order
extern "C" int rxg_rss_split(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                             uint32_t n, uint32_t off_unit_log2, uint32_t n_shards,
                             uint32_t *first, uint32_t *perm) {
    if (!first || n_shards == 0 || n_shards > RX_MAX_SHARDS) return RXG_EINVAL;
    if (n && (!pkts || !off || !len || !perm)) return RXG_EINVAL;
    if (off_unit_log2 > 16) return RXG_EINVAL;
    uint8_t *sh = new (std::nothrow) uint8_t[n ? n : 1];
    if (!sh) return RXG_ENOMEM;
    uint32_t cnt[RX_MAX_SHARDS + 1] = {0};
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *f = pkts + ((uint64_t)off[i] << off_unit_log2);
        uint32_t w[10];
        uint8_t b[40];
        for (uint32_t k = 0; k < 40; ++k) b[k] = k < len[i] ? f[k] : 0;
        memcpy(w, b, 40);
        sh[i] = (uint8_t)(rx_rss_frame(w) % n_shards);
        ++cnt[sh[i] + 1];
    }
    for (uint32_t s = 0; s < n_shards; ++s) cnt[s + 1] += cnt[s];
    for (uint32_t s = 0; s <= n_shards; ++s) first[s] = cnt[s];
    for (uint32_t i = 0; i < n; ++i) perm[cnt[sh[i]]++] = i;
    delete[] sh;
    return RXG_OK;
}

// ---------------------------------------------------------------------------
// Frames that live in registered host memory (rxg_register_host: the mbuf
// pool, pinned and mapped) into a staging burst on the device: the device
// pulls each frame over PCIe, as a NIC's DMA into the ring would, instead of
// a host memcpy into pinned staging followed by a copy.  Four lanes per
// frame, 16 frames per wave (a 64-B frame is one 16-B load per lane, so a
// wave instruction still moves 1 KiB), each group striding over its frame's
// 16-B chunks, four loads in flight per lane; stores at dst + (off << 6),
// bytes past the frame's length zeroed to its 64-B end (the staging layout
// the classify kernels read).  The host checked that every source is 16-B
// aligned and that its 16-B rounded end stays inside its registered region.
namespace {
__device__ __forceinline__ uint4 ingest_mask(uint4 v, uint32_t b, uint32_t l) {
    if (b >= l) return make_uint4(0u, 0u, 0u, 0u);
    if (b + 16u <= l) return v;
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t q = 0; q < 4u; ++q) {
        const uint32_t b0 = b + 4u * q;
        const uint32_t keep = l > b0 ? l - b0 : 0u;
        if (keep < 4u) w[q] &= keep ? ((1u << (8u * keep)) - 1u) : 0u;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ __launch_bounds__(256) void ingest_copy_kernel(const unsigned long long *__restrict__ src,
                                                          const uint32_t *__restrict__ off,
                                                          const uint16_t *__restrict__ len,
                                                          uint32_t n, uint8_t *__restrict__ dst) {
    const uint32_t f = blockIdx.x * 64u + (threadIdx.x >> 2), q = threadIdx.x & 3u;
    if (f >= n) return;
    const uint4 *s = reinterpret_cast<const uint4 *>(src[f]);
    const uint32_t l = len[f];
    const uint32_t nch = (l ? ((l + 63u) & ~63u) : 64u) >> 4; // chunks to the 64-B end
    const uint32_t nsrc = (l + 15u) >> 4;                     // chunks holding frame bytes
    uint4 *d = reinterpret_cast<uint4 *>(dst + ((uint64_t)off[f] << 6));
    for (uint32_t c0 = q; c0 < nch; c0 += 16u) {
        uint4 v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) {
            const uint32_t c = c0 + 4u * u;
            v[u] = c < nsrc ? s[c] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < 4u; ++u) {
            const uint32_t c = c0 + 4u * u;
            if (c < nch) d[c] = ingest_mask(v[u], 16u * c, l);
        }
    }
}
} // namespace

hipError_t rx_ingest_launch(const unsigned long long *src, const uint32_t *off, const uint16_t *len,
                            uint32_t n, uint8_t *dst, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(ingest_copy_kernel, dim3((n + 63u) / 64u), dim3(256), 0, s, src, off, len, n, dst);
    return hipGetLastError();
}
