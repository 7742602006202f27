// membw_window.hip — access-pattern study for 1536-B slot frames (cfg3 shape),
// diagnostics only, not part of the product.  Question: how close can a
// frame-aware read pattern (per-frame sums, one 16-B store per frame, an
// optional dependent table probe per frame) get to the plain grid-stride
// stream, as a function of resident blocks per CU (bytes in flight)?
//   hipcc --offload-arch=gfx950 -O3 tools/membw_window.hip -o tools/membw_window
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                                     \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                        \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldnt(const u32x4 *p) { return __builtin_nontemporal_load(p); }

__global__ __launch_bounds__(256) void k_stream(const u32x4 *__restrict__ in, size_t n16,
                                                unsigned *__restrict__ out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        u32x4 v = ldnt(in + i);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__device__ __forceinline__ unsigned wsum(unsigned a) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) a += __shfl_xor(a, o);
    return a;
}

// A wave owns W consecutive slots per trip (W*96 chunks = W*1.5 KiB, every
// wave instruction 1 KiB contiguous); wave tiles are grid-ordered (tile =
// trip * nwaves + global wave), so the resident waves read one compact
// window.  PIPE: the next trip's passes are issued before this trip's sums.
// PR: lane f < W probes tbl[hash(sum)] (a dependent load) before the store.
template <int W, bool PIPE, bool PR>
__global__ __launch_bounds__(256) void k_wave(const u32x4 *__restrict__ in, size_t nslots,
                                              const u32x4 *__restrict__ tbl, u32x4 *__restrict__ out) {
    constexpr int PASSES = W * 96 / 64;
    const unsigned lane = threadIdx.x & 63u;
    const size_t nw = (size_t)gridDim.x * 4;
    size_t t = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t ntiles = nslots / W;
    u32x4 v[PASSES], nx[PASSES];
    if (t < ntiles) {
#pragma unroll
        for (int q = 0; q < PASSES; ++q) v[q] = ldnt(in + t * W * 96 + q * 64 + lane);
    }
    for (; t < ntiles; t += nw) {
        const size_t tn = t + nw < ntiles ? t + nw : t;
        if constexpr (PIPE) {
#pragma unroll
            for (int q = 0; q < PASSES; ++q) nx[q] = ldnt(in + tn * W * 96 + q * 64 + lane);
        }
        unsigned acc[W];
#pragma unroll
        for (int f = 0; f < W; ++f) acc[f] = 0;
#pragma unroll
        for (int q = 0; q < PASSES; ++q) {
            const unsigned c = q * 64 + lane, r = c % 96;
            const unsigned s = r < 94 ? v[q].x + v[q].y + v[q].z + v[q].w : 0u;
            // chunk q*64+lane belongs to frame (q*64+lane)/96: at most 2 frames per pass
            const unsigned f0 = (q * 64) / 96;
#pragma unroll
            for (int k = 0; k < W; ++k)
                if (k == (int)f0 || k == (int)f0 + 1) acc[k] += (c / 96 == (unsigned)k) ? s : 0u;
        }
        unsigned mine = 0;
#pragma unroll
        for (int f = 0; f < W; ++f) {
            const unsigned a = wsum(acc[f]);
            mine = lane == (unsigned)f ? a : mine;
        }
        if (lane < W) {
            unsigned x = mine;
            if (PR) {
                const u32x4 sl = tbl[(mine * 2654435761u) >> 20]; // 4096-slot table
                x ^= sl.x;
            }
            u32x4 w = {x, (unsigned)(t * W + lane), 0, 0};
            __builtin_nontemporal_store(w, out + t * W + lane);
        }
        if constexpr (PIPE) {
#pragma unroll
            for (int q = 0; q < PASSES; ++q) v[q] = nx[q];
        } else if (t + nw < ntiles) {
#pragma unroll
            for (int q = 0; q < PASSES; ++q) v[q] = ldnt(in + (t + nw) * W * 96 + q * 64 + lane);
        }
    }
}

// G lanes per slot, all ceil(94/G) passes in flight, grid-ordered groups.
template <int G, bool PR>
__global__ __launch_bounds__(256) void k_grp(const u32x4 *__restrict__ in, size_t nslots,
                                             const u32x4 *__restrict__ tbl, u32x4 *__restrict__ out) {
    constexpr int PASSES = (94 + G - 1) / G;
    const unsigned gl = threadIdx.x & (G - 1);
    const size_t groups = (size_t)gridDim.x * (256 / G);
    for (size_t f = (size_t)blockIdx.x * (256 / G) + threadIdx.x / G; f < nslots; f += groups) {
        const u32x4 *p = in + f * 96;
        u32x4 v[PASSES];
#pragma unroll
        for (int q = 0; q < PASSES; ++q) {
            const unsigned c = q * G + gl;
            v[q] = ldnt(p + (c < 94 ? c : 0));
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < PASSES; ++q)
            acc += (q * G + gl < 94) ? v[q].x + v[q].y + v[q].z + v[q].w : 0u;
        for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o);
        if (gl == 0) {
            unsigned x = acc;
            if (PR) x ^= tbl[(acc * 2654435761u) >> 20].x;
            u32x4 w = {x, (unsigned)f, 0, 0};
            __builtin_nontemporal_store(w, out + f);
        }
    }
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    f();
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t nslots = 4u << 20, bytes = nslots * 1536;
    u32x4 *in, *out, *tbl;
    unsigned *sink;
    CHK(hipMalloc(&in, bytes));
    CHK(hipMalloc(&out, nslots * 16));
    CHK(hipMalloc(&tbl, 4096 * 16));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(in, 1, bytes));
    CHK(hipMemset(tbl, 0, 4096 * 16));
    int cu = 0;
    CHK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = 20;
    const double alg = (double)nslots * (1500 + 22);
    for (int bpc : {4, 6, 8, 10, 12}) {
        float ms = timeit([&] { k_stream<<<cu * bpc, 256>>>(in, bytes / 16, sink); }, reps);
        printf("bpc=%2d stream              %.3f ms %7.0f GB/s (raw)\n", bpc, ms, bytes / ms / 1e6);
    }
    for (int bpc : {1, 2, 3, 4, 6, 8}) {
        const int g = cu * bpc;
        float ms;
#define WV(W, PI, PR)                                                                              \
    ms = timeit([&] { k_wave<W, PI, PR><<<g, 256>>>(in, nslots, tbl, out); }, reps);              \
    printf("bpc=%2d wave W=%d pipe=%d pr=%d  %.3f ms %7.0f GB/s(alg)\n", bpc, W, PI, PR, ms,        \
           alg / ms / 1e6);
        WV(2, false, false) WV(2, true, false) WV(2, false, true) WV(2, true, true)
        WV(4, false, false) WV(4, true, true) WV(8, false, true)
#undef WV
#define GR(G, PR)                                                                                  \
    ms = timeit([&] { k_grp<G, PR><<<g, 256>>>(in, nslots, tbl, out); }, reps);                    \
    printf("bpc=%2d grp G=%d pr=%d          %.3f ms %7.0f GB/s(alg)\n", bpc, G, PR, ms, alg / ms / 1e6);
        GR(8, true) GR(16, true) GR(32, true)
#undef GR
    }
    return 0;
}
