// membw_large.hip — read-bandwidth ceilings for the large-frame workloads
// (diagnostics only; not part of the product).  6 GiB buffer (cfg3's burst
// size): plain coalesced streams at several loads-in-flight depths, and the
// cfg3 access pattern (1504 of every 1536 bytes read by 8-lane groups, one
// 16-B store per 1536-B slot) with no per-frame work.
//   hipcc --offload-arch=gfx950 -O3 tools/membw_large.hip -o tools/membw_large
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

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// U loads per lane per trip, each wave-instruction 1 KiB contiguous
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_stream(const u32x4 *__restrict__ in, size_t n16,
                                                unsigned *__restrict__ out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld<NT>(in + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) {
        u32x4 v = ld<NT>(in + i);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// cfg3 pattern: group of 8 lanes per 1536-B slot, 12 passes of 128 B (the
// last one 96 B: 1504 bytes), U passes in flight; lane 0 stores 16 B
template <bool NT, int U>
__global__ __launch_bounds__(256) void k_slot(const u32x4 *__restrict__ in, size_t nslots,
                                              u32x4 *__restrict__ out) {
    const unsigned gl = threadIdx.x & 7u;
    const size_t groups = (size_t)gridDim.x * 32;
    for (size_t f = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3); f < nslots; f += groups) {
        const u32x4 *p = in + f * 96; // 1536 B = 96 chunks
        unsigned acc = 0;
#pragma unroll
        for (int b = 0; b < 12; b += U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const unsigned c = (b + u) * 8 + gl;
                v[u] = (b + u < 12 && c < 94) ? ld<NT>(p + c) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (gl == 0) {
            u32x4 w = {acc, (unsigned)f, 0, 0};
            __builtin_nontemporal_store(w, out + f);
        }
    }
}

// group of G lanes per 1536-B slot (ceil(94/G) passes, all in flight), frames
// grid-strided over groups
template <int G>
__global__ __launch_bounds__(256) void k_slotg(const u32x4 *__restrict__ in, size_t nslots,
                                               u32x4 *__restrict__ out) {
    constexpr int PASSES = (94 + G - 1) / G;
    const unsigned gl = threadIdx.x & (G - 1);
    const size_t groups = (size_t)gridDim.x * (256 / G);
    for (size_t f = (size_t)blockIdx.x * (256 / G) + threadIdx.x / G; f < nslots; f += groups) {
        const u32x4 *p = in + f * 96;
        u32x4 v[PASSES];
#pragma unroll
        for (int q = 0; q < PASSES; ++q) {
            const unsigned c = q * G + gl;
            v[q] = c < 94 ? ld<true>(p + c) : u32x4{0, 0, 0, 0};
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < PASSES; ++q) acc += v[q].x + v[q].y + v[q].z + v[q].w;
        for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o);
        if (gl == 0) {
            u32x4 w = {acc, (unsigned)f, 0, 0};
            __builtin_nontemporal_store(w, out + f);
        }
    }
}

// a wave streams W consecutive slots (W*96 chunks, 1 KiB contiguous per
// instruction, all passes in flight); chunk c counts if c % 96 < 94
template <int W>
__global__ __launch_bounds__(256) void k_wavestream(const u32x4 *__restrict__ in, size_t nslots,
                                                    u32x4 *__restrict__ out) {
    constexpr int PASSES = W * 96 / 64;
    const unsigned lane = threadIdx.x & 63u;
    const size_t nw = (size_t)gridDim.x * 4;
    for (size_t t = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); t * W < nslots; t += nw) {
        const u32x4 *p = in + t * W * 96;
        u32x4 v[PASSES];
#pragma unroll
        for (int q = 0; q < PASSES; ++q) v[q] = ld<true>(p + q * 64 + lane);
        unsigned acc[W];
#pragma unroll
        for (int f = 0; f < W; ++f) acc[f] = 0;
#pragma unroll
        for (int q = 0; q < PASSES; ++q) {
            const unsigned c = q * 64 + lane, f = c / 96, r = c % 96;
            const unsigned s = r < 94 ? v[q].x + v[q].y + v[q].z + v[q].w : 0u;
#pragma unroll
            for (int k = 0; k < W; ++k) acc[k] += f == (unsigned)k ? s : 0u;
        }
#pragma unroll
        for (int f = 0; f < W; ++f)
            for (int o = 1; o < 64; o <<= 1) acc[f] += __shfl_xor(acc[f], o);
        if (lane < W) {
            unsigned a = acc[0];
#pragma unroll
            for (int f = 1; f < W; ++f) a = lane == (unsigned)f ? acc[f] : a;
            u32x4 w = {a, (unsigned)(t * W + lane), 0, 0};
            __builtin_nontemporal_store(w, out + t * W + lane);
        }
    }
}

// block-tile stream: a block owns T consecutive slots per trip and its 256
// lanes stream the tile's T*96 chunks (1 KiB contiguous per instruction,
// ceil(T*96/256) loads per lane); per-slot sums meet in LDS; tiles are
// grid-strided, so the resident blocks read one compact window
template <int T>
__global__ __launch_bounds__(256) void k_tile(const u32x4 *__restrict__ in, size_t nslots,
                                              u32x4 *__restrict__ out) {
    constexpr int CH = T * 96, PER = (CH + 255) / 256;
    __shared__ unsigned acc[2][T];
    const unsigned tid = threadIdx.x;
    unsigned b = 0;
    for (size_t tile = blockIdx.x; tile * T < nslots; tile += gridDim.x, b ^= 1) {
        if (tid < T) acc[b][tid] = 0;
        const u32x4 *p = in + tile * T * 96;
        u32x4 v[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const unsigned j = u * 256 + tid;
            v[u] = ld<true>(p + (j < CH ? j : 0));
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const unsigned j = u * 256 + tid, f = j / 96, r = j % 96;
            if (j < CH && r < 94) atomicAdd(&acc[b][f], v[u].x + v[u].y + v[u].z + v[u].w);
        }
        __syncthreads();
        if (tid < T) {
            u32x4 w = {acc[b][tid], (unsigned)(tile * T + tid), 0, 0};
            __builtin_nontemporal_store(w, out + tile * T + tid);
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
    u32x4 *in, *out;
    unsigned *sink;
    CHK(hipMalloc(&in, bytes));
    CHK(hipMalloc(&out, nslots * 16));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(in, 1, bytes));
    int cu = 0;
    CHK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = 20;
    for (int bpc : {1, 2, 4, 8, 16}) {
        const int g = cu * bpc;
        float ms = timeit([&] { k_stream<true, 1><<<g, 256>>>(in, bytes / 16, sink); }, reps);
        printf("bpc=%d stream nt=1 U=1          %.3f ms %7.0f GB/s\n", bpc, ms, bytes / ms / 1e6);
        const double alg = (double)nslots * (1500 + 22);
#define TT(T)                                                                                      \
    ms = timeit([&] { k_tile<T><<<g, 256>>>(in, nslots, out); }, reps);                            \
    printf("bpc=%d tile T=%d               %.3f ms %7.0f GB/s(alg)\n", bpc, T, ms, alg / ms / 1e6);
        TT(2) TT(4) TT(8) TT(16)
#undef TT
    }
    for (int bpc : {4, 8}) {
        const int g = cu * bpc;
        float ms;
#define S(NT, U)                                                                                   \
    ms = timeit([&] { k_stream<NT, U><<<g, 256>>>(in, bytes / 16, sink); }, reps);                 \
    printf("bpc=%d stream nt=%d U=%d          %.3f ms %7.0f GB/s\n", bpc, NT, U, ms, bytes / ms / 1e6);
        S(false, 1) S(true, 1) S(false, 4) S(true, 4) S(true, 8)
#undef S
        const double alg = (double)nslots * (1500 + 22);
#define L(NT, U)                                                                                   \
    ms = timeit([&] { k_slot<NT, U><<<g, 256>>>(in, nslots, out); }, reps);                        \
    printf("bpc=%d slot1536 nt=%d U=%d        %.3f ms %7.0f GB/s(alg 1522 B/frame)\n", bpc, NT, U, ms, \
           alg / ms / 1e6);
        L(false, 2) L(true, 2) L(true, 4) L(true, 6) L(true, 12)
#undef L
#define GG(G)                                                                                      \
    ms = timeit([&] { k_slotg<G><<<g, 256>>>(in, nslots, out); }, reps);                           \
    printf("bpc=%d slotg G=%d              %.3f ms %7.0f GB/s(alg)\n", bpc, G, ms, alg / ms / 1e6);
        GG(8) GG(16) GG(32) GG(64)
#undef GG
#define WS(W)                                                                                      \
    ms = timeit([&] { k_wavestream<W><<<g, 256>>>(in, nslots, out); }, reps);                      \
    printf("bpc=%d wavestream W=%d         %.3f ms %7.0f GB/s(alg)\n", bpc, W, ms, alg / ms / 1e6);
        WS(2) WS(4) WS(8)
#undef WS
    }
    return 0;
}
