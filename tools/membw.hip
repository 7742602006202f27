// membw.hip — access-pattern microbenchmark for the classify kernel's memory
// traffic (diagnostics only; not part of the product).  Reads a 1 GiB buffer of
// 64-B "frames" in the patterns K1 uses and reports achieved GB/s.
//   hipcc --offload-arch=gfx950 -O3 tools/membw.hip -o tools/membw && tools/membw
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

// (a) coalesced stream: each wave-instruction reads 1 KiB contiguous
template <bool NT>
__global__ void k_stream(const u32x4 *__restrict__ in, size_t n16, unsigned *__restrict__ out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = ld<NT>(in + i);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// (b) lane-per-frame: lane reads its 64-B frame as 4 x 16 B; optional 16-B
// write per frame; ORDER 0 = grid-stride tiles of 256 frames, 1 = each block
// walks a contiguous chunk
template <bool NT, bool WR, int ORDER>
__global__ void k_lane(const u32x4 *__restrict__ in, size_t nframes, u32x4 *__restrict__ out,
                       unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const size_t tiles = (nframes + 255) / 256;
    size_t t0, t1, dt;
    if (ORDER == 0) {
        t0 = blockIdx.x;
        t1 = tiles;
        dt = gridDim.x;
    } else {
        const size_t per = (tiles + gridDim.x - 1) / gridDim.x;
        t0 = blockIdx.x * per;
        t1 = t0 + per < tiles ? t0 + per : tiles;
        dt = 1;
    }
    for (size_t t = t0; t < t1; t += dt) {
        const size_t f = t * 256 + threadIdx.x;
        if (f >= nframes) continue;
        const u32x4 *p = in + f * 4;
        u32x4 a = ld<NT>(p), b = ld<NT>(p + 1), c = ld<NT>(p + 2), d = ld<NT>(p + 3);
        unsigned h = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
        if (WR) {
            u32x4 v = {h, a.y, b.z, c.w};
            if (NT) __builtin_nontemporal_store(v, out + f);
            else out[f] = v;
        } else {
            acc += h;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// (c) group of 4 lanes per frame: one 16-B chunk per lane (1 KiB per wave-instr)
template <bool NT, bool WR>
__global__ void k_group4(const u32x4 *__restrict__ in, size_t nframes, u32x4 *__restrict__ out,
                         unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const size_t n16 = nframes * 4;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (size_t)gridDim.x * blockDim.x) {
        u32x4 a = ld<NT>(in + i);
        unsigned h = a.x ^ a.y ^ a.z ^ a.w;
        if (WR) {
            if ((threadIdx.x & 3) == 0) {
                u32x4 v = {h, a.y, a.z, a.w};
                if (NT) __builtin_nontemporal_store(v, out + i / 4);
                else out[i / 4] = v;
            }
        } else {
            acc += h;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}


// (d) build-up: lane-per-frame with the kernel's extra steps added one at a time
//   STEP 0: frame at f*64 (no descriptor)             + 16-B plain store
//   STEP 1: descriptor indirection (off u32, len u16)  + store
//   STEP 2: 1 + one dependent 16-B probe into a 64 KiB table
//   STEP 3: 2 + LDS histogram atomic
//   STEP 4: 2 with next trip's descriptors prefetched
template <int STEP>
__global__ __launch_bounds__(256) void k_build(const u32x4 *__restrict__ in, const unsigned *__restrict__ off,
                        const unsigned short *__restrict__ len, size_t nframes,
                        const u32x4 *__restrict__ tbl, u32x4 *__restrict__ out) {
    __shared__ unsigned hist[1024];
    if (STEP == 3) {
        for (int i = threadIdx.x; i < 1024; i += 256) hist[i] = 0;
        __syncthreads();
    }
    const size_t stride = (size_t)gridDim.x * 256;
    size_t f = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned noff = 0, nlen = 64;
    if (STEP == 4 && f < nframes) {
        noff = off[f];
        nlen = len[f];
    }
    for (; f < nframes; f += stride) {
        const u32x4 *p;
        unsigned cap = 64;
        if (STEP == 0) {
            p = in + f * 4;
        } else if (STEP == 4) {
            p = in + (size_t)noff * 4;
            cap = nlen;
            const size_t g = f + stride;
            if (g < nframes) {
                noff = off[g];
                nlen = len[g];
            }
        } else {
            p = in + (size_t)off[f] * 4;
            cap = len[f];
        }
        u32x4 a = {0, 0, 0, 0}, b = a, c = a, d = a;
        if (cap > 0) a = p[0];
        if (cap > 16) b = p[1];
        if (cap > 32) c = p[2];
        if (cap > 48) d = p[3];
        unsigned h = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
        unsigned flow = h;
        if (STEP >= 2) {
            const u32x4 s = tbl[(h * 2654435761u) >> 20]; // 4096 slots x 16 B
            flow = s.w ^ s.x;
        }
        if (STEP == 3) atomicAdd(&hist[flow & 1023], 1u);
        u32x4 v = {flow, a.y, b.z, c.w};
        out[f] = v;
    }
    if (STEP == 3) {
        __syncthreads();
        if (hist[threadIdx.x] == 0x12345678u) out[0].x = 1;
    }
}

// (e) lane-per-frame through a per-wave LDS transpose: the wave's 64 frames
// (4 KiB contiguous) arrive as 4 coalesced 1-KiB loads, are written to LDS
// with a quarter swizzle (conflict-free ds_read_b128), and each lane reads its
// own frame's four quarters back
template <bool NT, bool WR>
__global__ __launch_bounds__(256) void k_lane_lds(const u32x4 *__restrict__ in, size_t nframes,
                                                  u32x4 *__restrict__ out,
                                                  unsigned *__restrict__ sink) {
    __shared__ u32x4 st[4][256];
    const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    u32x4 *my = st[wv];
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t f0 = (size_t)blockIdx.x * 256 + wv * 64; f0 + 64 <= nframes; f0 += stride) {
        const u32x4 *p = in + f0 * 4;
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ld<NT>(p + q * 64 + lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned c = q * 64 + lane, f = c >> 2;
            my[f * 4 + (((c & 3u) + (f >> 2)) & 3u)] = v[q];
        }
        __builtin_amdgcn_wave_barrier();
        const u32x4 a = my[lane * 4 + ((0 + (lane >> 2)) & 3u)];
        const u32x4 b = my[lane * 4 + ((1 + (lane >> 2)) & 3u)];
        const u32x4 c = my[lane * 4 + ((2 + (lane >> 2)) & 3u)];
        const u32x4 d = my[lane * 4 + ((3 + (lane >> 2)) & 3u)];
        __builtin_amdgcn_wave_barrier();
        const unsigned h = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
        if (WR) {
            u32x4 w = {h, a.y, b.z, c.w};
            if (NT) __builtin_nontemporal_store(w, out + f0 + lane);
            else out[f0 + lane] = w;
        } else {
            acc += h;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
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
    const size_t nframes = 16u << 20, bytes = nframes * 64;
    u32x4 *in, *out;
    unsigned *sink;
    CHK(hipMalloc(&in, bytes));
    CHK(hipMalloc(&out, nframes * 16));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(in, 1, bytes));
    int cu = 0;
    CHK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = 20;
    {
        unsigned *off;
        unsigned short *len;
        u32x4 *tbl;
        CHK(hipMalloc(&off, nframes * 4));
        CHK(hipMalloc(&len, nframes * 2));
        CHK(hipMalloc(&tbl, 4096 * 16));
        CHK(hipMemset(tbl, 3, 4096 * 16));
        unsigned *hoff = (unsigned *)malloc(nframes * 4);
        unsigned short *hlen = (unsigned short *)malloc(nframes * 2);
        for (size_t i = 0; i < nframes; ++i) {
            hoff[i] = (unsigned)i;
            hlen[i] = 64;
        }
        CHK(hipMemcpy(off, hoff, nframes * 4, hipMemcpyHostToDevice));
        CHK(hipMemcpy(len, hlen, nframes * 2, hipMemcpyHostToDevice));
        const size_t alg = nframes * (64 + 6 + 16);
        for (int bpc : {4, 8}) {
            const int g = cu * bpc;
            float ms;
            ms = timeit([&] { k_build<0><<<g, 256>>>(in, off, len, nframes, tbl, out); }, reps);
            printf("bpc=%d build0 frame+store          %.3f ms %7.0f GB/s(alg)\n", bpc, ms, alg / ms / 1e6);
            ms = timeit([&] { k_build<1><<<g, 256>>>(in, off, len, nframes, tbl, out); }, reps);
            printf("bpc=%d build1 +descriptor          %.3f ms %7.0f GB/s(alg)\n", bpc, ms, alg / ms / 1e6);
            ms = timeit([&] { k_build<2><<<g, 256>>>(in, off, len, nframes, tbl, out); }, reps);
            printf("bpc=%d build2 +probe               %.3f ms %7.0f GB/s(alg)\n", bpc, ms, alg / ms / 1e6);
            ms = timeit([&] { k_build<3><<<g, 256>>>(in, off, len, nframes, tbl, out); }, reps);
            printf("bpc=%d build3 +lds hist            %.3f ms %7.0f GB/s(alg)\n", bpc, ms, alg / ms / 1e6);
            ms = timeit([&] { k_build<4><<<g, 256>>>(in, off, len, nframes, tbl, out); }, reps);
            printf("bpc=%d build4 probe, desc prefetch %.3f ms %7.0f GB/s(alg)\n", bpc, ms, alg / ms / 1e6);
        }
    }
    for (int blocks_per_cu : {4, 6, 8}) {
        const int g = cu * blocks_per_cu;
        float ms;
        ms = timeit([&] { k_lane<false, true, 0><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane         rd+wr stride  %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_lane_lds<false, true><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane-lds     rd+wr         %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_lane_lds<true, true><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane-lds nt  rd+wr         %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_lane_lds<true, false><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane-lds nt  rd            %.3f ms %7.0f GB/s\n", blocks_per_cu, ms, bytes / ms / 1e6);
    }
    for (int blocks_per_cu : {8}) {
        const int g = cu * blocks_per_cu;
        float ms;
        ms = timeit([&] { k_stream<false><<<g, 256>>>(in, bytes / 16, sink); }, reps);
        printf("bpc=%d stream       rd            %.3f ms %7.0f GB/s\n", blocks_per_cu, ms, bytes / ms / 1e6);
        ms = timeit([&] { k_stream<true><<<g, 256>>>(in, bytes / 16, sink); }, reps);
        printf("bpc=%d stream nt    rd            %.3f ms %7.0f GB/s\n", blocks_per_cu, ms, bytes / ms / 1e6);
        ms = timeit([&] { k_lane<false, false, 0><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane         rd   stride   %.3f ms %7.0f GB/s\n", blocks_per_cu, ms, bytes / ms / 1e6);
        ms = timeit([&] { k_lane<false, false, 1><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane         rd   chunk    %.3f ms %7.0f GB/s\n", blocks_per_cu, ms, bytes / ms / 1e6);
        ms = timeit([&] { k_lane<true, true, 0><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane nt      rd+wr stride  %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_lane<false, true, 0><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane         rd+wr stride  %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_lane<false, true, 1><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d lane         rd+wr chunk   %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_group4<false, true><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d group4       rd+wr         %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
        ms = timeit([&] { k_group4<true, true><<<g, 256>>>(in, nframes, out, sink); }, reps);
        printf("bpc=%d group4 nt    rd+wr         %.3f ms %7.0f GB/s (+wr)\n", blocks_per_cu, ms, (bytes + nframes * 16) / ms / 1e6);
    }
    return 0;
}
