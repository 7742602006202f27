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
    for (int blocks_per_cu : {2, 4, 8}) {
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
