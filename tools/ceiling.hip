// ceiling.hip — the box's measured HBM read ceiling, for bench.py's line
// (hbm_read_ceiling_gbs).  Diagnostics only, not part of the product: a plain
// coalesced grid-stride read (16 B per lane per load, non-temporal, one load
// in flight per lane: the shape that reads fastest in tools/membw_large.hip,
// 7.07-7.25 TB/s, profiles/r03b, r03d) at 4 and 8 blocks of 256 per CU; the
// best of the two is returned.  Built by tools/Makefile into libceiling.so.
#include <hip/hip_runtime.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void ceiling_read_kernel(const u32x4 *__restrict__ in,
                                                           size_t n16, unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = __builtin_nontemporal_load(in + i);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc; // keeps the loads; never true for the fill
}

// the slot shape of the 1500-B classify (K1 group kernel, G = 8 lanes per
// slot): each group of 8 lanes reads the first nch 16-B chunks of its slot,
// all of a lane's (at most 12) loads in flight, then an 8-lane reduce and
// one 16-B store per slot — the kernel's reads and writes with no parsing
__global__ __launch_bounds__(256) void ceiling_slot_kernel(const u32x4 *__restrict__ in,
                                                           size_t nslots, unsigned slot16,
                                                           unsigned nch, u32x4 *__restrict__ out) {
    const unsigned gl = threadIdx.x & 7u;
    const size_t groups = (size_t)gridDim.x * 32;
    for (size_t f = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3); f < nslots; f += groups) {
        const u32x4 *p = in + f * slot16;
        u32x4 v[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const unsigned c = q * 8 + gl;
            v[q] = c < nch ? __builtin_nontemporal_load(p + c) : u32x4{0, 0, 0, 0};
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc += v[q].x + v[q].y + v[q].z + v[q].w;
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (gl == 0) __builtin_nontemporal_store(u32x4{acc, (unsigned)f, 0, 0}, out + f);
    }
}

// one wave spinning for `ticks` of the constant-rate wall clock
// (s_memrealtime), counting the shader clock (s_memtime) meanwhile
__global__ void clock_probe_kernel(unsigned long long ticks, unsigned long long *out) {
    const unsigned long long w0 = wall_clock64(), c0 = clock64();
    unsigned long long w1 = w0, c1 = c0;
    while (w1 - w0 < ticks) {
        __builtin_amdgcn_s_sleep(2);
        w1 = wall_clock64();
        c1 = clock64();
    }
    if (threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = w1 - w0;
    }
}

extern "C" {

// the shader clock while the probe runs: launch on `stream` (a HIP stream
// handle, or null), spinning for `ms`; *state is a device buffer of 2 u64
// (allocated here when *state is null); read the result with clock_probe_read
int clock_probe_launch(int device, void *stream, double ms, void **state) {
    int rate_khz = 0;
    hipError_t e = hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device);
    if (e != hipSuccess) return (int)e;
    if (!*state && (e = hipMalloc(state, 16)) != hipSuccess) return (int)e;
    const unsigned long long ticks = (unsigned long long)(ms * rate_khz);
    clock_probe_kernel<<<1, 64, 0, (hipStream_t)stream>>>(ticks, (unsigned long long *)*state);
    return (int)hipGetLastError();
}

// after the probe's stream is synchronized: shader-clock MHz (s_memtime
// ticks per wall microsecond)
int clock_probe_read(int device, void *state, double *mhz) {
    int rate_khz = 0;
    unsigned long long h[2] = {0, 0};
    hipError_t e = hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device);
    if (e == hipSuccess) e = hipMemcpy(h, state, 16, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return (int)e;
    *mhz = h[1] ? (double)h[0] / ((double)h[1] / (rate_khz * 1e-3)) : 0.0;
    return 0;
}

static float median(float *t, int n) {
    for (int i = 1; i < n; ++i)
        for (int j = i; j > 0 && t[j] < t[j - 1]; --j) {
            const float x = t[j];
            t[j] = t[j - 1];
            t[j - 1] = x;
        }
    return t[n / 2];
}

// Over a caller's burst in HBM (`buf`, nslots slots of slot_bytes, frames at
// each slot's start, read_bytes captured per frame): *slot_ms = the slot-shape
// read (ceiling_slot_kernel, read_bytes rounded up to 16-B chunks, 16 B
// stored per slot into a scratch buffer), *stream_ms = a plain read of the
// same nslots * slot_bytes; each the median of `reps` launches, best of 4 and
// 8 blocks per CU.  The same bytes, in the same allocation and process as the
// classify launch they bound.  0, or the HIP error (hipErrorInvalidValue: slot
// not a multiple of 16, or more than 96 chunks read).
int ceiling_slot_ms(int device, const void *buf, unsigned long long nslots, unsigned slot_bytes,
                    unsigned read_bytes, int reps, double *slot_ms, double *stream_ms) {
    if (slot_bytes % 16 || read_bytes > slot_bytes || (read_bytes + 15) / 16 > 96 || !nslots)
        return (int)hipErrorInvalidValue;
    int old = 0;
    hipGetDevice(&old);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return (int)e;
    u32x4 *out = nullptr;
    unsigned *sink = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s = nullptr;
    int cu = 0;
    double best_slot = 1e30, best_stream = 1e30;
    const unsigned nch = (read_bytes + 15) / 16;
    const size_t n16 = (size_t)nslots * (slot_bytes / 16);
    if (reps < 1) reps = 1;
    if (reps > 64) reps = 64;
    float t[64];
    if ((e = hipMalloc(&out, nslots * 16)) != hipSuccess) goto out;
    if ((e = hipMalloc(&sink, 64)) != hipSuccess) goto out;
    if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) goto out;
    if ((e = hipEventCreate(&a)) != hipSuccess) goto out;
    if ((e = hipEventCreate(&b)) != hipSuccess) goto out;
    if ((e = hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device)) !=
        hipSuccess)
        goto out;
    for (int kind = 0; kind < 2; ++kind)
        for (int bpc : {4, 8}) {
            const int grid = cu * bpc;
            auto launch = [&] {
                if (kind == 0)
                    ceiling_slot_kernel<<<grid, 256, 0, s>>>((const u32x4 *)buf, nslots,
                                                             slot_bytes / 16, nch, out);
                else
                    ceiling_read_kernel<<<grid, 256, 0, s>>>((const u32x4 *)buf, n16, sink);
            };
            for (int w = 0; w < 3; ++w) launch();
            for (int r = 0; r < reps; ++r) {
                hipEventRecord(a, s);
                launch();
                hipEventRecord(b, s);
                if ((e = hipEventSynchronize(b)) != hipSuccess) goto out;
                hipEventElapsedTime(&t[r], a, b);
            }
            const double m = median(t, reps);
            double &best = kind == 0 ? best_slot : best_stream;
            if (m < best) best = m;
        }
    *slot_ms = best_slot;
    *stream_ms = best_stream;
out:
    if (a) hipEventDestroy(a);
    if (b) hipEventDestroy(b);
    if (s) hipStreamDestroy(s);
    if (sink) hipFree(sink);
    if (out) hipFree(out);
    hipSetDevice(old);
    return (int)e;
}

// read rate of `nbytes` of HBM on `device` in GB/s (1e9 B/s), median of
// `reps` timed passes per grid, best grid; 0 on success, else the HIP error
int ceiling_read_gbs(int device, unsigned long long nbytes, int reps, double *gbs) {
    int old = 0;
    hipGetDevice(&old);
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return (int)e;
    u32x4 *in = nullptr;
    unsigned *sink = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s = nullptr;
    int cu = 0;
    double best = 0.0;
    const size_t n16 = nbytes / 16;
    if (reps < 1) reps = 1;
    if (reps > 64) reps = 64;
    float t[64];
    if ((e = hipMalloc(&in, n16 * 16)) != hipSuccess) goto out;
    if ((e = hipMalloc(&sink, 64)) != hipSuccess) goto out;
    if ((e = hipMemset(in, 0x5a, n16 * 16)) != hipSuccess) goto out;
    if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) goto out;
    if ((e = hipEventCreate(&a)) != hipSuccess) goto out;
    if ((e = hipEventCreate(&b)) != hipSuccess) goto out;
    if ((e = hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device)) !=
        hipSuccess)
        goto out;
    for (int bpc : {4, 8}) {
        const int grid = cu * bpc;
        for (int w = 0; w < 3; ++w) ceiling_read_kernel<<<grid, 256, 0, s>>>(in, n16, sink);
        for (int r = 0; r < reps; ++r) {
            hipEventRecord(a, s);
            ceiling_read_kernel<<<grid, 256, 0, s>>>(in, n16, sink);
            hipEventRecord(b, s);
            if ((e = hipEventSynchronize(b)) != hipSuccess) goto out;
            hipEventElapsedTime(&t[r], a, b);
        }
        const double g = (double)(n16 * 16) / (median(t, reps) * 1e-3) / 1e9;
        if (g > best) best = g;
    }
    *gbs = best;
out:
    if (a) hipEventDestroy(a);
    if (b) hipEventDestroy(b);
    if (s) hipStreamDestroy(s);
    if (sink) hipFree(sink);
    if (in) hipFree(in);
    hipSetDevice(old);
    return (int)e;
}
}
