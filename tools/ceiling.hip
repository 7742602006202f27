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
        for (int i = 1; i < reps; ++i) // insertion sort: median
            for (int j = i; j > 0 && t[j] < t[j - 1]; --j) {
                const float x = t[j];
                t[j] = t[j - 1];
                t[j - 1] = x;
            }
        const double g = (double)(n16 * 16) / (t[reps / 2] * 1e-3) / 1e9;
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
