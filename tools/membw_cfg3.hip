// membw_cfg3.hip — access-shape ceilings for the 1500-B workload (cfg3: 4M
// frames in 1536-B slots, 1504 captured bytes = 94 chunks of 16 B read per
// slot, one 16-B store per slot), with no per-frame work beyond a byte sum.
// Diagnostics only: is a shape whose
// wave-instructions read each wave's frames as contiguous 1-KiB spans faster
// than the G=8 group shape of the classify kernel?
//   stream  : plain grid-stride read of the whole buffer (the read ceiling)
//   slotg8  : G=8 lanes per slot, 12 passes in flight (the K1 shape, pipe 40)
//   waveF   : a wave owns F consecutive slots (F*1.5 KiB contiguous), each
//             lane 1.5*F 16-B loads, every load of the wave one 1-KiB
//             contiguous span; per-slot sums by a segmented wave reduce
//             (DPP / swizzle through __shfl_xor); PIPE = the next wave-tile's
//             loads issued before this one is reduced (register double buffer)
//   hipcc --offload-arch=gfx950 -O3 tools/membw_cfg3.hip -o tools/membw_cfg3
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
__device__ __forceinline__ unsigned csum(u32x4 v) { return v.x + v.y + v.z + v.w; }

__global__ __launch_bounds__(256) void k_stream(const u32x4 *__restrict__ in, size_t n16,
                                                unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        acc += csum(ldnt(in + i));
    if (acc == 0x12345678u) sink[0] = acc;
}

// the plain read with U independent 16-B loads in flight per lane (U blocks
// of the grid-stride sequence at once): does more in flight (a wider window
// of open DRAM rows) slow the plain read the way the slot shapes are slow?
template <int U>
__global__ __launch_bounds__(256) void k_stream_u(const u32x4 *__restrict__ in, size_t n16,
                                                  unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldnt(in + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += csum(v[u]);
    }
    for (; i < n16; i += stride) acc += csum(ldnt(in + i));
    if (acc == 0x12345678u) sink[0] = acc;
}

// G = 8 lanes per slot in two phases of 6 loads (half the bytes in flight)
__global__ __launch_bounds__(256) void k_slotg8_half(const u32x4 *__restrict__ in, size_t nslots,
                                                     u32x4 *__restrict__ out) {
    const unsigned gl = threadIdx.x & 7u;
    const size_t groups = (size_t)gridDim.x * 32;
    for (size_t f = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3); f < nslots; f += groups) {
        const u32x4 *p = in + f * 96;
        unsigned acc = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            u32x4 v[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const unsigned c = (h * 6 + q) * 8 + gl;
                v[q] = c < 94 ? ldnt(p + c) : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int q = 0; q < 6; ++q) acc += csum(v[q]);
        }
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (gl == 0) __builtin_nontemporal_store(u32x4{acc, (unsigned)f, 0, 0}, out + f);
    }
}

// G = 8 lanes per 1536-B slot, all 12 passes in flight (94 chunks read)
__global__ __launch_bounds__(256) void k_slotg8(const u32x4 *__restrict__ in, size_t nslots,
                                                u32x4 *__restrict__ out) {
    const unsigned gl = threadIdx.x & 7u;
    const size_t groups = (size_t)gridDim.x * 32;
    for (size_t f = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3); f < nslots; f += groups) {
        const u32x4 *p = in + f * 96;
        u32x4 v[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const unsigned c = q * 8 + gl;
            v[q] = c < 94 ? ldnt(p + c) : u32x4{0, 0, 0, 0};
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc += csum(v[q]);
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (gl == 0) __builtin_nontemporal_store(u32x4{acc, (unsigned)f, 0, 0}, out + f);
    }
}

// the decomposition: the G=8 slot shape of k_slotg8 with
// one component taken out at a time.  ST: the 16-B store per slot; RED: the
// cross-lane sum of the 8 lanes' partial sums (3 __shfl_xor); FULL: all 96
// chunks of the slot read (no masked last pass, 2 extra chunks = 2% more bytes)
template <bool ST, bool RED, bool FULL>
__global__ __launch_bounds__(256) void k_slot(const u32x4 *__restrict__ in, size_t nslots,
                                              u32x4 *__restrict__ out, unsigned *__restrict__ sink) {
    const unsigned gl = threadIdx.x & 7u;
    const size_t groups = (size_t)gridDim.x * 32;
    for (size_t f = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3); f < nslots; f += groups) {
        const u32x4 *p = in + f * 96;
        u32x4 v[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const unsigned c = q * 8 + gl;
            v[q] = (FULL || c < 94) ? ldnt(p + c) : u32x4{0, 0, 0, 0};
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc += csum(v[q]);
        if (RED) {
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            acc += __shfl_xor(acc, 4);
        }
        if (ST && gl == 0) __builtin_nontemporal_store(u32x4{acc, (unsigned)f, 0, 0}, out + f);
        else if (acc == 0x12345678u) sink[gl] = acc; // (keeps the sum live, never taken)
    }
}

// store flavours for the slot shape's verdict: 0 nt, 1 plain (write-back,
// the L2 absorbs the lines), 2 sc1 (write-through, K1's pipe 40)
template <int SM>
__device__ __forceinline__ void st16(u32x4 *p, u32x4 w) {
    if constexpr (SM == 0) __builtin_nontemporal_store(w, p);
    else if constexpr (SM == 1) *p = w;
    else asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 0" ::"v"(p), "v"(w) : "memory");
}

// the slot shape with the verdict store in flavour SM
template <int SM>
__global__ __launch_bounds__(256) void k_slot_sm(const u32x4 *__restrict__ in, size_t nslots,
                                                 u32x4 *__restrict__ out) {
    const unsigned gl = threadIdx.x & 7u;
    const size_t groups = (size_t)gridDim.x * 32;
    for (size_t f = (size_t)blockIdx.x * 32 + (threadIdx.x >> 3); f < nslots; f += groups) {
        const u32x4 *p = in + f * 96;
        u32x4 v[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const unsigned c = q * 8 + gl;
            v[q] = c < 94 ? ldnt(p + c) : u32x4{0, 0, 0, 0};
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc += csum(v[q]);
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (gl == 0) st16<SM>(out + f, u32x4{acc, (unsigned)f, 0, 0});
    }
}

// a wave owns runs of 64 consecutive slots (8 trips of 8 slots, G=8 as
// above); WIDE: the 64 verdicts are gathered into lane i (lane 8t+g takes
// group g's sum at trip t over ds_bpermute) and leave as ONE 1-KiB store per
// run; else each trip's 8 verdicts leave as one 128-B store (same mapping)
template <int SM, bool WIDE>
__global__ __launch_bounds__(256) void k_slotrun(const u32x4 *__restrict__ in, size_t nslots,
                                                 u32x4 *__restrict__ out) {
    const unsigned lane = threadIdx.x & 63u, gl = lane & 7u, g = lane >> 3;
    const size_t nw = (size_t)gridDim.x * 4, nruns = nslots / 64;
    for (size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < nruns; r += nw) {
        unsigned keep = 0;
#pragma unroll 1
        for (unsigned t = 0; t < 8; ++t) {
            const size_t f = r * 64 + t * 8 + g;
            const u32x4 *p = in + f * 96;
            u32x4 v[12];
#pragma unroll
            for (int q = 0; q < 12; ++q) {
                const unsigned c = q * 8 + gl;
                v[q] = c < 94 ? ldnt(p + c) : u32x4{0, 0, 0, 0};
            }
            unsigned acc = 0;
#pragma unroll
            for (int q = 0; q < 12; ++q) acc += csum(v[q]);
            acc += __shfl_xor(acc, 1);
            acc += __shfl_xor(acc, 2);
            acc += __shfl_xor(acc, 4);
            if (WIDE) {
                const unsigned x = __shfl(acc, (int)((lane & 7u) * 8u)); // group (lane & 7)'s sum
                keep = (lane >> 3) == t ? x : keep;
            } else if (gl == 0) {
                st16<SM>(out + f, u32x4{acc, (unsigned)f, 0, 0});
            }
        }
        if (WIDE) st16<SM>(out + r * 64 + lane, u32x4{keep, (unsigned)(r * 64 + lane), 0, 0});
    }
}

// time-batched verdict writes: a block owns a contiguous range of slots
// (CONTIG) or strided 32-slot tiles, keeps the verdicts of T consecutive trips
// in LDS and writes them out together (T * 512 B; T = 1: every trip).  If the
// cost of the sparse verdict stream is in the memory controller's read/write
// turnarounds, writes bunched in time across the chip should cost less
template <int T, int SM, bool CONTIG>
__global__ __launch_bounds__(256) void k_slotbuf(const u32x4 *__restrict__ in, size_t nslots,
                                                 u32x4 *__restrict__ out) {
    __shared__ u32x4 buf[T * 32];
    const unsigned gl = threadIdx.x & 7u, grp = threadIdx.x >> 3;
    const size_t ntiles = nslots / 32;
    const size_t per = (ntiles + gridDim.x - 1) / gridDim.x; // CONTIG: tiles per block
    const size_t t0 = CONTIG ? blockIdx.x * per : blockIdx.x;
    const size_t t1 = CONTIG ? (t0 + per < ntiles ? t0 + per : ntiles) : ntiles;
    const size_t tstep = CONTIG ? 1 : gridDim.x;
    unsigned k = 0;
    size_t first = t0; // first tile of the batch in LDS (CONTIG)
    for (size_t t = t0; t < t1; t += tstep) {
        const size_t f = t * 32 + grp;
        const u32x4 *p = in + f * 96;
        u32x4 v[12];
#pragma unroll
        for (int q = 0; q < 12; ++q) {
            const unsigned c = q * 8 + gl;
            v[q] = c < 94 ? ldnt(p + c) : u32x4{0, 0, 0, 0};
        }
        unsigned acc = 0;
#pragma unroll
        for (int q = 0; q < 12; ++q) acc += csum(v[q]);
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        acc += __shfl_xor(acc, 4);
        if (T == 1) {
            if (gl == 0) st16<SM>(out + f, u32x4{acc, (unsigned)f, 0, 0});
            continue;
        }
        if (gl == 0) buf[k * 32 + grp] = u32x4{acc, (unsigned)f, 0, 0};
        if (++k == T || t + tstep >= t1) {
            __syncthreads();
            const unsigned m = k * 32; // verdicts in the batch
            for (unsigned i = threadIdx.x; i < m; i += 256) {
                // CONTIG: one contiguous run; else tile i/32 of the batch is t - (k-1-i/32) * tstep
                const size_t tt = CONTIG ? first + i / 32 : t - (size_t)(k - 1 - i / 32) * tstep;
                st16<SM>(out + tt * 32 + (i & 31u), buf[i]);
            }
            __syncthreads();
            k = 0;
            first = t + tstep;
        }
    }
}

// the jumbo shape (cfg5: 1.25M 9000-B frames in 9024-B slots; the stream
// kernel reads a block's 16 frames as one contiguous span, 1 KiB per wave
// instruction, and writes their 16 verdicts at the block's end): one block
// per 16-slot span, U loads per thread in flight; ST: 16 verdict stores (nt)
// by threads 0..15 after the span; a non-resident grid as the stream kernel's
template <bool ST, int U>
__global__ __launch_bounds__(256) void k_span(const u32x4 *__restrict__ in, size_t nslots, size_t slot16,
                                              u32x4 *__restrict__ out, unsigned *__restrict__ sink) {
    __shared__ unsigned part[4];
    const size_t s0 = (size_t)blockIdx.x * 16;
    const size_t c0 = s0 * slot16, c1 = (s0 + 16 < nslots ? s0 + 16 : nslots) * slot16;
    unsigned acc = 0;
    size_t c = c0 + threadIdx.x;
    for (; c + (U - 1) * 256 < c1; c += U * 256) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldnt(in + c + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += csum(v[u]);
    }
    for (; c < c1; c += 256) acc += csum(ldnt(in + c));
    for (int o = 1; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    const unsigned tot = part[0] + part[1] + part[2] + part[3];
    if (ST) {
        if (threadIdx.x < 16 && s0 + threadIdx.x < nslots)
            __builtin_nontemporal_store(u32x4{tot, (unsigned)(s0 + threadIdx.x), 0, 0}, out + s0 + threadIdx.x);
    } else if (tot == 0x12345678u) {
        sink[0] = tot;
    }
}

// the plain grid-stride read plus one 16-B non-temporal store per 96 chunks
// (per 1536-B slot), issued by the lane that reads the slot's first chunk
__global__ __launch_bounds__(256) void k_stream_st(const u32x4 *__restrict__ in, size_t n16,
                                                   u32x4 *__restrict__ out, unsigned *__restrict__ sink) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    // slot q and chunk r of index i, advanced incrementally (no division per trip)
    size_t q = i / 96;
    unsigned r = (unsigned)(i % 96);
    const size_t qs = stride / 96;
    const unsigned rs = (unsigned)(stride % 96);
    for (; i < n16; i += stride) {
        acc += csum(ldnt(in + i));
        if (r == 0) __builtin_nontemporal_store(u32x4{acc, (unsigned)q, 0, 0}, out + q);
        q += qs;
        r += rs;
        if (r >= 96) { r -= 96; ++q; }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// a wave owns F consecutive slots per trip (F even: 1.5 * F loads per lane);
// load j of lane l reads chunk 64 j + l of the wave-tile, which belongs to
// slot (64 j + l) / 96; chunks 94, 95 of each slot are padding (not counted)
template <int F, bool PIPE>
__global__ __launch_bounds__(256) void k_wave(const u32x4 *__restrict__ in, size_t nslots,
                                              u32x4 *__restrict__ out) {
    constexpr int NL = F * 96 / 64;
    const unsigned lane = threadIdx.x & 63u;
    const size_t nw = (size_t)gridDim.x * 4;
    const size_t ntiles = nslots / F; // (the buffer holds whole wave-tiles)
    size_t t = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    u32x4 v[NL], nv[NL];
    auto load = [&](u32x4 *dst, size_t tile) {
        const u32x4 *p = in + (tile < ntiles ? tile : 0) * (F * 96);
#pragma unroll
        for (int j = 0; j < NL; ++j) dst[j] = ldnt(p + 64 * j + lane);
    };
    if (t < ntiles) load(v, t);
    for (; t < ntiles; t += nw) {
        if (PIPE) load(nv, t + nw);
        unsigned s[F];
#pragma unroll
        for (int k = 0; k < F; ++k) s[k] = 0;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const unsigned c = 64 * j + lane; // chunk in the tile
#pragma unroll
            for (int k = 0; k < F; ++k) {
                // compile-time: which slots load j can touch
                if (64 * j + 63 >= 96 * k && 64 * j < 96 * k + 96) {
                    const unsigned r = c - 96u * k;
                    s[k] += (r < 94u) ? csum(v[j]) : 0u;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < F; ++k) {
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) s[k] += __shfl_xor(s[k], o);
        }
        if (lane < (unsigned)F) {
            unsigned a = s[0];
#pragma unroll
            for (int k = 1; k < F; ++k) a = lane == (unsigned)k ? s[k] : a;
            __builtin_nontemporal_store(u32x4{a, (unsigned)(t * F + lane), 0, 0}, out + t * F + lane);
        }
        if (PIPE) {
#pragma unroll
            for (int j = 0; j < NL; ++j) v[j] = nv[j];
        } else if (t + nw < ntiles) {
            load(v, t + nw);
        }
    }
}

template <typename K>
float timeit(K f, int reps) {
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
    const double alg = (double)nslots * (1500 + 22);
    u32x4 *in, *out;
    unsigned *sink;
    const size_t inbytes = bytes > (size_t)1250000 * 9024 ? bytes : (size_t)1250000 * 9024;
    CHK(hipMalloc(&in, inbytes));
    CHK(hipMalloc(&out, nslots * 16));
    CHK(hipMalloc(&sink, 64));
    CHK(hipMemset(in, 1, inbytes));
    int cu = 0;
    CHK(hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0));
    const int reps = 20;
    // (the in-flight sweep of r06b: profiles/r06b/membw_cfg3_r06b.txt)
    // cfg5's span shape with and without its verdict stores (r06)
    {
        const size_t nj = 1250000, slot16 = 9024 / 16;
        if (nj * slot16 * 16 <= inbytes) {
            const double jb = (double)nj * 9024;
            for (int round = 0; round < 3; ++round) {
                float ms;
#define J(name, launch)                                                                            \
    ms = timeit([&] { launch; }, reps);                                                            \
    printf("j%d %-24s %.4f ms %7.0f GB/s (read)\n", round, name, ms, jb / ms / 1e6);
                J("span U=4 no store", (k_span<false, 4><<<(nj + 15) / 16, 256>>>(in, nj, slot16, out, sink)))
                J("span U=4 + 16 verdicts", (k_span<true, 4><<<(nj + 15) / 16, 256>>>(in, nj, slot16, out, sink)))
                J("span U=8 no store", (k_span<false, 8><<<(nj + 15) / 16, 256>>>(in, nj, slot16, out, sink)))
                J("span U=8 + 16 verdicts", (k_span<true, 8><<<(nj + 15) / 16, 256>>>(in, nj, slot16, out, sink)))
#undef J
            }
        }
    }
    // the decomposition, interleaved, 3 rounds: which component of the slot
    // shape costs the 0.912 -> 1.042 ms
    for (int round = 0; round < 3; ++round) {
        for (int bpc : {4, 8}) {
            const int g = cu * bpc;
            float ms;
#define D(name, launch, B)                                                                         \
    ms = timeit([&] { launch; }, reps);                                                            \
    printf("d%d bpc=%d %-26s %.4f ms %7.0f GB/s (read)\n", round, bpc, name, ms, (B) / ms / 1e6);
            D("stream", (k_stream<<<g, 256>>>(in, bytes / 16, sink)), (double)bytes)
            D("stream+store", (k_stream_st<<<g, 256>>>(in, bytes / 16, out, sink)), (double)bytes)
            D("slot st red", (k_slot<true, true, false><<<g, 256>>>(in, nslots, out, sink)), nslots * 1504.0)
            D("slot nost red", (k_slot<false, true, false><<<g, 256>>>(in, nslots, out, sink)), nslots * 1504.0)
            D("slot st nored", (k_slot<true, false, false><<<g, 256>>>(in, nslots, out, sink)), nslots * 1504.0)
            D("slot nost nored", (k_slot<false, false, false><<<g, 256>>>(in, nslots, out, sink)), nslots * 1504.0)
            D("slot st red full96", (k_slot<true, true, true><<<g, 256>>>(in, nslots, out, sink)), (double)bytes)
            D("slot nost nored full96", (k_slot<false, false, true><<<g, 256>>>(in, nslots, out, sink)), (double)bytes)
            D("slot st plain", (k_slot_sm<1><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("slot st sc1", (k_slot_sm<2><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("run64 st nt 128B/trip", (k_slotrun<0, false><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("run64 st nt 1KiB/run", (k_slotrun<0, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("run64 st plain 1KiB/run", (k_slotrun<1, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("run64 st sc1 1KiB/run", (k_slotrun<2, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf strided T1 sc1", (k_slotbuf<1, 2, false><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf strided T8 sc1", (k_slotbuf<8, 2, false><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf strided T32 sc1", (k_slotbuf<32, 2, false><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf contig T1 sc1", (k_slotbuf<1, 2, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf contig T8 sc1", (k_slotbuf<8, 2, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf contig T32 sc1", (k_slotbuf<32, 2, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf contig T32 nt", (k_slotbuf<32, 0, true><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
            D("buf strided T32 nt", (k_slotbuf<32, 0, false><<<g, 256>>>(in, nslots, out)), nslots * 1504.0)
#undef D
        }
    }
    // (the wave-contiguous shapes: profiles/r05c, r06c)
    return 0;
}
