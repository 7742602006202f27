// rx_device.h — gfx950 device helpers shared by the classify (rx_classify.hip)
// and TX checksum (tx_cksum.hip) kernels: lane-group broadcast / reduction
// over DPP and ds_swizzle, the dot2 word-sum, byte masks at a frame's end, and
// 16-B streaming loads / stores.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

// ---- intra-group broadcast / reduction (group = G aligned lanes) ----------
// A cross-lane result is pinned by an empty asm: under register pressure the
// compiler may otherwise REMATERIALISE the DPP / ds_swizzle inside a later
// divergent region (e.g. the group's lane-0 verdict store), where the source
// lanes are inactive and the read returns 0 — observed on gfx950 / ROCm 7.2
// as UDP dgram_len read as 0 by the (8,1,2) variant at the 8-wave register cap.
__device__ __forceinline__ uint32_t pin(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

template <int G, int K>
__device__ __forceinline__ uint32_t gbcast(uint32_t x) {
    static_assert(K < G, "lane out of group");
    if constexpr (G == 4) {
        return pin(__builtin_amdgcn_update_dpp(0u, x, K * 0x55, 0xF, 0xF, false)); // quad_perm [K,K,K,K]
    } else if constexpr (G <= 32) {
        // ds_swizzle bitmask mode: lane' = (lane & and) | or, within 32 lanes
        return pin((uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (0x1F & ~(G - 1)) | (K << 5)));
    } else {
        return __builtin_amdgcn_readlane(x, K);
    }
}

template <int G>
__device__ __forceinline__ uint32_t gsum(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
    x += __builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += __builtin_amdgcn_update_dpp(0u, x, 0x141, 0xF, 0xF, false); // row_half_mirror
    if constexpr (G >= 16) x += __builtin_amdgcn_update_dpp(0u, x, 0x140, 0xF, 0xF, false); // row_mirror
    if constexpr (G >= 32) x += (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (0x10 << 10)); // xor 16
    if constexpr (G == 64) x = __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 32);
    return pin(x);
}

typedef unsigned short rx_us2 __attribute__((ext_vector_type(2)));

// acc + x.lo + x.hi in one v_dot2_u32_u16
__device__ __forceinline__ uint32_t add_halves(uint32_t acc, uint32_t x) {
    const rx_us2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(rx_us2, x), one, acc, false);
}

// keep only the bytes of dword x (at frame offset pos) that lie below `end`
__device__ __forceinline__ uint32_t keep_below(uint32_t x, int32_t pos, int32_t end) {
    int32_t k = end - pos;
    k = k < 0 ? 0 : (k > 4 ? 4 : k);
    return k == 4 ? x : (x & ((1u << (8 * k)) - 1u));
}

__device__ __forceinline__ uint4 chunk_below(uint4 c, int32_t s, int32_t end) {
    c.x = keep_below(c.x, s + 0, end);
    c.y = keep_below(c.y, s + 4, end);
    c.z = keep_below(c.z, s + 8, end);
    c.w = keep_below(c.w, s + 12, end);
    return c;
}

typedef unsigned int rx_u32x4 __attribute__((ext_vector_type(4)));

// streaming 16-B load / store.  nt (non-temporal) pays for coalesced 1-KiB
// wave accesses and costs for 16-B-per-lane strided ones (tools/membw.hip), so
// the policy is a template choice of each kernel.
template <bool NT = true>
__device__ __forceinline__ uint4 ldg16(const uint8_t *p) {
    if constexpr (NT) {
        const rx_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const rx_u32x4 *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else {
        return *reinterpret_cast<const uint4 *>(p);
    }
}
// one 16-B flow-table slot in a single dwordx4 load (a uint4 member-wise load
// lets the compiler split off .w, test it, then load .xyz: two round trips)
__device__ __forceinline__ uint4 ld_slot(const uint4 *p) {
    const rx_u32x4 v = *reinterpret_cast<const rx_u32x4 *>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// LDS byte address of a __shared__ object
__device__ __forceinline__ uint32_t rx_lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char *)p);
}
// LDS-DMA (global_load_lds_dwordx4): each active lane loads the 16 B at src
// (16-B aligned) into LDS at lds + 16 * lane; lds is wave-uniform.  No VGPR
// is written.  The compiler does not count it: its data is read only after an
// s_waitcnt vmcnt the caller places (by the issuing wave; other waves also
// need a barrier after that wait).  The lgkmcnt(0) retires the wave's pending
// LDS reads first, so none of them can see the DMA's bytes.  M0 is set and
// restored inside the statement (the compiler owns it).
__device__ __forceinline__ void rx_dma16(const void *src, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_waitcnt lgkmcnt(0)\n\t"
                 "s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %2\n\t"
                 "s_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds)
                 : "memory");
}

// the streamed 16-B outputs (verdicts, count indices).  RX_ST_POLICY 0: nt
// stores, which KEEP the written line in the XCD's L2; 1: sc1 (write-through)
// stores, which drop it (MI355X_MICROARCH.md, store flavours), so hundreds of
// MB of verdicts per burst do not evict the flow tables the probes read
#ifndef RX_ST_POLICY
#define RX_ST_POLICY 0
#endif
__device__ __forceinline__ void st_stream16(rx_u32x4 *p, rx_u32x4 w) {
#if RX_ST_POLICY == 1
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 0" ::"v"(p), "v"(w) : "memory");
#else
    __builtin_nontemporal_store(w, p);
#endif
}

// a write-through 16-B store (sc1) whatever RX_ST_POLICY says.  The s_nop is
// the one wait state a store of more than 8 bytes needs before a VALU may
// overwrite its data registers: the compiler inserts it after its own stores,
// but cannot see inside inline asm
__device__ __forceinline__ void stg16_wt(uint4 *p, uint4 v) {
    const rx_u32x4 w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 0" ::"v"(p), "v"(w) : "memory");
}

__device__ __forceinline__ void stg16(uint4 *p, uint4 v) {
    const rx_u32x4 w = {v.x, v.y, v.z, v.w};
    st_stream16(reinterpret_cast<rx_u32x4 *>(p), w);
}

// The first 64 B of a wave's 64 frames that sit in consecutive 64-B slots
// starting at b, one frame per lane, read as four coalesced 1-KiB loads (lane
// l holds chunk q*64 + l = quarter l%4 of frame 16q + l/4), written to the
// wave's 4-KiB LDS stage st with the quarter index rotated by (frame>>2)&3 so
// that the read-back (lane f reads its frame's four quarters, ds_read_b128) is
// bank-conflict free.  The caller checks that the 4 KiB lie in the buffer.
__device__ __forceinline__ void stage64_load(const uint8_t *b, uint4 *st, uint32_t lane,
                                             uint4 (&c)[4]) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = ldg16<true>(b + 16u * (q * 64u + lane));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t k = q * 64u + lane, f = k >> 2;
        st[f * 4u + (((k & 3u) + (f >> 2)) & 3u)] = v[q];
    }
    __builtin_amdgcn_wave_barrier(); // LDS ops of one wave run in order; keep the compiler's too
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = st[lane * 4u + ((k + (lane >> 2)) & 3u)];
    __builtin_amdgcn_wave_barrier();
}

// Frame heads at arbitrary positions, gathered four lanes per head: lane l
// loads chunk (l & 3) of the head of the wave's frame 16q + (l >> 2), q = 0..3
// (its position and caplen fetched from the owning lane with ds_bpermute), so
// one load instruction touches 16 heads instead of 64 (one 16-B piece per
// lane, 64 distinct 64-B segments).  Chunks at or past a frame's caplen load
// its chunk 0 (valid memory) and are masked by the consumer.
__device__ __forceinline__ void head_gather_issue(const uint8_t *pkts, uint64_t fpos, int32_t cp,
                                                  uint32_t lane, uint4 (&v)[4]) {
    const int lo = (int)(uint32_t)fpos, hi = (int)(uint32_t)(fpos >> 32);
    const uint32_t k = lane & 3u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int src = (int)((16u * q + (lane >> 2)) << 2);
        const uint64_t f = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(src, hi) << 32) |
                           (uint32_t)__builtin_amdgcn_ds_bpermute(src, lo);
        const int32_t fc = __builtin_amdgcn_ds_bpermute(src, cp);
        v[q] = ldg16<false>(pkts + f + (16 * (int32_t)k < fc ? 16u * k : 0u));
    }
}

// head_gather_issue's chunks into each lane's own four (the stage64_load
// layout through the wave's 4-KiB LDS stage st)
__device__ __forceinline__ void head_gather_stage(uint4 *st, uint32_t lane, const uint4 (&v)[4],
                                                  uint4 (&c)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t kk = q * 64u + lane, f = kk >> 2;
        st[f * 4u + (((kk & 3u) + (f >> 2)) & 3u)] = v[q];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = st[lane * 4u + ((k + (lane >> 2)) & 3u)];
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
    s = (s >> 16) + (s & 0xFFFFu);
    s = (s >> 16) + (s & 0xFFFFu);
    return s;
}

} // namespace
