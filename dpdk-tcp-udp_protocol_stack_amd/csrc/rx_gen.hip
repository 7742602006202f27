// rx_gen.hip — deterministic synthetic traffic (a pktgen for the benchmarks
// and parity tests).  Frame i is a pure function of (cfg, i): the host path
// and the device kernel call the same rx_common.h code, so any subset of a
// device-generated burst can be regenerated on the CPU.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "rx_common.h"

namespace {

RX_HD uint32_t gen_one(const rxg_gen_cfg &cfg, uint64_t i, uint32_t *dst, uint32_t slot_words) {
    rx_frame_plan pl = rx_gen_plan(cfg, i);
    rx_hdr64 h;
    uint32_t hl = rx_build_header(cfg, i, pl, h);
    uint32_t nw = (pl.len + 3) / 4;
    for (uint32_t j = 0; j < nw; ++j) dst[j] = rx_frame_word(cfg, i, pl, h, hl, j);
    uint32_t pad_to = ((pl.len + 15) / 16) * 4; // zero the rest of the last 16-B granule
    if (pad_to > slot_words) pad_to = slot_words;
    for (uint32_t j = nw; j < pad_to; ++j) dst[j] = 0;
    return pl.len;
}

// frame t of the burst: written at the offset off_in[t] (packed layout) or
// at t * slot_bytes
__global__ void rx_gen_kernel(rxg_gen_cfg cfg, uint64_t first, uint32_t n, uint8_t *pkts,
                              uint32_t *off, uint16_t *len, uint32_t unit_log2,
                              const uint32_t *off_in) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint64_t base = off_in ? ((uint64_t)off_in[t] << unit_log2) : t * (uint64_t)cfg.slot_bytes;
    const uint32_t l = gen_one(cfg, first + t, reinterpret_cast<uint32_t *>(pkts + base),
                               cfg.slot_bytes / 4);
    off[t] = (uint32_t)(base >> unit_log2);
    len[t] = (uint16_t)l;
}

// packed layout offsets (units of 1 << unit_log2, each frame 64-B aligned)
static uint64_t packed_offsets(const rxg_gen_cfg &cfg, uint64_t first, uint32_t n,
                               uint32_t unit_log2, uint32_t *off) {
    uint64_t pos = 0;
    for (uint32_t t = 0; t < n; ++t) {
        off[t] = (uint32_t)(pos >> unit_log2);
        const uint32_t l = rx_gen_len(cfg, first + t);
        pos += ((uint64_t)(l < 60 ? 60 : l) + 63) & ~63ull;
    }
    return pos;
}

int check_cfg(const rxg_gen_cfg *cfg, uint32_t unit_log2) {
    if (!cfg) return RXG_EINVAL;
    if (cfg->slot_bytes == 0 || (cfg->slot_bytes & 15u)) return RXG_EINVAL;
    if (unit_log2 < 4 || unit_log2 > 16 || (cfg->slot_bytes & ((1u << unit_log2) - 1u)))
        return RXG_EINVAL;
    uint32_t maxlen = cfg->size_mode == 1 ? 1500u : cfg->frame_len;
    if (maxlen < 64 || maxlen > 65535 || maxlen > cfg->slot_bytes) return RXG_EINVAL;
    if (cfg->n_udp == 0 && cfg->n_tcp == 0) return RXG_EINVAL;
    if (cfg->n_shards > 1 && cfg->shard >= cfg->n_shards) return RXG_EINVAL;
    if (cfg->packed > 1 || (cfg->packed && unit_log2 > 6)) return RXG_EINVAL;
    if (cfg->n_udp && (uint32_t)cfg->udp_base_port + cfg->n_udp > 65536u) return RXG_EINVAL;
    if (cfg->n_udp && cfg->udp_base_port <= 7 && cfg->udp_base_port + cfg->n_udp > 7)
        return RXG_EINVAL; // :7 is the generator's "unknown flow" port
    if (cfg->n_tcp && cfg->tcp_port == 7) return RXG_EINVAL;
    return RXG_OK;
}

} // namespace

extern int rx_set_hip_error(hipError_t e);

extern "C" int rxg_gen_flows(const rxg_gen_cfg *cfg, rxg_udp_sock *u, rxg_tcb *t) {
    if (!cfg) return RXG_EINVAL;
    // UDP sockets in creation order: nsocket + nbind(local_ip, base+k)
    for (uint32_t k = 0; u && k < cfg->n_udp; ++k) {
        u[k].localip = cfg->local_ip;
        u[k].localport = (uint16_t)rx_hton16((uint32_t)cfg->udp_base_port + k);
        u[k].protocol = 17;
        u[k]._pad = 0;
    }
    // TCP: the listener is created first (nsocket/nbind/nlisten, common.c:304-386;
    // sip = sport = 0 from the memset), then one tcb per connection
    // (tcp_stream_create, tcp.c:3-41) — here already ESTABLISHED (status 4).
    if (t && cfg->n_tcp) {
        t[0].sip = 0;
        t[0].dip = cfg->local_ip;
        t[0].sport = 0;
        t[0].dport = (uint16_t)rx_hton16(cfg->tcp_port);
        t[0].status = RXG_TCP_STATUS_LISTEN;
        for (uint32_t k = 0; k < cfg->n_tcp; ++k) {
            uint32_t sip, sport;
            rx_gen_tcb(*cfg, k, &sip, &sport);
            t[k + 1].sip = sip;
            t[k + 1].dip = cfg->local_ip;
            t[k + 1].sport = (uint16_t)sport;
            t[k + 1].dport = (uint16_t)rx_hton16(cfg->tcp_port);
            t[k + 1].status = 4; // TCP_STATUS_ESTABLISHED, tcp.h:15
        }
    }
    return RXG_OK;
}

extern "C" int rxg_gen_host(const rxg_gen_cfg *cfg, uint64_t first, uint32_t n, uint8_t *pkts,
                            uint32_t *off, uint16_t *len, uint32_t off_unit_log2) {
    int rc = check_cfg(cfg, off_unit_log2);
    if (rc) return rc;
    if (n && (!pkts || !off || !len)) return RXG_EINVAL;
    if (cfg->packed) packed_offsets(*cfg, first, n, off_unit_log2, off);
    for (uint32_t t = 0; t < n; ++t) {
        const uint64_t base =
            cfg->packed ? ((uint64_t)off[t] << off_unit_log2) : (uint64_t)t * cfg->slot_bytes;
        uint32_t l = gen_one(*cfg, first + t, reinterpret_cast<uint32_t *>(pkts + base),
                             cfg->slot_bytes / 4);
        off[t] = (uint32_t)(base >> off_unit_log2);
        len[t] = (uint16_t)l;
    }
    return RXG_OK;
}

extern "C" int rxg_gen_dev(const rxg_gen_cfg *cfg, uint64_t first, uint32_t n, uint8_t *d_pkts,
                           uint32_t *d_off, uint16_t *d_len, uint32_t off_unit_log2,
                           void *stream) {
    int rc = check_cfg(cfg, off_unit_log2);
    if (rc) return rc;
    if (n == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len) return RXG_EINVAL;
    if (((uint64_t)n * cfg->slot_bytes - 1) >> off_unit_log2 > 0xFFFFFFFFull) return RXG_ERANGE;
    const uint32_t threads = 256;
    const uint32_t blocks = (n + threads - 1) / threads;
    uint32_t *d_off_in = nullptr;
    if (cfg->packed) { // offsets: host prefix sum of the (RNG-determined) frame sizes
        uint32_t *h = (uint32_t *)malloc((size_t)n * 4);
        if (!h) return RXG_ENOMEM;
        packed_offsets(*cfg, first, n, off_unit_log2, h);
        hipError_t e = hipMalloc(&d_off_in, (size_t)n * 4);
        if (e == hipSuccess) e = hipMemcpy(d_off_in, h, (size_t)n * 4, hipMemcpyHostToDevice);
        free(h);
        if (e != hipSuccess) {
            (void)hipFree(d_off_in);
            return rx_set_hip_error(e);
        }
    }
    hipLaunchKernelGGL(rx_gen_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, *cfg,
                       first, n, d_pkts, d_off, d_len, off_unit_log2, d_off_in);
    if (d_off_in) {
        hipError_t e = hipStreamSynchronize((hipStream_t)stream);
        (void)hipFree(d_off_in);
        if (e != hipSuccess) return rx_set_hip_error(e);
    }
    return rx_set_hip_error(hipGetLastError());
}
