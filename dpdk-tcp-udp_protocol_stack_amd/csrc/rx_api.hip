// rx_api.hip — host side of librxgpu: context, flow-table build/upload, the
// burst entry points of include/rxgpu.h.  Device work is in rx_classify.hip;
// there is no CPU classification path in this library: every verdict comes
// from the gfx950 kernel, and a missing/failed device is an error.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <vector>

#include "rx_common.h"

void rx_pick_variant(uint32_t len_hint, uint32_t *g, uint32_t *p, uint32_t *fpg, uint32_t *pipe);
void rx_set_bpc_cap(uint32_t cap);
hipError_t rx_classify_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                              uint32_t n, uint32_t unit_log2, uint32_t g, uint32_t p, uint32_t fpg,
                              uint32_t pipe, const rx_ft_dev &ft, uint4 *out,
                              unsigned long long *counts, hipStream_t s, uint32_t *ws);
size_t rx_classify_ws_bytes(uint32_t n, uint32_t g, uint32_t pipe, const rx_ft_dev &ft,
                            bool counts);

static thread_local std::string g_last_hip;

int rx_set_hip_error(hipError_t e) {
    if (e == hipSuccess) return RXG_OK;
    g_last_hip = std::string(hipGetErrorName(e)) + ": " + hipGetErrorString(e);
    return RXG_EHIP;
}

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) return rx_set_hip_error(e_);                                         \
    } while (0)

// ---------------------------------------------------------------------------
// Host flow-table image (see rx_common.h for the device layout)
struct ft_host {
    std::vector<uint4> slots;
    uint32_t mask = 0, probe = 1;

    // entries: x,y,z = key, w = value, in creation order (newest wins)
    void build(const std::vector<uint4> &entries) {
        const uint64_t n = entries.size();
        uint64_t ns = 16;
        while (ns < 4 * n) ns <<= 1; // load factor <= 1/4: always an empty slot
        slots.assign(ns, make_uint4(0, 0, 0, RX_SLOT_EMPTY));
        mask = (uint32_t)(ns - 1);
        probe = 1;
        for (const uint4 &e : entries) {
            uint32_t i = rx_hash3(e.x, e.y, e.z) & mask;
            for (uint32_t d = 0;; ++d, i = (i + 1) & mask) {
                uint4 &sl = slots[i];
                if (sl.w == RX_SLOT_EMPTY) {
                    sl = e;
                } else if (sl.x == e.x && sl.y == e.y && sl.z == e.z) {
                    sl.w = e.w; // a newer control block with the same key wins
                } else {
                    continue;
                }
                probe = std::max(probe, d + 1);
                break;
            }
        }
    }

    uint32_t lookup(uint32_t a, uint32_t b, uint32_t c) const {
        uint32_t i = rx_hash3(a, b, c) & mask;
        for (uint32_t d = 0; d < probe; ++d, i = (i + 1) & mask) {
            const uint4 &sl = slots[i];
            if (sl.w == RX_SLOT_EMPTY) break;
            if (sl.x == a && sl.y == b && sl.z == c) return sl.w;
        }
        return RXG_FLOW_NONE;
    }
};

// Compact UDP table for socket sets of <= RX_UDPC_MAX_FLOWS: the same keys and
// flow ids as the main table (already deduplicated, newest wins), 8-B slots at
// load <= 1/2 so the lane kernel can keep it in LDS.
static void build_udpc(const ft_host &u, uint32_t nu, std::vector<uint2> *out, uint32_t *probe) {
    out->clear();
    *probe = 0;
    if (nu == 0 || nu > RX_UDPC_MAX_FLOWS) return;
    uint32_t ns = 16;
    while (ns < 2 * nu) ns <<= 1;
    out->assign(ns, make_uint2(0, 0xFFFFFFFFu));
    const uint32_t mask = ns - 1;
    for (const uint4 &sl : u.slots) {
        if (sl.w == RX_SLOT_EMPTY) continue; // key (dip, dport, 17) -> flow
        uint32_t i = rx_hash3(sl.x, sl.y, sl.z) & mask;
        uint32_t d = 0;
        while ((*out)[i].y != 0xFFFFFFFFu) i = (i + 1) & mask, ++d;
        (*out)[i] = make_uint2(sl.x, (sl.y & 0xFFFFu) | (sl.w << 16));
        *probe = std::max(*probe, d + 1);
    }
}

struct rxg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // flow tables
    ft_host h_udp, h_tcp;
    std::vector<uint32_t> h_listen;
    std::vector<uint2> h_udpc; // compact UDP table (small socket sets), empty if none
    uint32_t udpc_probe = 0;
    uint4 *d_udp = nullptr, *d_tcp = nullptr;
    uint2 *d_udpc = nullptr;
    size_t d_udp_cap = 0, d_tcp_cap = 0, d_udpc_cap = 0;
    uint32_t *d_listen = nullptr;
    rx_ft_dev ft{};
    uint32_t tune_g = 0, tune_p = 0, tune_fpg = 0, tune_pipe = ~0u; // rxg_tune override
    uint32_t tune_bpc = 0; // rxg_tune_grid: resident blocks per CU cap (0 = occupancy)
    uint32_t *d_ws = nullptr; // launch workspace (binned lists, count slabs), grown on demand
    size_t d_ws_cap = 0;
    // context-owned per-flow counts (host-buffer path)
    unsigned long long *d_counts = nullptr;
    uint32_t counts_cap = 0;
    // staging for the host-buffer path
    uint32_t max_pkts = 0;
    uint64_t max_bytes = 0;
    uint8_t *h_stage = nullptr; // pinned, mbuf gather
    uint32_t *h_off = nullptr;
    uint16_t *h_len = nullptr;
    uint8_t *d_pkts = nullptr;
    uint32_t *d_off = nullptr;
    uint16_t *d_len = nullptr;
    uint4 *d_out = nullptr;
};

static int ensure_dev(void **p, size_t *cap, size_t bytes) {
    if (*cap >= bytes && *p) return RXG_OK;
    if (*p) HIPCHK(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipMalloc(p, bytes));
    *cap = bytes;
    return RXG_OK;
}

extern "C" {

const char *rxg_strerror(int err) {
    switch (err) {
    case RXG_OK:
        return "ok";
    case RXG_EINVAL:
        return "invalid argument";
    case RXG_ENOMEM:
        return "out of memory";
    case RXG_ENODEV:
        return "no HIP device";
    case RXG_ERANGE:
        return "burst exceeds the context's staging capacity or 32-bit offsets";
    case RXG_EHIP:
        return "HIP runtime error (see rxg_last_hip_error)";
    default:
        return "unknown error";
    }
}

const char *rxg_last_hip_error(void) { return g_last_hip.c_str(); }

int rxg_open(rxg_ctx **out, int device, uint32_t max_pkts, uint64_t max_bytes) {
    if (!out) return RXG_EINVAL;
    *out = nullptr;
    rxg_ctx *c;
    int rc = RXG_OK;
    if (device == RXG_HOST_ONLY) { // control-plane context: flow tables + host lookups only
        c = new (std::nothrow) rxg_ctx();
        if (!c) return RXG_ENOMEM;
        c->device = RXG_HOST_ONLY;
        rc = rxg_flows_sync(c, nullptr, 0, nullptr, 0);
        if (rc != RXG_OK) {
            rxg_close(c);
            return rc;
        }
        *out = c;
        return RXG_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RXG_ENODEV;
    if (device < 0 || device >= ndev) return RXG_ENODEV;
    c = new (std::nothrow) rxg_ctx();
    if (!c) return RXG_ENOMEM;
    c->device = device;
    do {
        if ((rc = rx_set_hip_error(hipSetDevice(device)))) break;
        if ((rc = rx_set_hip_error(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking))))
            break;
        if ((rc = rx_set_hip_error(hipMalloc(&c->d_listen, 65536 * sizeof(uint32_t))))) break;
        c->max_pkts = max_pkts;
        c->max_bytes = (max_bytes + 15) & ~15ull;
        if (max_pkts && c->max_bytes) {
            if ((rc = rx_set_hip_error(hipHostMalloc((void **)&c->h_stage, c->max_bytes, 0)))) break;
            if ((rc = rx_set_hip_error(hipHostMalloc((void **)&c->h_off, max_pkts * 4ull, 0)))) break;
            if ((rc = rx_set_hip_error(hipHostMalloc((void **)&c->h_len, max_pkts * 2ull, 0)))) break;
            if ((rc = rx_set_hip_error(hipMalloc(&c->d_pkts, c->max_bytes)))) break;
            if ((rc = rx_set_hip_error(hipMalloc(&c->d_off, max_pkts * 4ull)))) break;
            if ((rc = rx_set_hip_error(hipMalloc(&c->d_len, max_pkts * 2ull)))) break;
            if ((rc = rx_set_hip_error(hipMalloc(&c->d_out, max_pkts * 16ull)))) break;
        }
    } while (0);
    if (rc == RXG_OK) rc = rxg_flows_sync(c, nullptr, 0, nullptr, 0);
    if (rc != RXG_OK) {
        rxg_close(c);
        return rc;
    }
    *out = c;
    return RXG_OK;
}

void rxg_close(rxg_ctx *c) {
    if (!c) return;
    if (c->device == RXG_HOST_ONLY) {
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->d_udp);
    (void)hipFree(c->d_tcp);
    (void)hipFree(c->d_listen);
    (void)hipFree(c->d_counts);
    (void)hipFree(c->d_ws);
    (void)hipFree(c->d_udpc);
    (void)hipFree(c->d_pkts);
    (void)hipFree(c->d_off);
    (void)hipFree(c->d_len);
    (void)hipFree(c->d_out);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_off) (void)hipHostFree(c->h_off);
    if (c->h_len) (void)hipHostFree(c->h_len);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int rxg_flows_sync(rxg_ctx *c, const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t, uint32_t nt) {
    if (!c || (nu && !u) || (nt && !t)) return RXG_EINVAL;
    // UDP: get_hostinfo_fromip_port matches (dip, dport, proto); every socket
    // the reference creates has protocol 17 (nsocket, common.c:281), and the
    // lookup is only ever called with 17 (udp.c:14), so others never match.
    std::vector<uint4> ue;
    ue.reserve(nu);
    for (uint32_t i = 0; i < nu; ++i)
        if (u[i].protocol == 17) ue.push_back(make_uint4(u[i].localip, u[i].localport, 17u, i));
    std::vector<uint4> te;
    te.reserve(nt);
    for (uint32_t i = 0; i < nt; ++i)
        te.push_back(make_uint4(t[i].sip, t[i].dip,
                                (uint32_t)t[i].sport | ((uint32_t)t[i].dport << 16), i));
    c->h_udp.build(ue);
    c->h_tcp.build(te);
    build_udpc(c->h_udp, nu, &c->h_udpc, &c->udpc_probe);
    c->h_listen.assign(65536, RXG_FLOW_NONE);
    for (uint32_t i = 0; i < nt; ++i)
        if (t[i].status == RXG_TCP_STATUS_LISTEN) c->h_listen[t[i].dport] = i;
    c->ft.nu = nu;
    c->ft.nt = nt;
    if (c->device == RXG_HOST_ONLY) return RXG_OK;
    HIPCHK(hipSetDevice(c->device));

    // control-plane operation: wait for in-flight bursts before replacing tables
    HIPCHK(hipDeviceSynchronize());
    int rc;
    if ((rc = ensure_dev((void **)&c->d_udp, &c->d_udp_cap, c->h_udp.slots.size() * sizeof(uint4))))
        return rc;
    if ((rc = ensure_dev((void **)&c->d_tcp, &c->d_tcp_cap, c->h_tcp.slots.size() * sizeof(uint4))))
        return rc;
    HIPCHK(hipMemcpy(c->d_udp, c->h_udp.slots.data(), c->h_udp.slots.size() * sizeof(uint4),
                     hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_tcp, c->h_tcp.slots.data(), c->h_tcp.slots.size() * sizeof(uint4),
                     hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(c->d_listen, c->h_listen.data(), 65536 * sizeof(uint32_t),
                     hipMemcpyHostToDevice));
    c->ft.udpc = nullptr;
    c->ft.udpc_mask = c->ft.udpc_probe = 0;
    if (!c->h_udpc.empty()) {
        if ((rc = ensure_dev((void **)&c->d_udpc, &c->d_udpc_cap, c->h_udpc.size() * sizeof(uint2))))
            return rc;
        HIPCHK(hipMemcpy(c->d_udpc, c->h_udpc.data(), c->h_udpc.size() * sizeof(uint2),
                         hipMemcpyHostToDevice));
        c->ft.udpc = c->d_udpc;
        c->ft.udpc_mask = (uint32_t)c->h_udpc.size() - 1;
        c->ft.udpc_probe = c->udpc_probe;
    }
    c->ft.udp = c->d_udp;
    c->ft.tcp = c->d_tcp;
    c->ft.listen = c->d_listen;
    c->ft.udp_mask = c->h_udp.mask;
    c->ft.tcp_mask = c->h_tcp.mask;
    c->ft.udp_probe = c->h_udp.probe;
    c->ft.tcp_probe = c->h_tcp.probe;
    // context counts follow the flow set
    const uint32_t nf = nu + nt;
    if (c->counts_cap < nf || !c->d_counts) {
        (void)hipFree(c->d_counts);
        c->d_counts = nullptr;
        c->counts_cap = 0;
        HIPCHK(hipMalloc(&c->d_counts, (size_t)std::max(nf, 1u) * 8));
        c->counts_cap = std::max(nf, 1u);
    }
    HIPCHK(hipMemset(c->d_counts, 0, (size_t)c->counts_cap * 8));
    return RXG_OK;
}

int rxg_tune(rxg_ctx *c, uint32_t lanes_per_frame, uint32_t passes, uint32_t frames_per_group,
             uint32_t pipeline) {
    if (!c) return RXG_EINVAL;
    if (lanes_per_frame == 0 && (pipeline == 20 || pipeline == 30 || pipeline == 31 || pipeline == 130)) {
        c->tune_g = 0; // size-class binned path (20) / stream kernel (30, 31)
        c->tune_p = c->tune_fpg = 0;
        c->tune_pipe = pipeline;
        return RXG_OK;
    }
    if (lanes_per_frame && (lanes_per_frame == 2 || lanes_per_frame > 64 ||
                            (lanes_per_frame & (lanes_per_frame - 1))))
        return RXG_EINVAL;
    c->tune_g = lanes_per_frame;
    c->tune_p = lanes_per_frame ? passes : 0;
    c->tune_fpg = lanes_per_frame ? frames_per_group : 0;
    c->tune_pipe = lanes_per_frame ? pipeline : ~0u;
    return RXG_OK;
}

int rxg_tune_grid(rxg_ctx *c, uint32_t blocks_per_cu) {
    if (!c || blocks_per_cu > 32) return RXG_EINVAL;
    c->tune_bpc = blocks_per_cu;
    return RXG_OK;
}

uint32_t rxg_num_flows(const rxg_ctx *c) { return c ? c->ft.nu + c->ft.nt : 0; }

uint32_t rxg_ft_lookup_udp(const rxg_ctx *c, uint32_t dip, uint16_t dport) {
    return c ? c->h_udp.lookup(dip, dport, 17u) : RXG_FLOW_NONE;
}

uint32_t rxg_ft_lookup_tcp(const rxg_ctx *c, uint32_t sip, uint32_t dip, uint16_t sport,
                           uint16_t dport) {
    if (!c) return RXG_FLOW_NONE;
    uint32_t f = c->h_tcp.lookup(sip, dip, (uint32_t)sport | ((uint32_t)dport << 16));
    if (f == RXG_FLOW_NONE && !c->h_listen.empty()) f = c->h_listen[dport];
    return f;
}

uint32_t rxg_rss_hash(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport) {
    return rx_rss_hash(sip, dip, sport, dport);
}

int rxg_classify_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                     const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t len_hint,
                     rxg_verdict *d_out, uint64_t *d_counts, void *stream) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len || !d_out) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    uint32_t g = c->tune_g, p = c->tune_p, fpg = c->tune_fpg, pipe = c->tune_pipe;
    if (!g && pipe == ~0u) rx_pick_variant(len_hint, &g, &p, &fpg, &pipe);
    // workspace (binned lists, count slabs): grown on demand, so size it once
    // per burst shape before any graph capture
    if (size_t ws = rx_classify_ws_bytes(n, g, pipe, c->ft, d_counts != nullptr)) {
        int rc = ensure_dev((void **)&c->d_ws, &c->d_ws_cap, ws);
        if (rc) return rc;
    }
    rx_set_bpc_cap(c->tune_bpc);
    HIPCHK(rx_classify_launch(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft, reinterpret_cast<uint4 *>(d_out),
                              reinterpret_cast<unsigned long long *>(d_counts),
                              (hipStream_t)stream, c->d_ws));
    return RXG_OK;
}

int rxg_classify_span(rxg_ctx *c, const uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
                      const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!pkts || !off || !len || !out) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    if (n > c->max_pkts || !c->d_pkts) return RXG_ERANGE;
    const uint64_t span = (span_bytes + 15) & ~15ull;
    if (span > c->max_bytes) return RXG_ERANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->d_pkts, pkts, span, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_off, off, n * 4ull, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_len, len, n * 2ull, hipMemcpyHostToDevice, c->stream));
    uint32_t g = c->tune_g, p = c->tune_p, fpg = c->tune_fpg, pipe = c->tune_pipe;
    if (!g && pipe == ~0u) rx_pick_variant((uint32_t)(span / n), &g, &p, &fpg, &pipe);
    if (size_t ws = rx_classify_ws_bytes(n, g, pipe, c->ft, c->d_counts != nullptr)) {
        int rc = ensure_dev((void **)&c->d_ws, &c->d_ws_cap, ws);
        if (rc) return rc;
    }
    rx_set_bpc_cap(c->tune_bpc);
    HIPCHK(rx_classify_launch(c->d_pkts, c->d_off, c->d_len, n, off_unit_log2, g, p, fpg, pipe,
                              c->ft, c->d_out, c->d_counts, c->stream, c->d_ws));
    HIPCHK(hipMemcpyAsync(out, c->d_out, n * 16ull, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RXG_OK;
}

int rxg_classify(rxg_ctx *c, const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                 uint32_t n, uint32_t off_unit_log2, rxg_verdict *out) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!pkts || !off || !len || !out) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    uint64_t span = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t e = ((uint64_t)off[i] << off_unit_log2) + len[i];
        span = std::max(span, e);
    }
    return rxg_classify_span(c, pkts, span, off, len, n, off_unit_log2, out);
}

int rxg_process_mbufs(rxg_ctx *c, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!m || !out) return RXG_EINVAL;
    if (n > c->max_pkts || !c->h_stage) return RXG_ERANGE;
    // gather frames (buf_addr + data_off, data_len bytes) at 64-B aligned slots
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!m[i] || !m[i]->buf_addr) return RXG_EINVAL;
        const uint32_t l = m[i]->data_len;
        const uint64_t slot = (l + 63ull) & ~63ull;
        if (pos + std::max<uint64_t>(slot, 64) > c->max_bytes) return RXG_ERANGE;
        memcpy(c->h_stage + pos, (const uint8_t *)m[i]->buf_addr + m[i]->data_off, l);
        if (slot > l) memset(c->h_stage + pos + l, 0, slot - l);
        c->h_off[i] = (uint32_t)(pos >> 6);
        c->h_len[i] = (uint16_t)l;
        pos += std::max<uint64_t>(slot, 64);
    }
    return rxg_classify(c, c->h_stage, c->h_off, c->h_len, n, 6, out);
}

int rxg_flow_counts(rxg_ctx *c, uint64_t *counts, uint32_t ncounts) {
    if (!c || (ncounts && !counts)) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    const uint32_t nf = c->ft.nu + c->ft.nt;
    if (ncounts < nf) return RXG_ERANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (nf) HIPCHK(hipMemcpy(counts, c->d_counts, nf * 8ull, hipMemcpyDeviceToHost));
    return RXG_OK;
}

int rxg_counts_reset(rxg_ctx *c) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemset(c->d_counts, 0, (size_t)c->counts_cap * 8));
    return RXG_OK;
}

} // extern "C"
