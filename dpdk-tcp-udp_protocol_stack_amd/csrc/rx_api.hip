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
#include <unordered_map>
#include <vector>

#include "rx_common.h"

void rx_pick_variant(uint32_t len_hint, uint32_t *g, uint32_t *p, uint32_t *fpg, uint32_t *pipe);
void rx_set_bpc_cap(uint32_t cap);
bool rx_variant_exists(uint32_t g, uint32_t pipe);
hipError_t rx_classify_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                              uint32_t n, uint32_t unit_log2, uint32_t g, uint32_t p, uint32_t fpg,
                              uint32_t pipe, const rx_ft_dev &ft, uint4 *out,
                              unsigned long long *counts, hipStream_t s, uint32_t *ws,
                              uint32_t phase, uint32_t buf, uint32_t nbuf);
size_t rx_classify_ws_bytes(uint32_t n, uint32_t g, uint32_t pipe, const rx_ft_dev &ft,
                            bool counts, uint32_t nbuf);
bool rx_count_uses_slabs(const rx_ft_dev &ft, bool counts);
hipError_t tx_cksum_launch(uint8_t *pkts, const uint32_t *off, const uint16_t *len, uint32_t n,
                           uint32_t unit_log2, uint32_t len_hint, uint32_t variant,
                           uint32_t bpc_cap, hipStream_t s);
uint32_t tx_num_variants();
size_t rx_split_ws_bytes(uint32_t n, uint32_t nsh);
hipError_t rx_split_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                           uint32_t n, uint32_t unit_log2, uint32_t nsh, uint32_t *first,
                           uint32_t *perm, void *ws, hipStream_t s);
size_t rx_gather_ws_bytes(uint32_t count);
hipError_t rx_gather_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                            uint32_t unit_log2, const uint32_t *idx, uint32_t count, uint8_t *dst,
                            uint64_t cap, uint32_t *dst_off, uint16_t *dst_len, void *ws,
                            hipStream_t s);
int rx_group_allreduce_u64(rxg_group *g, void *d, uint32_t n, hipStream_t s);

static thread_local std::string g_last_hip;

int rx_set_hip_error(hipError_t e) {
    if (e == hipSuccess) return RXG_OK;
    g_last_hip = std::string(hipGetErrorName(e)) + ": " + hipGetErrorString(e);
    return RXG_EHIP;
}

void rx_set_last_error(const std::string &msg) { g_last_hip = msg; }

hipError_t rx_occupancy(const void *fn, uint32_t threads, size_t lds, int *cu, int *occ) {
    struct entry {
        int dev;
        const void *fn;
        uint32_t threads;
        size_t lds;
        int cu, occ;
    };
    static thread_local std::vector<entry> cache;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    for (const entry &x : cache)
        if (x.dev == dev && x.fn == fn && x.threads == threads && x.lds == lds) {
            *cu = x.cu;
            *occ = x.occ;
            return hipSuccess;
        }
    entry x{dev, fn, threads, lds, 0, 0};
    if ((e = hipDeviceGetAttribute(&x.cu, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
        return e;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&x.occ, fn, (int)threads, lds)) !=
        hipSuccess)
        return e;
    if (x.occ < 1) x.occ = 1;
    cache.push_back(x);
    *cu = x.cu;
    *occ = x.occ;
    return hipSuccess;
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

    // entries: x,y,z = key, w = value, in creation order (newest wins); load
    // factor <= 2^-load_log2 (>= 1: always an empty slot)
    void build(const std::vector<uint4> &entries, uint32_t load_log2) {
        const uint64_t n = entries.size();
        uint64_t ns = 16;
        while (ns < (n << load_log2)) ns <<= 1;
        // RX_FT_MIRROR slots past the end mirror slots 0.., so a probe window of
        // up to RX_FT_MIRROR + 1 slots at any index reads in bounds (the stream
        // kernels' first probe)
        slots.assign(ns + RX_FT_MIRROR, make_uint4(0, 0, 0, RX_SLOT_EMPTY));
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
        for (uint32_t k = 0; k < RX_FT_MIRROR; ++k) slots[ns + k] = slots[k];
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
    for (uint32_t j = 0; j <= u.mask; ++j) { // (past the mask: mirrors)
        const uint4 &sl = u.slots[j];
        if (sl.w == RX_SLOT_EMPTY) continue; // key (dip, dport, 17) -> flow
        uint32_t i = rx_hash3(sl.x, sl.y, sl.z) & mask;
        uint32_t d = 0;
        while ((*out)[i].y != 0xFFFFFFFFu) i = (i + 1) & mask, ++d;
        (*out)[i] = make_uint2(sl.x, (sl.y & 0xFFFFu) | (sl.w << 16));
        *probe = std::max(*probe, d + 1);
    }
}

// UDP direct port table (rx_common.h): the address most sockets are bound to
// gets a u32[65536] entry per port (flow id, or RX_PORT_NONE); a port that also
// has a socket on another address is flagged RX_PORT_HASHED, and lookups for
// those other addresses probe the hashed table, which holds every key.
static uint32_t build_udp_port(const ft_host &u, std::vector<uint32_t> *port) {
    std::unordered_map<uint32_t, uint32_t> dips; // dip -> sockets bound to it
    for (uint32_t i = 0; i <= u.mask; ++i)
        if (u.slots[i].w != RX_SLOT_EMPTY) ++dips[u.slots[i].x];
    uint32_t dip = 0, best = 0;
    for (const auto &d : dips)
        if (d.second > best || (d.second == best && d.first < dip)) best = d.second, dip = d.first;
    port->assign(65536, RX_PORT_NONE);
    for (uint32_t i = 0; i <= u.mask; ++i) { // (past the mask: mirrors)
        const uint4 &sl = u.slots[i];
        if (sl.w == RX_SLOT_EMPTY) continue; // key (dip, dport, 17) -> newest flow
        uint32_t &e = (*port)[sl.y & 0xFFFFu];
        if (sl.x == dip)
            e = (e & RX_PORT_HASHED) | sl.w;
        else
            e |= RX_PORT_HASHED;
    }
    return dip;
}

// UDP port window (rx_common.h): the host-order port range of the sockets
// bound to udp_dip, when it spans <= RX_UDPW_MAX_PORTS ports and the compact
// table exists; u16 flow ids, 0xFFFF = no socket on (udp_dip, port).  Empty
// otherwise.  *lo = its first port.
static void build_udpw(const std::vector<uint32_t> &port, bool compact, std::vector<uint16_t> *w,
                       uint32_t *lo) {
    w->clear();
    *lo = 0;
    if (!compact || port.empty()) return;
    uint32_t mn = 65536, mx = 0;
    for (uint32_t r = 0; r < 65536; ++r)
        if ((port[r] & RX_PORT_NONE) != RX_PORT_NONE) {
            const uint32_t h = ((r & 0xFFu) << 8) | (r >> 8);
            mn = std::min(mn, h);
            mx = std::max(mx, h);
        }
    if (mn > mx || mx - mn + 1 > RX_UDPW_MAX_PORTS) return;
    w->assign(mx - mn + 1, 0xFFFFu);
    for (uint32_t h = mn; h <= mx; ++h) {
        const uint32_t f = port[((h & 0xFFu) << 8) | (h >> 8)] & RX_PORT_NONE;
        if (f != RX_PORT_NONE) (*w)[h - mn] = (uint16_t)f; // < RX_UDPC_MAX_FLOWS
    }
    *lo = mn;
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
    std::vector<uint32_t> h_udp_port; // UDP direct port table (empty: not built)
    uint32_t udp_dip = 0;
    uint32_t *d_udp_port = nullptr;
    std::vector<uint16_t> h_udpw; // UDP port window (empty: not built)
    uint32_t udpw_lo = 0;
    uint16_t *d_udpw = nullptr;
    size_t d_udpw_cap = 0;
    uint32_t tune_tables = 0; // rxg_tune_tables flags
    rx_ft_dev ft{};
    uint32_t tune_g = 0, tune_p = 0, tune_fpg = 0, tune_pipe = ~0u; // rxg_tune override
    uint32_t tune_bpc = 0; // rxg_tune_grid: resident blocks per CU cap (0 = occupancy)
    uint32_t tune_tx = RXG_TX_AUTO, tune_tx_bpc = 0; // rxg_tune_tx
    uint32_t ft_load_log2 = RX_FT_LOAD_LOG2;           // rxg_tune_flow_load
    // launch workspace, grown on demand: [binned lists][count indices x 2][count
    // slabs].  Three regions are tracked, each by the event of its last use and
    // that use's stream: index buffer 0 (with the lists), index buffer 1, the
    // slabs.  A launch that uses a region on another stream than its last use
    // waits for that event first, so bursts on different streams never share a
    // region in flight, and rxg_classify_dev_cs can classify burst k+1 into one
    // index buffer while burst k is counted from the other on the count stream.
    uint32_t *d_ws = nullptr;
    size_t d_ws_cap = 0;
    struct ws_use {
        hipEvent_t ev = nullptr;
        hipStream_t st = nullptr;
        bool used = false;
    } wu[3];
    // region offsets depend on the burst shape (frame count, binned path, size);
    // a change of shape waits on every region
    struct ws_shape {
        uint32_t n = 0;
        bool lists = false;
        size_t bytes = 0;
        bool operator!=(const ws_shape &o) const { return n != o.n || lists != o.lists || bytes != o.bytes; }
    } ws_layout;
    uint32_t ws_flip = 0; // index buffer of the next split-stream burst
    hipEvent_t ev_k1 = nullptr; // split-stream burst: classify done (count stream waits on it)
    void *d_aux = nullptr; // RSS split / gather workspace, grown on demand
    size_t d_aux_cap = 0;
    // context-owned per-flow counts (host-buffer path)
    unsigned long long *d_counts = nullptr;
    uint32_t counts_cap = 0;
    // host-buffer path: a ring of RXG_PIPE_DEPTH staging slots; burst t uses
    // slot t % depth.  Copies in run on s_h2d, kernels on `stream`, verdict
    // copies out on s_d2h, chained by events, so burst t+1's frames cross PCIe
    // while burst t is classified and burst t-1's verdicts come back.
    uint32_t max_pkts = 0;
    uint64_t max_bytes = 0;
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    struct slot {
        uint8_t *h_stage = nullptr; // pinned, mbuf gather
        uint32_t *h_off = nullptr;
        uint16_t *h_len = nullptr;
        uint8_t *d_pkts = nullptr;
        uint32_t *d_off = nullptr;
        uint16_t *d_len = nullptr;
        uint4 *d_out = nullptr;
        hipEvent_t ev_in = nullptr;   // inputs copied (h_stage reusable, kernel may start)
        hipEvent_t ev_k = nullptr;    // kernel done (d_pkts/d_off/d_len reusable)
        hipEvent_t ev_done = nullptr; // verdicts in host memory (d_out reusable)
        uint64_t ticket = 0;          // last burst submitted to this slot (0 = none)
    } slots[RXG_PIPE_DEPTH];
    uint64_t next_ticket = 1;
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
    case RXG_ECOMM:
        return "RCCL error (see rxg_last_hip_error)";
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
        for (rxg_ctx::ws_use &u : c->wu)
            if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&u.ev, hipEventDisableTiming))))
                break;
        if (rc) break;
        if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&c->ev_k1, hipEventDisableTiming))))
            break;
        c->max_pkts = max_pkts;
        c->max_bytes = (max_bytes + 15) & ~15ull;
        if (max_pkts && c->max_bytes) {
            if ((rc = rx_set_hip_error(hipStreamCreateWithFlags(&c->s_h2d, hipStreamNonBlocking))))
                break;
            if ((rc = rx_set_hip_error(hipStreamCreateWithFlags(&c->s_d2h, hipStreamNonBlocking))))
                break;
            for (rxg_ctx::slot &sl : c->slots) {
                if ((rc = rx_set_hip_error(hipHostMalloc((void **)&sl.h_stage, c->max_bytes, 0)))) break;
                if ((rc = rx_set_hip_error(hipHostMalloc((void **)&sl.h_off, max_pkts * 4ull, 0)))) break;
                if ((rc = rx_set_hip_error(hipHostMalloc((void **)&sl.h_len, max_pkts * 2ull, 0)))) break;
                if ((rc = rx_set_hip_error(hipMalloc(&sl.d_pkts, c->max_bytes)))) break;
                if ((rc = rx_set_hip_error(hipMalloc(&sl.d_off, max_pkts * 4ull)))) break;
                if ((rc = rx_set_hip_error(hipMalloc(&sl.d_len, max_pkts * 2ull)))) break;
                if ((rc = rx_set_hip_error(hipMalloc(&sl.d_out, max_pkts * 16ull)))) break;
                const unsigned fl = hipEventDisableTiming;
                if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&sl.ev_in, fl)))) break;
                if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&sl.ev_k, fl)))) break;
                if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&sl.ev_done, fl)))) break;
            }
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
    if (c->s_h2d) (void)hipStreamSynchronize(c->s_h2d);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->s_d2h) (void)hipStreamSynchronize(c->s_d2h);
    (void)hipFree(c->d_udp);
    (void)hipFree(c->d_tcp);
    (void)hipFree(c->d_listen);
    (void)hipFree(c->d_udp_port);
    (void)hipFree(c->d_counts);
    (void)hipFree(c->d_ws);
    (void)hipFree(c->d_aux);
    (void)hipFree(c->d_udpc);
    (void)hipFree(c->d_udpw);
    for (rxg_ctx::ws_use &u : c->wu)
        if (u.ev) (void)hipEventDestroy(u.ev);
    if (c->ev_k1) (void)hipEventDestroy(c->ev_k1);
    for (rxg_ctx::slot &sl : c->slots) {
        (void)hipFree(sl.d_pkts);
        (void)hipFree(sl.d_off);
        (void)hipFree(sl.d_len);
        (void)hipFree(sl.d_out);
        if (sl.h_stage) (void)hipHostFree(sl.h_stage);
        if (sl.h_off) (void)hipHostFree(sl.h_off);
        if (sl.h_len) (void)hipHostFree(sl.h_len);
        if (sl.ev_in) (void)hipEventDestroy(sl.ev_in);
        if (sl.ev_k) (void)hipEventDestroy(sl.ev_k);
        if (sl.ev_done) (void)hipEventDestroy(sl.ev_done);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->s_h2d) (void)hipStreamDestroy(c->s_h2d);
    if (c->s_d2h) (void)hipStreamDestroy(c->s_d2h);
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
    c->h_udp.build(ue, c->ft_load_log2);
    c->h_tcp.build(te, c->ft_load_log2);
    build_udpc(c->h_udp, nu, &c->h_udpc, &c->udpc_probe);
    c->h_udp_port.clear();
    if (!ue.empty() && !(c->tune_tables & RXG_TT_NO_UDP_PORT))
        c->udp_dip = build_udp_port(c->h_udp, &c->h_udp_port);
    build_udpw(c->h_udp_port, !c->h_udpc.empty(), &c->h_udpw, &c->udpw_lo);
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
    c->ft.udp_port = nullptr;
    if (!c->h_udp_port.empty()) {
        if (!c->d_udp_port) HIPCHK(hipMalloc(&c->d_udp_port, 65536 * sizeof(uint32_t)));
        HIPCHK(hipMemcpy(c->d_udp_port, c->h_udp_port.data(), 65536 * sizeof(uint32_t),
                         hipMemcpyHostToDevice));
        c->ft.udp_port = c->d_udp_port;
        c->ft.udp_dip = c->udp_dip;
    }
    c->ft.udpw = nullptr;
    c->ft.udpw_lo = c->ft.udpw_n = 0;
    if (!c->h_udpw.empty()) {
        if ((rc = ensure_dev((void **)&c->d_udpw, &c->d_udpw_cap, c->h_udpw.size() * sizeof(uint16_t))))
            return rc;
        HIPCHK(hipMemcpy(c->d_udpw, c->h_udpw.data(), c->h_udpw.size() * sizeof(uint16_t),
                         hipMemcpyHostToDevice));
        c->ft.udpw = c->d_udpw;
        c->ft.udpw_lo = c->udpw_lo;
        c->ft.udpw_n = (uint32_t)c->h_udpw.size();
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
    if (lanes_per_frame == 0 && pipeline != ~0u) {
        // size-class binned path (20) / stream kernel variants: anything else
        // would silently run the automatic choice (r02o measured "ablations"
        // that were the default kernel), so it is refused
        if (pipeline != 20 && !rx_variant_exists(0, pipeline)) return RXG_EINVAL;
        c->tune_g = 0;
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

int rxg_tune_tx(rxg_ctx *c, uint32_t variant, uint32_t blocks_per_cu) {
    if (!c || blocks_per_cu > 32 || (variant != RXG_TX_AUTO && variant >= tx_num_variants()))
        return RXG_EINVAL;
    c->tune_tx = variant;
    c->tune_tx_bpc = blocks_per_cu;
    return RXG_OK;
}

int rxg_tune_tables(rxg_ctx *c, uint32_t flags) {
    if (!c || (flags & ~(uint32_t)(RXG_TT_NO_UDP_PORT | RXG_TT_COUNT_4B))) return RXG_EINVAL;
    c->tune_tables = flags;
    c->ft.count_4b = (flags & RXG_TT_COUNT_4B) ? 1u : 0u;
    return RXG_OK;
}

int rxg_tune_flow_load(rxg_ctx *c, uint32_t load_log2) {
    if (!c || load_log2 > 4) return RXG_EINVAL;
    c->ft_load_log2 = load_log2 ? load_log2 : RX_FT_LOAD_LOG2;
    return RXG_OK;
}

uint32_t rxg_num_flows(const rxg_ctx *c) { return c ? c->ft.nu + c->ft.nt : 0; }

uint32_t rxg_ft_lookup_udp(const rxg_ctx *c, uint32_t dip, uint16_t dport) {
    if (!c) return RXG_FLOW_NONE;
    uint32_t f;
    if (!c->h_udp_port.empty() && rx_udp_port_decide(c->h_udp_port[dport], dip, c->udp_dip, &f))
        return f;
    return c->h_udp.lookup(dip, dport, 17u);
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

// workspace regions (rxg_ctx::wu)
enum { WS_BUF0 = 0, WS_BUF1 = 1, WS_SLAB = 2 };

static hipError_t ws_wait(rxg_ctx *c, int r, hipStream_t s) {
    const rxg_ctx::ws_use &u = c->wu[r];
    return (u.used && u.st != s) ? hipStreamWaitEvent(s, u.ev, 0) : hipSuccess;
}

static hipError_t ws_mark(rxg_ctx *c, int r, hipStream_t s) {
    rxg_ctx::ws_use &u = c->wu[r];
    hipError_t e = hipEventRecord(u.ev, s);
    if (e == hipSuccess) u.st = s, u.used = true;
    return e;
}

// size the workspace for a burst before its launches (growth drains every use
// of the old one) and, when the burst shape moves the regions, order stream s
// after every earlier use
static int ws_prepare(rxg_ctx *c, size_t ws, const rxg_ctx::ws_shape &layout, hipStream_t s) {
    if (ws > c->d_ws_cap) {
        for (rxg_ctx::ws_use &u : c->wu)
            if (u.used) HIPCHK(hipEventSynchronize(u.ev));
        int rc = ensure_dev((void **)&c->d_ws, &c->d_ws_cap, ws);
        if (rc) return rc;
    } else if (layout != c->ws_layout) {
        for (int r = 0; r < 3; ++r) HIPCHK(ws_wait(c, r, s));
    }
    c->ws_layout = layout;
    return RXG_OK;
}

// one burst on the workspace: classify + count on s (count_stream null or s),
// or classify on s and the slab count on count_stream (double-buffered indices)
static int classify_ws(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                       const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t g,
                       uint32_t p, uint32_t fpg, uint32_t pipe, uint4 *d_out,
                       unsigned long long *d_counts, hipStream_t s, hipStream_t cs) {
    const size_t ws = rx_classify_ws_bytes(n, g, pipe, c->ft, d_counts != nullptr, 2);
    const bool split = cs && cs != s && pipe != 20 && rx_count_uses_slabs(c->ft, d_counts != nullptr);
    // counts the classify kernel adds itself (few flows), or the binned path's:
    // the count stream is ordered after this burst's kernels, as promised
    auto join_cs = [&]() -> int {
        if (cs && cs != s && d_counts) {
            HIPCHK(hipEventRecord(c->ev_k1, s));
            HIPCHK(hipStreamWaitEvent(cs, c->ev_k1, 0));
        }
        return RXG_OK;
    };
    rx_set_bpc_cap(c->tune_bpc);
    if (!ws) {
        HIPCHK(rx_classify_launch(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                                  d_out, d_counts, s, c->d_ws, RX_PH_ALL, 0, 2));
        return join_cs();
    }
    rxg_ctx::ws_shape layout;
    layout.n = n;
    layout.lists = pipe == 20;
    layout.bytes = ws;
    int rc = ws_prepare(c, ws, layout, s);
    if (rc) return rc;
    if (!split) {
        HIPCHK(ws_wait(c, WS_BUF0, s));
        HIPCHK(ws_wait(c, WS_SLAB, s));
        HIPCHK(rx_classify_launch(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                                  d_out, d_counts, s, c->d_ws, RX_PH_ALL, 0, 2));
        HIPCHK(ws_mark(c, WS_BUF0, s));
        HIPCHK(ws_mark(c, WS_SLAB, s));
        return join_cs();
    }
    const uint32_t b = c->ws_flip;
    c->ws_flip ^= 1u;
    HIPCHK(ws_wait(c, b, s)); // the count that last read this index buffer
    HIPCHK(rx_classify_launch(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                              d_out, d_counts, s, c->d_ws, RX_PH_CLASSIFY, b, 2));
    HIPCHK(hipEventRecord(c->ev_k1, s));
    HIPCHK(hipStreamWaitEvent(cs, c->ev_k1, 0));
    HIPCHK(ws_wait(c, WS_SLAB, cs));
    HIPCHK(rx_classify_launch(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                              d_out, d_counts, cs, c->d_ws, RX_PH_COUNT, b, 2));
    HIPCHK(ws_mark(c, b, cs)); // covers the classify too (cs waited on it)
    HIPCHK(ws_mark(c, WS_SLAB, cs));
    return RXG_OK;
}

static int classify_dev_impl(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                             const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                             uint32_t len_hint, rxg_verdict *d_out, uint64_t *d_counts,
                             hipStream_t s, hipStream_t cs) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len || !d_out) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    uint32_t g = c->tune_g, p = c->tune_p, fpg = c->tune_fpg, pipe = c->tune_pipe;
    if (!g && pipe == ~0u) rx_pick_variant(len_hint, &g, &p, &fpg, &pipe);
    return classify_ws(c, d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe,
                       reinterpret_cast<uint4 *>(d_out),
                       reinterpret_cast<unsigned long long *>(d_counts), s, cs);
}

int rxg_classify_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                     const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t len_hint,
                     rxg_verdict *d_out, uint64_t *d_counts, void *stream) {
    return classify_dev_impl(c, d_pkts, d_off, d_len, n, off_unit_log2, len_hint, d_out,
                             d_counts, (hipStream_t)stream, nullptr);
}

int rxg_classify_dev_cs(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        uint32_t len_hint, rxg_verdict *d_out, uint64_t *d_counts, void *stream,
                        void *count_stream) {
    return classify_dev_impl(c, d_pkts, d_off, d_len, n, off_unit_log2, len_hint, d_out,
                             d_counts, (hipStream_t)stream, (hipStream_t)count_stream);
}

// Frames of a host burst into a slot: exactly `span` bytes cross PCIe (the
// caller's buffer may end there), and the device copy is zero-filled up to the
// next 16-B boundary, which the kernels read as the frame's padding.
static hipError_t copy_in_frames(rxg_ctx *c, rxg_ctx::slot &sl, const uint8_t *pkts,
                                 uint64_t span) {
    hipError_t e = hipMemcpyAsync(sl.d_pkts, pkts, span, hipMemcpyHostToDevice, c->s_h2d);
    const uint64_t pad = ((span + 15) & ~15ull) - span;
    if (e == hipSuccess && pad) e = hipMemsetAsync(sl.d_pkts + span, 0, pad, c->s_h2d);
    return e;
}

// burst -> slot: device-side ordering only (the host blocks in rxg_wait):
// the copy in waits until the slot's previous kernel has read its inputs, the
// kernel until the slot's previous verdicts have left d_out.
static int submit_slot(rxg_ctx *c, rxg_ctx::slot &sl, const uint8_t *pkts, uint64_t span,
                       const uint32_t *off, const uint16_t *len, uint32_t n,
                       uint32_t off_unit_log2, rxg_verdict *out, uint64_t ticket) {
    const bool reused = sl.ticket != 0;
    if (reused) HIPCHK(hipStreamWaitEvent(c->s_h2d, sl.ev_k, 0));
    HIPCHK(copy_in_frames(c, sl, pkts, span));
    HIPCHK(hipMemcpyAsync(sl.d_off, off, n * 4ull, hipMemcpyHostToDevice, c->s_h2d));
    HIPCHK(hipMemcpyAsync(sl.d_len, len, n * 2ull, hipMemcpyHostToDevice, c->s_h2d));
    HIPCHK(hipEventRecord(sl.ev_in, c->s_h2d));
    HIPCHK(hipStreamWaitEvent(c->stream, sl.ev_in, 0));
    if (reused) HIPCHK(hipStreamWaitEvent(c->stream, sl.ev_done, 0));
    uint32_t g = c->tune_g, p = c->tune_p, fpg = c->tune_fpg, pipe = c->tune_pipe;
    if (!g && pipe == ~0u) rx_pick_variant((uint32_t)(span / n), &g, &p, &fpg, &pipe);
    int rc = classify_ws(c, sl.d_pkts, sl.d_off, sl.d_len, n, off_unit_log2, g, p, fpg, pipe,
                         sl.d_out, c->d_counts, c->stream, nullptr);
    if (rc) return rc;
    HIPCHK(hipEventRecord(sl.ev_k, c->stream));
    HIPCHK(hipStreamWaitEvent(c->s_d2h, sl.ev_k, 0));
    HIPCHK(hipMemcpyAsync(out, sl.d_out, n * 16ull, hipMemcpyDeviceToHost, c->s_d2h));
    HIPCHK(hipEventRecord(sl.ev_done, c->s_d2h));
    sl.ticket = ticket;
    return RXG_OK;
}

static int check_host_burst(rxg_ctx *c, const uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
                            const uint16_t *len, uint32_t n, uint32_t off_unit_log2) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (!pkts || !off || !len) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    if (n > c->max_pkts || !c->slots[0].d_pkts) return RXG_ERANGE;
    if (((span_bytes + 15) & ~15ull) > c->max_bytes) return RXG_ERANGE;
    return RXG_OK;
}

int rxg_submit(rxg_ctx *c, const uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
               const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out,
               uint64_t *ticket) {
    if (ticket) *ticket = 0;
    if (n == 0) return c ? RXG_OK : RXG_EINVAL;
    if (!out) return RXG_EINVAL;
    int rc = check_host_burst(c, pkts, span_bytes, off, len, n, off_unit_log2);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t t = c->next_ticket++;
    rc = submit_slot(c, c->slots[t % RXG_PIPE_DEPTH], pkts, span_bytes, off, len, n,
                     off_unit_log2, out, t);
    if (rc == RXG_OK && ticket) *ticket = t;
    return rc;
}

int rxg_wait(rxg_ctx *c, uint64_t ticket) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (ticket == 0) return RXG_OK; // empty burst
    if (ticket >= c->next_ticket) return RXG_EINVAL;
    const rxg_ctx::slot &sl = c->slots[ticket % RXG_PIPE_DEPTH];
    // a slot reused by a later burst: its events now mark that burst, which
    // completes after this one (stream order), so waiting on it is safe
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipEventSynchronize(sl.ev_done));
    return RXG_OK;
}

int rxg_classify_span(rxg_ctx *c, const uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
                      const uint16_t *len, uint32_t n, uint32_t off_unit_log2, rxg_verdict *out) {
    uint64_t t = 0;
    int rc = rxg_submit(c, pkts, span_bytes, off, len, n, off_unit_log2, out, &t);
    return rc ? rc : rxg_wait(c, t);
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
    if (n > c->max_pkts || !c->slots[0].h_stage) return RXG_ERANGE;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t t = c->next_ticket++;
    rxg_ctx::slot &sl = c->slots[t % RXG_PIPE_DEPTH];
    if (sl.ticket) HIPCHK(hipEventSynchronize(sl.ev_in)); // the slot's last copy-in read h_stage
    // gather frames (buf_addr + data_off, data_len bytes) at 64-B aligned slots
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!m[i] || !m[i]->buf_addr) return RXG_EINVAL;
        const uint32_t l = m[i]->data_len;
        const uint64_t step = std::max<uint64_t>((l + 63ull) & ~63ull, 64);
        if (pos + step > c->max_bytes) return RXG_ERANGE;
        memcpy(sl.h_stage + pos, (const uint8_t *)m[i]->buf_addr + m[i]->data_off, l);
        if (step > l) memset(sl.h_stage + pos + l, 0, step - l);
        sl.h_off[i] = (uint32_t)(pos >> 6);
        sl.h_len[i] = (uint16_t)l;
        pos += step;
    }
    int rc = submit_slot(c, sl, sl.h_stage, pos, sl.h_off, sl.h_len, n, 6, out, t);
    return rc ? rc : rxg_wait(c, t);
}

int rxg_tx_cksum_dev(rxg_ctx *c, uint8_t *d_pkts, const uint32_t *d_off, const uint16_t *d_len,
                     uint32_t n, uint32_t off_unit_log2, uint32_t len_hint, void *stream) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(tx_cksum_launch(d_pkts, d_off, d_len, n, off_unit_log2, len_hint, c->tune_tx,
                           c->tune_tx_bpc, (hipStream_t)stream));
    return RXG_OK;
}

// host frames through one staging slot: copy in, K2, frames copied back
int rxg_tx_cksum(rxg_ctx *c, uint8_t *pkts, uint64_t span_bytes, const uint32_t *off,
                 const uint16_t *len, uint32_t n, uint32_t off_unit_log2) {
    if (n == 0) return c ? RXG_OK : RXG_EINVAL;
    int rc = check_host_burst(c, pkts, span_bytes, off, len, n, off_unit_log2);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    const uint64_t span = span_bytes;
    const uint64_t t = c->next_ticket++;
    rxg_ctx::slot &sl = c->slots[t % RXG_PIPE_DEPTH];
    if (sl.ticket) HIPCHK(hipStreamWaitEvent(c->s_h2d, sl.ev_k, 0));
    HIPCHK(copy_in_frames(c, sl, pkts, span));
    HIPCHK(hipMemcpyAsync(sl.d_off, off, n * 4ull, hipMemcpyHostToDevice, c->s_h2d));
    HIPCHK(hipMemcpyAsync(sl.d_len, len, n * 2ull, hipMemcpyHostToDevice, c->s_h2d));
    HIPCHK(hipEventRecord(sl.ev_in, c->s_h2d));
    HIPCHK(hipStreamWaitEvent(c->stream, sl.ev_in, 0));
    if (sl.ticket) HIPCHK(hipStreamWaitEvent(c->stream, sl.ev_done, 0));
    HIPCHK(tx_cksum_launch(sl.d_pkts, sl.d_off, sl.d_len, n, off_unit_log2,
                           (uint32_t)(span / n),
                           c->tune_tx, c->tune_tx_bpc, c->stream));
    HIPCHK(hipEventRecord(sl.ev_k, c->stream));
    HIPCHK(hipStreamWaitEvent(c->s_d2h, sl.ev_k, 0));
    HIPCHK(hipMemcpyAsync(pkts, sl.d_pkts, span, hipMemcpyDeviceToHost, c->s_d2h));
    HIPCHK(hipEventRecord(sl.ev_done, c->s_d2h));
    sl.ticket = t;
    HIPCHK(hipEventSynchronize(sl.ev_done));
    return RXG_OK;
}

int rxg_rss_split_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                      const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t n_shards,
                      uint32_t *d_first, uint32_t *d_perm, void *stream) {
    if (!c || !d_first || n_shards == 0 || n_shards > RXG_MAX_SHARDS) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n && (!d_pkts || !d_off || !d_len || !d_perm)) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    const hipStream_t s = (hipStream_t)stream;
    const size_t ws = rx_split_ws_bytes(n, n_shards);
    if (ws > c->d_aux_cap) { // grows between bursts only
        HIPCHK(hipDeviceSynchronize());
        int rc = ensure_dev(&c->d_aux, &c->d_aux_cap, ws);
        if (rc) return rc;
    }
    HIPCHK(rx_split_launch(d_pkts, d_off, d_len, n, off_unit_log2, n_shards, d_first, d_perm,
                           c->d_aux, s));
    return RXG_OK;
}

int rxg_gather_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                   const uint16_t *d_len, uint32_t off_unit_log2, const uint32_t *d_idx,
                   uint32_t count, uint8_t *d_dst, uint64_t dst_cap, uint32_t *d_dst_off,
                   uint16_t *d_dst_len, uint64_t *span, void *stream) {
    if (!c) return RXG_EINVAL;
    if (span) *span = 0;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (count == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len || !d_idx || !d_dst || !d_dst_off || !d_dst_len)
        return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    HIPCHK(hipSetDevice(c->device));
    const hipStream_t s = (hipStream_t)stream;
    const size_t ws = rx_gather_ws_bytes(count);
    if (ws > c->d_aux_cap) {
        HIPCHK(hipDeviceSynchronize());
        int rc = ensure_dev(&c->d_aux, &c->d_aux_cap, ws);
        if (rc) return rc;
    }
    HIPCHK(rx_gather_launch(d_pkts, d_off, d_len, off_unit_log2, d_idx, count, d_dst, dst_cap,
                            d_dst_off, d_dst_len, c->d_aux, s));
    // the packed size (64-B units) sits after the per-chunk sums
    const size_t nchunks = (ws - 8) / 8;
    uint64_t units = 0;
    HIPCHK(hipMemcpyAsync(&units, reinterpret_cast<uint64_t *>(c->d_aux) + nchunks, 8,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (span) *span = units << 6;
    if ((units << 6) > dst_cap || units > 0xFFFFFFFFull) return RXG_ERANGE;
    return RXG_OK;
}

int rxg_ctx_counts_allreduce(rxg_ctx *c, rxg_group *g) {
    if (!c || !g) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    HIPCHK(hipSetDevice(c->device));
    const uint32_t nf = c->ft.nu + c->ft.nt;
    int rc = rx_group_allreduce_u64(g, c->d_counts, nf, c->stream); // after the bursts' kernels
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return RXG_OK;
}

int rxg_flow_counts(rxg_ctx *c, uint64_t *counts, uint32_t ncounts) {
    if (!c || (ncounts && !counts)) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    const uint32_t nf = c->ft.nu + c->ft.nt;
    if (ncounts < nf) return RXG_ERANGE;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream)); // every submitted burst's kernel has counted
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
