// rx_api.hip — host side of librxgpu: context, flow-table build/upload, the
// burst entry points of include/rxgpu.h.  Device work is in rx_classify.hip;
// there is no CPU classification path in this library: every verdict comes
// from the gfx950 kernel, and a missing/failed device is an error.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "rx_common.h"
#include "rx_flows.h"

void rx_pick_variant(uint32_t len_hint, uint32_t *g, uint32_t *p, uint32_t *fpg, uint32_t *pipe,
                     bool v8 = false);
bool rx_variant_exists(uint32_t g, uint32_t p, uint32_t fpg, uint32_t pipe);
const char *rx_variant_kernel(uint32_t g, uint32_t pipe);
hipError_t rx_classify_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                              uint32_t n, uint32_t unit_log2, uint32_t g, uint32_t p, uint32_t fpg,
                              uint32_t pipe, const rx_ft_dev &ft, uint4 *out,
                              unsigned long long *counts, hipStream_t s, uint32_t *ws,
                              uint32_t phase, uint32_t buf, uint32_t nbuf);
// the same kernels writing 8-B verdicts (rx_classify.hip built with RX_V8=1)
hipError_t rx_classify_launch8(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
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
size_t rx_segsort_ws_bytes(uint32_t n);
hipError_t rx_ingest_launch(const unsigned long long *src, const uint32_t *off, const uint16_t *len,
                            uint32_t n, uint8_t *dst, hipStream_t s);
hipError_t rx_segsort_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                             uint32_t n, uint32_t unit_log2, const uint4 *verd, uint32_t nt,
                             rxg_segment *seg, uint8_t *payload, uint64_t cap, uint32_t *totals,
                             void *ws, hipStream_t s);
size_t rx_compact_ws_bytes(uint32_t n, uint32_t nflows);
hipError_t rx_compact_launch(const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                             uint32_t n, uint32_t unit_log2, const uint4 *verd, uint32_t nflows,
                             rxg_dgram *dg, uint32_t *first, uint8_t *payload, uint64_t cap,
                             uint32_t *totals, void *ws, hipStream_t s);

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

// one incremental table write (rxg_flows_commit): rx_delta_kernel stores v
// at element idx of table `which`
// (RX_D_CZERO: count index idx of a removed block, zeroed in both of the
// context's count vectors before its id can name a new block)
enum { RX_D_UDP = 0, RX_D_TCP = 1, RX_D_LISTEN = 2, RX_D_PORT = 3, RX_D_UDPC = 4, RX_D_UDPW = 5,
       RX_D_CZERO = 6 };
struct rx_delta {
    uint32_t which, idx, _r0, _r1;
    uint4 v;
};
#define RX_DELTA_CAP 65536u // records per commit; more: whole arrays are uploaded
#define RX_DELTA_ROOM (RX_DELTA_CAP + 2048u) // staging records (the small tables ride on top)

__global__ __launch_bounds__(256) void rx_delta_kernel(const rx_delta *__restrict__ d, uint32_t n,
                                                       uint4 *udp, uint4 *tcp, uint32_t *listen,
                                                       uint32_t *port, uint4 *udpc, uint4 *udpw,
                                                       unsigned long long *cnt,
                                                       unsigned long long *cnt_base) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const rx_delta r = d[i];
    switch (r.which) {
    case RX_D_UDP: udp[r.idx] = r.v; break;
    case RX_D_TCP: tcp[r.idx] = r.v; break;
    case RX_D_LISTEN: listen[r.idx] = r.v.x; break;
    case RX_D_PORT: port[r.idx] = r.v.x; break;
    case RX_D_UDPC: udpc[r.idx] = r.v; break;
    case RX_D_CZERO: cnt[r.idx] = 0ull, cnt_base[r.idx] = 0ull; break;
    default: udpw[r.idx] = r.v; break;
    }
}

// fold of two u64 count vectors: base += delta, delta = 0 (the all-reduced
// increment of rxg_ctx_counts_allreduce joins the running total)
__global__ __launch_bounds__(256) void rx_counts_fold_kernel(unsigned long long *base,
                                                             unsigned long long *delta, uint32_t n) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    base[i] += delta[i];
    delta[i] = 0;
}

// a stream bursts of this context ran on, and the event recorded after its
// last burst: table writes wait on it, so they never overtake a burst still
// reading the tables (a per-context wait, never a device-wide one)
struct rx_track {
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    uint64_t commit_seen = 0; // last table commit this stream is ordered after
    uint64_t last_use = 0;
    bool used = false;
};
#define RX_TRACK 4

struct rxg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // flow tables: host images + registry (rx_flows.h), device copies
    rx_flowset fs;
    bool dirty = false; // host changes not yet on the device (rxg_flows_commit)
    uint4 *d_udp = nullptr, *d_tcp = nullptr;
    size_t d_udp_cap = 0, d_tcp_cap = 0; // bytes
    uint32_t *d_listen = nullptr;   // 65536
    uint32_t *d_udp_port = nullptr; // 65536
    uint2 *d_udpc = nullptr;        // up to 2 * RX_UDPC_MAX_FLOWS slots
    uint16_t *d_udpw = nullptr;     // up to RX_UDPW_MAX_PORTS
    rx_delta *h_delta = nullptr, *d_delta = nullptr; // pinned staging + device copy
    hipEvent_t ev_commit = nullptr; // after the last commit's writes
    uint64_t commit_gen = 0;
    rx_track trk[RX_TRACK];
    rx_track *cur = nullptr; // the stream of the latest burst (its event not yet recorded)
    uint64_t use_clock = 0;
    uint32_t tune_tables = 0; // rxg_tune_tables flags
    uint32_t tune_ingest = RXG_INGEST_AUTO; // rxg_tune_ingest
    uint32_t deliver_flags = 0;             // rxg_tune_deliver (RXG_DLV_*)
    rx_ft_dev ft{};
    uint32_t tune_g = 0, tune_p = 0, tune_fpg = 0, tune_pipe = ~0u; // rxg_tune override
    uint32_t tune_bpc = 0; // rxg_tune_grid: resident blocks per CU cap (0 = occupancy)
    uint32_t tune_tx = RXG_TX_AUTO, tune_tx_bpc = 0; // rxg_tune_tx
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
    } wu[4]; // index buffers 0..2, slabs (WS_*)
    // region offsets depend on the burst shape (frame count, binned path, size);
    // a change of shape waits on every region
    struct ws_shape {
        uint32_t n = 0;
        bool lists = false;
        size_t bytes = 0;
        bool operator!=(const ws_shape &o) const { return n != o.n || lists != o.lists || bytes != o.bytes; }
    } ws_layout;
    uint32_t ws_flip = 0; // index buffer of the next split-stream burst
    uint32_t ws_nbuf = 3; // index buffers of the split-stream bursts (RXG_TT_COUNT_2BUF: 2)
    hipEvent_t ev_k1 = nullptr; // split-stream burst: classify done (count stream waits on it)
    void *d_aux = nullptr; // RSS split / gather workspace, grown on demand
    size_t d_aux_cap = 0;
    hipEvent_t ev_aux = nullptr; // after the last split / gather that used d_aux
    hipStream_t aux_st = nullptr;
    bool aux_used = false;
    // context-owned per-flow counts (host-buffer path): d_counts since the last
    // rxg_ctx_counts_allreduce, d_counts_base the all-reduced total before it
    unsigned long long *d_counts = nullptr, *d_counts_base = nullptr;
    uint32_t counts_cap = 0;
    // ids removed since the last commit: their counts are zeroed by that
    // commit (RX_D_CZERO), so a reused id starts from 0
    std::vector<uint32_t> czero_udp, czero_tcp;
    // host-buffer path: a ring of RXG_PIPE_DEPTH staging slots; burst t uses
    // slot t % depth.  Copies in run on s_h2d, kernels on `stream`, verdict
    // copies out on s_d2h, chained by events, so burst t+1's frames cross PCIe
    // while burst t is classified and burst t-1's verdicts come back.
    uint32_t max_pkts = 0;
    uint64_t max_bytes = 0;
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    struct slot {
        uint8_t *h_stage = nullptr; // pinned, mbuf gather
        unsigned long long *h_src = nullptr, *d_src = nullptr; // device-pulled frames (registered)
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
    // UDP compaction results of the host-buffer path (rxg_process_mbufs_udp):
    // device buffers and their pinned host copies, sized by max_pkts / max_bytes
    rxg_dgram *d_cp_dg = nullptr, *h_cp_dg = nullptr;
    uint32_t *d_cp_first = nullptr, *h_cp_first = nullptr;
    uint8_t *d_cp_payload = nullptr, *h_cp_payload = nullptr;
    uint32_t *d_cp_totals = nullptr, *h_cp_totals = nullptr;
    void *d_cp_ws = nullptr;
    size_t d_cp_ws_cap = 0;
    // TCP segment sort + payload gather (K4, rxg_process_mbufs_deliver): device
    // results and their pinned host copies, sized by max_pkts / max_bytes
    rxg_segment *d_ss_seg = nullptr;
    uint8_t *d_ss_payload = nullptr;
    // pinned payload buffers a caller may keep past the next burst
    // (rxg_payload_hold / _release: the receive fragments of a burst point
    // into them until the application has read them); refs counts the holds,
    // the library's own one included (until its next burst call)
    struct pl_buf {
        uint8_t *h = nullptr;
        std::atomic<int> refs{0};
    } pl[RXG_PAYLOAD_BUFS];
    // the delivery sets (rxg_deliver_submit / _wait): up to RXG_DELIVER_DEPTH
    // bursts in flight, each with its own pinned copies of the results (the
    // device buffers are shared: every step runs on `stream`, in order) and its
    // phase events; a set's results stay valid until the set is reused
    struct delivery_set {
        bool on = false, udp = false, tcp = false;
        uint64_t ticket = 0;
        double t0 = 0, t1 = 0;
        int pl = -1; // the pooled payload buffer the library holds for this set
        rxg_dgram *h_cp_dg = nullptr;
        uint32_t *h_cp_first = nullptr, *h_cp_totals = nullptr;
        uint8_t *h_cp_payload = nullptr;
        rxg_segment *h_ss_seg = nullptr;
        uint8_t *h_ss_payload = nullptr;
        uint32_t *h_ss_totals = nullptr;
        hipEvent_t tev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    } dls[RXG_DELIVER_DEPTH];
    uint32_t dl_next = 0; // the set the next submit takes (round robin)
    uint32_t *d_ss_totals = nullptr;
    void *d_ss_ws = nullptr;
    size_t d_ss_ws_cap = 0;
    // registered host memory (rxg_register_host): frames of an mbuf burst that
    // all lie in it are pulled by the device instead of gathered on the host
    struct host_region {
        uint8_t *h = nullptr, *d = nullptr;
        uint64_t bytes = 0;
        bool ours = false; // registered here (unregistered at close)
    };
    std::vector<host_region> regions;
    uint32_t region_hint = 0;
};

// a flow-table array of at least `bytes`, stream-ordered on s (hipMallocAsync /
// hipFreeAsync: neither synchronises the device, unlike hipFree)
static int ensure_dev_async(void **p, size_t *cap, size_t bytes, hipStream_t s) {
    if (*cap >= bytes && *p) return RXG_OK;
    if (*p) HIPCHK(hipFreeAsync(*p, s));
    *p = nullptr;
    *cap = 0;
    HIPCHK(hipMallocAsync(p, bytes, s));
    *cap = bytes;
    return RXG_OK;
}

// Save the calling thread's current device, switch to the context's, restore
// it on scope exit: the API never leaves a C host thread on another device.
struct dev_guard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit dev_guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~dev_guard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};
#define DEVGUARD(c)                                                                                \
    dev_guard dg_((c)->device);                                                                    \
    HIPCHK(dg_.err)

// a fresh hash seed (rx_hash3s): random at rxg_open, then a mix on reseeds
static uint32_t next_seed(uint32_t s) {
    uint64_t z = rx_mix64(((uint64_t)s << 32) ^ 0xA0761D6478BD642Full);
    return (uint32_t)(z >> 32) | 1u;
}
static uint32_t random_seed() {
    uint32_t s = 0;
    FILE *f = fopen("/dev/urandom", "rb");
    if (f) {
        if (fread(&s, sizeof(s), 1, f) != 1) s = 0;
        fclose(f);
    }
    s ^= (uint32_t)(uintptr_t)&s ^ (uint32_t)clock();
    return next_seed(s);
}

// ---- burst tracking ----------------------------------------------------
// Table writes (commits, rxg_flows_sync) must follow every burst of this
// context still reading the tables, on whatever stream it ran — never the
// device's other work.  An event per burst would do it but costs the burst
// loop ~1% at cfg2 (0.2361 vs 0.2330 ms, interleaved A/B in one process,
// profiles/r03a/ab_track.txt), so events are recorded only when needed: on a
// stream switch, on the stream the context leaves (it was used a moment
// ago), and lazily on the current stream when a table write comes.  The
// stream of the context's most recent burst must therefore still exist at
// the context's next call (rxgpu.h).
static int track_slot(rxg_ctx *c, hipStream_t s, rx_track **out) {
    rx_track *t = nullptr, *old = &c->trk[0];
    for (rx_track &x : c->trk) {
        if (x.used && x.s == s) t = &x;
        if (!x.used || (old->used && x.last_use < old->last_use)) old = &x;
    }
    if (!t) {
        t = old;
        if (t->used) HIPCHK(hipEventSynchronize(t->ev)); // (never the current stream: LRU)
        t->s = s;
        t->used = true;
        t->commit_seen = c->commit_gen; // (a new stream: tables already on the device
                                        // unless a commit is pending, which runs on s)
        if (c->commit_gen) HIPCHK(hipStreamWaitEvent(s, c->ev_commit, 0));
    }
    t->last_use = ++c->use_clock;
    *out = t;
    return RXG_OK;
}

// the event of tracking entry x marks its stream's last burst: recorded now
// for the current stream (lazily), already recorded for the others
static hipError_t track_mark(rxg_ctx *c, rx_track &x) {
    if (&x != c->cur) return hipSuccess;
    hipError_t e = hipEventRecord(x.ev, x.s);
    if (e == hipSuccess) c->cur = nullptr; // (its event now covers all its bursts)
    return e;
}

// before a burst on s: the pending table changes, then order s after the last commit
static int commit_on(rxg_ctx *c, hipStream_t s);
static int burst_begin(rxg_ctx *c, hipStream_t s) {
    if (c->dirty) {
        int rc = commit_on(c, s);
        if (rc) return rc;
    }
    rx_track *t;
    int rc = track_slot(c, s, &t);
    if (rc) return rc;
    if (c->cur && c->cur != t) HIPCHK(track_mark(c, *c->cur)); // leaving a stream
    c->cur = t;
    if (t->commit_seen < c->commit_gen) {
        HIPCHK(hipStreamWaitEvent(s, c->ev_commit, 0));
        t->commit_seen = c->commit_gen;
    }
    return RXG_OK;
}
// host wait for every burst of this context (a table rebuild in place)
static int bursts_drain(rxg_ctx *c) {
    for (rx_track &x : c->trk)
        if (x.used) {
            HIPCHK(track_mark(c, x));
            HIPCHK(hipEventSynchronize(x.ev));
        }
    for (rxg_ctx::ws_use &u : c->wu)
        if (u.used) HIPCHK(hipEventSynchronize(u.ev));
    if (c->stream) HIPCHK(hipStreamSynchronize(c->stream));
    if (c->s_h2d) HIPCHK(hipStreamSynchronize(c->s_h2d));
    if (c->s_d2h) HIPCHK(hipStreamSynchronize(c->s_d2h));
    return RXG_OK;
}

// ---- device upload of the flow tables ------------------------------------
static void ft_fill(rxg_ctx *c) {
    const rx_flowset &fs = c->fs;
    c->ft.udp = c->d_udp;
    c->ft.tcp = c->d_tcp;
    c->ft.listen = c->d_listen;
    c->ft.udp_mask = fs.udp.tab.mask;
    c->ft.tcp_mask = fs.tcp.tab.mask;
    c->ft.udp_probe = fs.udp.live ? fs.udp.tab.probe : 0;
    c->ft.tcp_probe = fs.tcp.live ? fs.tcp.tab.probe : 0;
    c->ft.hseed = fs.seed;
    c->ft.udpc = fs.udpc.empty() ? nullptr : c->d_udpc;
    c->ft.udpc_mask = fs.udpc.empty() ? 0 : (uint32_t)fs.udpc.size() - 1;
    c->ft.udpc_probe = fs.udpc_probe;
    c->ft.udpc_other = fs.udpc_other;
    c->ft.udp_port = fs.port.empty() ? nullptr : c->d_udp_port;
    c->ft.udp_dip = fs.udp_dip;
    c->ft.udpw = fs.udpw.empty() ? nullptr : c->d_udpw;
    c->ft.udpw_lo = fs.udpw_lo;
    c->ft.udpw_n = (uint32_t)fs.udpw.size();
}

// whole arrays (a rebuild, or more changes than one delta batch holds), on s;
// the host waits for the copies (pageable sources)
static int upload_tab(rx_slot_table &t, uint4 **d, size_t *cap, hipStream_t s) {
    const size_t bytes = t.slots.size() * sizeof(uint4);
    int rc = ensure_dev_async((void **)d, cap, bytes, s);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(*d, t.slots.data(), bytes, hipMemcpyHostToDevice, s));
    t.all_dirty = false;
    t.dirty.clear();
    return RXG_OK;
}

// the counts follow the id space: UDP ids [0, nu), TCP ids at nu + id; a
// grown id space moves the context's own count vectors to the new layout
static int counts_layout(rxg_ctx *c, uint32_t nu, uint32_t nt, hipStream_t s) {
    const uint32_t onu = c->ft.nu, ont = c->ft.nt;
    const uint32_t nf = std::max(nu + nt, 1u);
    if (c->d_counts && nu == onu && nt == ont) return RXG_OK;
    unsigned long long *a = nullptr, *b = nullptr;
    HIPCHK(hipMallocAsync((void **)&a, (size_t)nf * 8, s));
    HIPCHK(hipMallocAsync((void **)&b, (size_t)nf * 8, s));
    HIPCHK(hipMemsetAsync(a, 0, (size_t)nf * 8, s));
    HIPCHK(hipMemsetAsync(b, 0, (size_t)nf * 8, s));
    if (c->d_counts) {
        unsigned long long *src[2] = {c->d_counts, c->d_counts_base}, *dst[2] = {a, b};
        for (int k = 0; k < 2; ++k) {
            const uint32_t ku = std::min(onu, nu), kt = std::min(ont, nt);
            if (ku) HIPCHK(hipMemcpyAsync(dst[k], src[k], ku * 8ull, hipMemcpyDeviceToDevice, s));
            if (kt)
                HIPCHK(hipMemcpyAsync(dst[k] + nu, src[k] + onu, kt * 8ull, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipFreeAsync(src[k], s));
        }
    }
    c->d_counts = a;
    c->d_counts_base = b;
    c->counts_cap = nf;
    c->ft.nu = nu;
    c->ft.nt = nt;
    return RXG_OK;
}

// every pending host change of the flow tables onto the device, in stream
// order on s (after the bursts of other streams that may still read them)
static int commit_on(rxg_ctx *c, hipStream_t s) {
    if (c->device == RXG_HOST_ONLY) {
        c->dirty = false;
        return RXG_OK;
    }
    rx_flowset &fs = c->fs;
    for (rx_track &x : c->trk)
        if (x.used && x.s != s) {
            HIPCHK(track_mark(c, x));
            HIPCHK(hipStreamWaitEvent(s, x.ev, 0));
        }
    for (rxg_ctx::ws_use &u : c->wu)
        if (u.used && u.st != s) HIPCHK(hipStreamWaitEvent(s, u.ev, 0));
    int rc = counts_layout(c, fs.udp.id_space(), fs.tcp.id_space(), s);
    if (rc) return rc;
    // the previous commit's staging copy must be done before it is refilled
    if (c->commit_gen) HIPCHK(hipEventSynchronize(c->ev_commit));
    const size_t nrec = fs.udp.tab.dirty.size() + fs.tcp.tab.dirty.size() +
                        fs.listen_dirty.size() + fs.port_dirty.size() +
                        (fs.small_dirty ? (fs.udpc.size() / 2 + (fs.udpw.size() + 7) / 8) : 0);
    const bool whole = nrec > RX_DELTA_CAP;
    bool sync = false;
    if (fs.udp.tab.all_dirty || whole) {
        if ((rc = upload_tab(fs.udp.tab, &c->d_udp, &c->d_udp_cap, s))) return rc;
        sync = true;
    }
    if (fs.tcp.tab.all_dirty || whole) {
        if ((rc = upload_tab(fs.tcp.tab, &c->d_tcp, &c->d_tcp_cap, s))) return rc;
        sync = true;
    }
    if (fs.listen_all_dirty || whole) {
        HIPCHK(hipMemcpyAsync(c->d_listen, fs.listen.data(), 65536 * 4, hipMemcpyHostToDevice, s));
        fs.listen_all_dirty = false;
        fs.listen_dirty.clear();
        sync = true;
    }
    if ((fs.port_all_dirty || whole) && !fs.port.empty()) {
        HIPCHK(hipMemcpyAsync(c->d_udp_port, fs.port.data(), 65536 * 4, hipMemcpyHostToDevice, s));
        sync = true;
    }
    if (fs.port_all_dirty || whole) fs.port_all_dirty = false, fs.port_dirty.clear();
    uint32_t n = 0;
    rx_delta *r = c->h_delta;
    auto put = [&](uint32_t which, uint32_t idx, uint4 v) {
        r[n].which = which;
        r[n].idx = idx;
        r[n]._r0 = r[n]._r1 = 0;
        r[n].v = v;
        ++n;
    };
    for (uint32_t i : fs.udp.tab.dirty) put(RX_D_UDP, i, fs.udp.tab.slots[i]);
    for (uint32_t i : fs.tcp.tab.dirty) put(RX_D_TCP, i, fs.tcp.tab.slots[i]);
    for (uint32_t p : fs.listen_dirty) put(RX_D_LISTEN, p, make_uint4(fs.listen[p], 0, 0, 0));
    if (!fs.port.empty())
        for (uint32_t p : fs.port_dirty) put(RX_D_PORT, p, make_uint4(fs.port[p], 0, 0, 0));
    if (fs.small_dirty) {
        for (size_t k = 0; 2 * k < fs.udpc.size(); ++k) {
            const uint2 x = fs.udpc[2 * k], y = fs.udpc[2 * k + 1];
            put(RX_D_UDPC, (uint32_t)k, make_uint4(x.x, x.y, y.x, y.y));
        }
        for (size_t k = 0; 8 * k < fs.udpw.size(); ++k) {
            uint32_t w[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
            for (size_t j = 0; j < 8 && 8 * k + j < fs.udpw.size(); ++j) {
                const uint32_t sh = 16u * (uint32_t)(j & 1);
                w[j / 2] = (w[j / 2] & ~(0xFFFFu << sh)) | ((uint32_t)fs.udpw[8 * k + j] << sh);
            }
            put(RX_D_UDPW, (uint32_t)k, make_uint4(w[0], w[1], w[2], w[3]));
        }
        fs.small_dirty = false;
    }
    fs.udp.tab.dirty.clear();
    fs.tcp.tab.dirty.clear();
    fs.listen_dirty.clear();
    fs.port_dirty.clear();
    // the staged records to the device and the scatter kernel; a full staging
    // buffer (more removed ids than it holds) is flushed and refilled after
    // its copy has left
    auto flush = [&]() -> int {
        if (!n) return RXG_OK;
        HIPCHK(hipMemcpyAsync(c->d_delta, c->h_delta, n * sizeof(rx_delta), hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(rx_delta_kernel, dim3((n + 255) / 256), dim3(256), 0, s, c->d_delta, n,
                           c->d_udp, c->d_tcp, c->d_listen, c->d_udp_port,
                           reinterpret_cast<uint4 *>(c->d_udpc), reinterpret_cast<uint4 *>(c->d_udpw),
                           c->d_counts, c->d_counts_base);
        HIPCHK(hipGetLastError());
        n = 0;
        return RXG_OK;
    };
    // counts of removed ids (in the layout counts_layout just made: TCP at nu + id)
    const uint32_t nf = c->ft.nu + c->ft.nt;
    for (int k = 0; k < 2; ++k)
        for (uint32_t id : k ? c->czero_tcp : c->czero_udp) {
            const uint32_t idx = k ? c->ft.nu + id : id;
            if (idx >= nf || (!k && id >= c->ft.nu)) continue;
            if (n == RX_DELTA_ROOM) {
                if ((rc = flush())) return rc;
                HIPCHK(hipEventRecord(c->ev_commit, s));
                HIPCHK(hipEventSynchronize(c->ev_commit)); // (the staging copy has left)
            }
            put(RX_D_CZERO, idx, make_uint4(0, 0, 0, 0));
        }
    c->czero_udp.clear();
    c->czero_tcp.clear();
    if ((rc = flush())) return rc;
    HIPCHK(hipEventRecord(c->ev_commit, s));
    ++c->commit_gen;
    for (rx_track &x : c->trk)
        if (x.used && x.s == s) x.commit_seen = c->commit_gen;
    ft_fill(c);
    c->dirty = false;
    if (sync) HIPCHK(hipStreamSynchronize(s)); // (pageable whole-array sources)
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
        c->fs.seed = random_seed();
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
    c->fs.seed = random_seed();
    dev_guard dg(device);
    do {
        if ((rc = rx_set_hip_error(dg.err))) break;
        if ((rc = rx_set_hip_error(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking))))
            break;
        if ((rc = rx_set_hip_error(hipMalloc(&c->d_listen, 65536 * sizeof(uint32_t))))) break;
        if ((rc = rx_set_hip_error(hipMalloc(&c->d_udp_port, 65536 * sizeof(uint32_t))))) break;
        if ((rc = rx_set_hip_error(hipMalloc(&c->d_udpc, 2 * RX_UDPC_MAX_FLOWS * sizeof(uint2))))) break;
        if ((rc = rx_set_hip_error(hipMalloc(&c->d_udpw, RX_UDPW_MAX_PORTS * sizeof(uint16_t))))) break;
        const size_t dbytes = RX_DELTA_ROOM * sizeof(rx_delta);
        if ((rc = rx_set_hip_error(hipHostMalloc((void **)&c->h_delta, dbytes, 0)))) break;
        if ((rc = rx_set_hip_error(hipMalloc(&c->d_delta, dbytes)))) break;
        if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&c->ev_commit, hipEventDisableTiming))))
            break;
        for (rx_track &t : c->trk)
            if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&t.ev, hipEventDisableTiming)))) break;
        if (rc) break;
        for (rxg_ctx::ws_use &u : c->wu)
            if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&u.ev, hipEventDisableTiming))))
                break;
        if (rc) break;
        if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&c->ev_k1, hipEventDisableTiming))))
            break;
        if ((rc = rx_set_hip_error(hipEventCreateWithFlags(&c->ev_aux, hipEventDisableTiming))))
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
    dev_guard dg(c->device);
    // waits for what the context can name without touching the caller's
    // streams: their recorded events and the context's own streams.  The
    // stream of the latest burst (c->cur, its event not recorded) may already
    // be destroyed (the usual teardown order: synchronise, destroy the stream,
    // close), so nothing is recorded on it; hipFree below synchronises the
    // device before it releases memory a kernel could still read.
    for (rx_track &x : c->trk)
        if (x.used && &x != c->cur) (void)hipEventSynchronize(x.ev);
    for (rxg_ctx::ws_use &u : c->wu)
        if (u.used) (void)hipEventSynchronize(u.ev);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->s_h2d) (void)hipStreamSynchronize(c->s_h2d);
    if (c->s_d2h) (void)hipStreamSynchronize(c->s_d2h);
    (void)hipFree(c->d_udp);
    (void)hipFree(c->d_tcp);
    (void)hipFree(c->d_listen);
    (void)hipFree(c->d_udp_port);
    (void)hipFree(c->d_udpc);
    (void)hipFree(c->d_udpw);
    (void)hipFree(c->d_delta);
    if (c->h_delta) (void)hipHostFree(c->h_delta);
    (void)hipFree(c->d_counts);
    (void)hipFree(c->d_counts_base);
    (void)hipFree(c->d_ws);
    (void)hipFree(c->d_aux);
    (void)hipFree(c->d_cp_dg);
    (void)hipFree(c->d_cp_first);
    (void)hipFree(c->d_cp_payload);
    (void)hipFree(c->d_cp_totals);
    (void)hipFree(c->d_cp_ws);
    (void)hipFree(c->d_ss_seg);
    (void)hipFree(c->d_ss_payload);
    (void)hipFree(c->d_ss_totals);
    (void)hipFree(c->d_ss_ws);
    for (rxg_ctx::delivery_set &ds : c->dls) {
        for (void *h : {(void *)ds.h_cp_dg, (void *)ds.h_cp_first, (void *)ds.h_cp_totals,
                        (void *)ds.h_cp_payload, (void *)ds.h_ss_seg, (void *)ds.h_ss_payload,
                        (void *)ds.h_ss_totals})
            if (h) (void)hipHostFree(h);
        for (hipEvent_t e : ds.tev)
            if (e) (void)hipEventDestroy(e);
    }
    for (rxg_ctx::pl_buf &b : c->pl)
        if (b.h) (void)hipHostFree(b.h);
    if (c->h_cp_dg) (void)hipHostFree(c->h_cp_dg);
    if (c->h_cp_first) (void)hipHostFree(c->h_cp_first);
    if (c->h_cp_payload) (void)hipHostFree(c->h_cp_payload);
    if (c->h_cp_totals) (void)hipHostFree(c->h_cp_totals);
    for (rxg_ctx::ws_use &u : c->wu)
        if (u.ev) (void)hipEventDestroy(u.ev);
    for (rx_track &t : c->trk)
        if (t.ev) (void)hipEventDestroy(t.ev);
    if (c->ev_commit) (void)hipEventDestroy(c->ev_commit);
    if (c->ev_k1) (void)hipEventDestroy(c->ev_k1);
    if (c->ev_aux) (void)hipEventDestroy(c->ev_aux);
    for (rxg_ctx::slot &sl : c->slots) {
        (void)hipFree(sl.d_pkts);
        (void)hipFree(sl.d_off);
        (void)hipFree(sl.d_len);
        (void)hipFree(sl.d_out);
        if (sl.h_stage) (void)hipHostFree(sl.h_stage);
        if (sl.h_off) (void)hipHostFree(sl.h_off);
        if (sl.h_len) (void)hipHostFree(sl.h_len);
        if (sl.h_src) (void)hipHostFree(sl.h_src);
        (void)hipFree(sl.d_src);
        if (sl.ev_in) (void)hipEventDestroy(sl.ev_in);
        if (sl.ev_k) (void)hipEventDestroy(sl.ev_k);
        if (sl.ev_done) (void)hipEventDestroy(sl.ev_done);
    }
    for (const rxg_ctx::host_region &r : c->regions)
        if (r.ours) (void)hipHostUnregister(r.h);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->s_h2d) (void)hipStreamDestroy(c->s_h2d);
    if (c->s_d2h) (void)hipStreamDestroy(c->s_d2h);
    delete c;
}

// ---- control blocks (rx_flows.h) ------------------------------------------
static void udp_set(rx_block &x, const rxg_udp_sock &u) {
    x.a = u.localip;
    x.b = u.localport;
    x.c = 17u;
    x.status = u.protocol;
    // get_hostinfo_fromip_port matches (dip, dport, proto); every socket the
    // reference creates has protocol 17 (nsocket, common.c:281) and the lookup
    // is only called with 17 (udp.c:14), so other protocols never match
    x.keyed = u.protocol == 17;
}
static void tcp_set(rx_block &x, const rxg_tcb &t) {
    x.a = t.sip;
    x.b = t.dip;
    x.c = (uint32_t)t.sport | ((uint32_t)t.dport << 16);
    x.status = t.status;
    x.keyed = true;
}

// the whole flow set, then every device table: a control-plane operation that
// waits for this context's own bursts (never the device's other work)
static int full_upload(rxg_ctx *c) {
    c->fs.rebuild_all(next_seed);
    c->dirty = true;
    if (c->device == RXG_HOST_ONLY) {
        c->ft.nu = c->fs.udp.id_space();
        c->ft.nt = c->fs.tcp.id_space();
        c->ft.hseed = c->fs.seed;
        c->dirty = false;
        return RXG_OK;
    }
    DEVGUARD(c);
    int rc = bursts_drain(c);
    if (rc) return rc;
    rc = commit_on(c, c->stream);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return RXG_OK;
}

int rxg_flows_sync(rxg_ctx *c, const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t, uint32_t nt) {
    if (!c || (nu && !u) || (nt && !t)) return RXG_EINVAL;
    rx_flowset &fs = c->fs;
    fs.clear();
    c->czero_udp.clear(); // (the counts are zeroed whole below)
    c->czero_tcp.clear();
    fs.port_table = !(c->tune_tables & RXG_TT_NO_UDP_PORT);
    fs.udp.blk.resize(nu);
    for (uint32_t i = 0; i < nu; ++i) {
        rx_block &x = fs.udp.blk[i];
        udp_set(x, u[i]);
        x.seq = fs.udp.seq_next++;
        x.live = true;
    }
    fs.udp.live = nu;
    fs.tcp.blk.resize(nt);
    for (uint32_t i = 0; i < nt; ++i) {
        rx_block &x = fs.tcp.blk[i];
        tcp_set(x, t[i]);
        x.seq = fs.tcp.seq_next++;
        x.live = true;
    }
    fs.tcp.live = nt;
    for (uint32_t i = 0; i < nt; ++i)
        if (t[i].status == RXG_TCP_STATUS_LISTEN) fs.listen_add(i);
    int rc = full_upload(c); // (rebuild_all places each key's newest block)
    if (rc) return rc;
    // chains of duplicate keys, newest first: one walk over the blocks, newest first
    for (rx_registry *r : {&fs.udp, &fs.tcp}) {
        std::vector<uint32_t> tail(r->tab.ns(), RXG_FLOW_NONE);
        for (uint32_t id = (uint32_t)r->blk.size(); id-- > 0;) {
            rx_block &x = r->blk[id];
            x.older = RXG_FLOW_NONE;
            if (!x.keyed) continue;
            const uint32_t i = r->tab.find(x.a, x.b, x.c);
            if (tail[i] != RXG_FLOW_NONE) r->blk[tail[i]].older = id;
            tail[i] = id;
        }
    }
    if (c->device != RXG_HOST_ONLY) { // context counts follow the flow set
        DEVGUARD(c);
        HIPCHK(hipMemsetAsync(c->d_counts, 0, (size_t)c->counts_cap * 8, c->stream));
        HIPCHK(hipMemsetAsync(c->d_counts_base, 0, (size_t)c->counts_cap * 8, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return RXG_OK;
}

// a table past load 1/2 or a probe sequence past RX_PROBE_CAP: rebuilt whole
// (the next commit uploads it); the registry changes stay O(1) otherwise
static void after_change(rxg_ctx *c, bool cap_ok) {
    rx_flowset &fs = c->fs;
    if (!cap_ok || fs.needs_rebuild(fs.udp, false) || fs.needs_rebuild(fs.tcp, false))
        fs.rebuild_all(next_seed);
    c->dirty = true;
}

static bool udp_link(rx_flowset &fs, uint32_t id) {
    rx_block &x = fs.udp.blk[id];
    if (!x.keyed) return true;
    const bool ok = fs.udp.link(id);
    if (fs.port_table && (fs.port.empty() || (fs.on_dip == 0 && x.a != fs.udp_dip)))
        fs.port_rebuild(); // first socket, or none left on the table's address
    else
        fs.port_track(x, +1);
    return ok;
}
static void udp_unlink(rx_flowset &fs, uint32_t id) {
    rx_block &x = fs.udp.blk[id];
    if (!x.keyed) return;
    fs.udp.unlink(id);
    fs.port_track(x, -1);
}

int rxg_flows_add(rxg_ctx *c, const rxg_udp_sock *u, uint32_t nu, const rxg_tcb *t, uint32_t nt,
                  uint32_t *udp_ids, uint32_t *tcp_ids) {
    if (!c || (nu && (!u || !udp_ids)) || (nt && (!t || !tcp_ids))) return RXG_EINVAL;
    rx_flowset &fs = c->fs;
    const uint32_t onu = fs.udp.id_space(), ont = fs.tcp.id_space();
    // room first: no table may pass load 1/2 while the batch goes in
    if ((uint64_t)(fs.udp.tab.used + nu) * 2 > fs.udp.tab.ns() ||
        (uint64_t)(fs.tcp.tab.used + nt) * 2 > fs.tcp.tab.ns())
        fs.rebuild_all(next_seed, nu, nt);
    bool ok = true;
    for (uint32_t k = 0; k < nu; ++k) {
        const uint32_t id = fs.udp.alloc_id();
        rx_block &x = fs.udp.blk[id];
        udp_set(x, u[k]);
        x.seq = fs.udp.seq_next++;
        x.live = true;
        x.older = RXG_FLOW_NONE;
        ++fs.udp.live;
        ok &= udp_link(fs, id);
        udp_ids[k] = id;
    }
    for (uint32_t k = 0; k < nt; ++k) {
        const uint32_t id = fs.tcp.alloc_id();
        rx_block &x = fs.tcp.blk[id];
        tcp_set(x, t[k]);
        x.seq = fs.tcp.seq_next++;
        x.live = true;
        x.older = RXG_FLOW_NONE;
        ++fs.tcp.live;
        ok &= fs.tcp.link(id); // tcp_stream_create + LL_ADD (tcp.c:3-52)
        if (x.status == RXG_TCP_STATUS_LISTEN) fs.listen_add(id);
        tcp_ids[k] = id;
    }
    if (nu) fs.small_rebuild();
    after_change(c, ok);
    // 1: the count layout (rxg_num_udp_ids) grew
    return (fs.udp.id_space() != onu && ont + onu > 0 && fs.tcp.id_space() > 0) ? 1 : 0;
}

int rxg_flows_remove(rxg_ctx *c, const uint32_t *udp_ids, uint32_t nu, const uint32_t *tcp_ids,
                     uint32_t nt) {
    if (!c || (nu && !udp_ids) || (nt && !tcp_ids)) return RXG_EINVAL;
    rx_flowset &fs = c->fs;
    for (uint32_t k = 0; k < nu; ++k)
        if (udp_ids[k] >= fs.udp.id_space() || !fs.udp.blk[udp_ids[k]].live) return RXG_EINVAL;
    for (uint32_t k = 0; k < nt; ++k)
        if (tcp_ids[k] >= fs.tcp.id_space() || !fs.tcp.blk[tcp_ids[k]].live) return RXG_EINVAL;
    for (uint32_t k = 0; k < nu; ++k) {
        const uint32_t id = udp_ids[k];
        if (!fs.udp.blk[id].live) continue; // (listed twice)
        udp_unlink(fs, id);
        fs.udp.blk[id].live = false;
        --fs.udp.live;
        fs.udp.free_ids.push_back(id);
        if (c->device != RXG_HOST_ONLY) c->czero_udp.push_back(id);
    }
    for (uint32_t k = 0; k < nt; ++k) {
        const uint32_t id = tcp_ids[k];
        rx_block &x = fs.tcp.blk[id];
        if (!x.live) continue;
        if (x.status == RXG_TCP_STATUS_LISTEN) fs.listen_del(id);
        fs.tcp.unlink(id); // LL_REMOVE (tcp.c:321, common.c:620,660)
        x.live = false;
        --fs.tcp.live;
        fs.tcp.free_ids.push_back(id);
        if (c->device != RXG_HOST_ONLY) c->czero_tcp.push_back(id);
    }
    if (nu) fs.small_rebuild();
    after_change(c, true);
    return RXG_OK;
}

int rxg_flows_update_udp(rxg_ctx *c, uint32_t id, const rxg_udp_sock *u) {
    if (!c || !u) return RXG_EINVAL;
    rx_flowset &fs = c->fs;
    if (id >= fs.udp.id_space() || !fs.udp.blk[id].live) return RXG_EINVAL;
    udp_unlink(fs, id);
    udp_set(fs.udp.blk[id], *u); // nbind (common.c:350-353): same list position
    const bool ok = udp_link(fs, id);
    fs.small_rebuild();
    after_change(c, ok);
    return RXG_OK;
}

int rxg_flows_update_tcb(rxg_ctx *c, uint32_t id, const rxg_tcb *t) {
    if (!c || !t) return RXG_EINVAL;
    rx_flowset &fs = c->fs;
    if (id >= fs.tcp.id_space() || !fs.tcp.blk[id].live) return RXG_EINVAL;
    rx_block &x = fs.tcp.blk[id];
    const bool was_listen = x.status == RXG_TCP_STATUS_LISTEN;
    const uint32_t c2 = (uint32_t)t->sport | ((uint32_t)t->dport << 16);
    const bool rekey = x.a != t->sip || x.b != t->dip || x.c != c2;
    const bool is_listen = t->status == RXG_TCP_STATUS_LISTEN;
    if (!rekey && was_listen == is_listen) { // a state change the tables do not see
        x.status = t->status;
        return RXG_OK;
    }
    if (was_listen) fs.listen_del(id);
    bool ok = true;
    if (rekey) {
        fs.tcp.unlink(id);
        tcp_set(x, *t); // nbind / nlisten (common.c:358-386): same list position
        ok = fs.tcp.link(id);
    } else {
        x.status = t->status;
    }
    if (is_listen) fs.listen_add(id);
    after_change(c, ok);
    return RXG_OK;
}

int rxg_flows_commit(rxg_ctx *c, void *stream) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) {
        c->dirty = false;
        return RXG_OK;
    }
    DEVGUARD(c);
    const hipStream_t s = (hipStream_t)stream;
    return burst_begin(c, s); // commits on s and tracks s
}

uint32_t rxg_num_udp_ids(const rxg_ctx *c) { return c ? c->fs.udp.id_space() : 0; }

uint32_t rxg_flows_rebuilds(const rxg_ctx *c) { return c ? c->fs.rebuilds : 0; }

int rxg_tune(rxg_ctx *c, uint32_t lanes_per_frame, uint32_t passes, uint32_t frames_per_group,
             uint32_t pipeline) {
    if (!c) return RXG_EINVAL;
    if (lanes_per_frame == 0 && pipeline != ~0u) {
        // size-class binned path (20) / stream kernel variants: anything else
        // would silently run the automatic choice (r02o measured "ablations"
        // that were the default kernel), so it is refused
        if (!rx_variant_exists(0, 0, 0, pipeline)) return RXG_EINVAL;
        c->tune_g = 0;
        c->tune_p = c->tune_fpg = 0;
        c->tune_pipe = pipeline;
        return RXG_OK;
    }
    if (lanes_per_frame && (lanes_per_frame == 2 || lanes_per_frame > 64 ||
                            (lanes_per_frame & (lanes_per_frame - 1))))
        return RXG_EINVAL;
    // a combination that is not compiled in (in the product library: every
    // tuning shape and ablation of the RX_DIAG build) is refused here, not at
    // the next burst
    if (lanes_per_frame && !rx_variant_exists(lanes_per_frame, passes, frames_per_group, pipeline))
        return RXG_EINVAL;
    c->tune_g = lanes_per_frame;
    c->tune_p = lanes_per_frame ? passes : 0;
    c->tune_fpg = lanes_per_frame ? frames_per_group : 0;
    c->tune_pipe = lanes_per_frame ? pipeline : ~0u;
    return RXG_OK;
}

int rxg_register_host(rxg_ctx *c, void *base, uint64_t bytes) {
    if (!c || !base || !bytes) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    DEVGUARD(c);
    rxg_ctx::host_region r;
    r.h = static_cast<uint8_t *>(base);
    r.bytes = bytes;
    hipError_t e = hipHostRegister(base, bytes, hipHostRegisterMapped);
    if (e == hipErrorHostMemoryAlreadyRegistered) {
        (void)hipGetLastError();
    } else {
        HIPCHK(e);
        r.ours = true;
    }
    void *d = nullptr;
    e = hipHostGetDevicePointer(&d, base, 0);
    if (e != hipSuccess) {
        if (r.ours) (void)hipHostUnregister(base);
        return rx_set_hip_error(e);
    }
    r.d = static_cast<uint8_t *>(d);
    c->regions.push_back(r);
    return RXG_OK;
}

int rxg_unregister_host(rxg_ctx *c, void *base) {
    if (!c || !base) return RXG_EINVAL;
    for (size_t k = 0; k < c->regions.size(); ++k)
        if (c->regions[k].h == base) {
            DEVGUARD(c);
            int rc = bursts_drain(c); // no burst may still be pulling from it
            if (rc) return rc;
            if (c->regions[k].ours) HIPCHK(hipHostUnregister(base));
            c->regions.erase(c->regions.begin() + (long)k);
            c->region_hint = 0;
            return RXG_OK;
        }
    return RXG_EINVAL;
}

int rxg_kernel_variant(const rxg_ctx *c, uint32_t len_hint, uint32_t variant[4], char *name,
                       uint32_t name_cap) {
    if (!c) return RXG_EINVAL;
    uint32_t g = c->tune_g, p = c->tune_p, fpg = c->tune_fpg, pipe = c->tune_pipe;
    if (!g && pipe == ~0u) rx_pick_variant(len_hint, &g, &p, &fpg, &pipe); // as classify_dev_impl
    if (variant) variant[0] = g, variant[1] = p, variant[2] = fpg, variant[3] = pipe;
    if (name && name_cap) {
        strncpy(name, rx_variant_kernel(g, pipe), name_cap - 1);
        name[name_cap - 1] = '\0';
    }
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
    if (!c || (flags & ~(uint32_t)(RXG_TT_NO_UDP_PORT | RXG_TT_COUNT_4B | RXG_TT_COUNT_2BUF |
                                   RXG_TT_SLAB_HALF | RXG_TT_SLAB_QUARTER)))
        return RXG_EINVAL;
    c->tune_tables = flags;
    c->ft.count_4b = (flags & RXG_TT_COUNT_4B) ? 1u : 0u;
    c->ft.slab_div_log2 = (flags & RXG_TT_SLAB_QUARTER) ? 2u : (flags & RXG_TT_SLAB_HALF) ? 1u : 0u;
    c->ws_nbuf = (flags & RXG_TT_COUNT_2BUF) ? 2u : 3u;
    return RXG_OK;
}

int rxg_tune_deliver(rxg_ctx *c, uint32_t flags) {
    if (!c || (flags & ~RXG_DLV_TCP_IN_PLACE)) return RXG_EINVAL;
    c->deliver_flags = flags;
    return RXG_OK;
}

int rxg_tune_ingest(rxg_ctx *c, uint32_t mode) {
    if (!c || mode > RXG_INGEST_GATHER) return RXG_EINVAL;
    c->tune_ingest = mode;
    return RXG_OK;
}

int rxg_tune_flow_load(rxg_ctx *c, uint32_t load_log2) {
    if (!c || load_log2 > 4) return RXG_EINVAL;
    c->fs.load_log2 = load_log2 ? load_log2 : RX_FT_LOAD_LOG2;
    return RXG_OK;
}

// the count layout of the next burst (pending changes included)
uint32_t rxg_num_flows(const rxg_ctx *c) {
    return c ? c->fs.udp.id_space() + c->fs.tcp.id_space() : 0;
}

// diagnostics: the device image of a flow table next to the host one
int rxg_ft_dump(rxg_ctx *c, uint32_t which, int device_copy, void *dst, uint64_t bytes,
                uint32_t info[8]) {
    if (!c || (!dst && bytes)) return RXG_EINVAL;
    const rx_flowset &fs = c->fs;
    const void *h = nullptr;
    const void *d = nullptr;
    uint64_t n = 0;
    if (which == 0) h = fs.udp.tab.slots.data(), d = c->d_udp, n = fs.udp.tab.slots.size() * 16ull;
    else if (which == 1) h = fs.tcp.tab.slots.data(), d = c->d_tcp, n = fs.tcp.tab.slots.size() * 16ull;
    else if (which == 2) h = fs.listen.data(), d = c->d_listen, n = 65536 * 4ull;
    else if (which == 3) h = fs.udpc.data(), d = c->d_udpc, n = fs.udpc.size() * 8ull;
    else if (which == 4) h = fs.udpw.data(), d = c->d_udpw, n = fs.udpw.size() * 2ull;
    else return RXG_EINVAL;
    if (info && which >= 3) {
        info[0] = fs.udpc.empty() ? 0u : (uint32_t)fs.udpc.size() - 1, info[1] = fs.udpc_probe;
        info[2] = fs.seed, info[3] = fs.udpc_other, info[4] = fs.udpw_lo;
        info[5] = (uint32_t)fs.udpw.size(), info[6] = fs.udp_dip;
        info[7] = which == 3 ? (uint32_t)fs.udpc.size() : (uint32_t)fs.udpw.size();
    } else if (info) {
        info[0] = c->ft.tcp_mask, info[1] = c->ft.tcp_probe, info[2] = c->ft.hseed;
        info[3] = fs.tcp.tab.mask, info[4] = fs.tcp.tab.probe, info[5] = fs.seed;
        info[6] = c->dirty ? 1u : 0u, info[7] = (uint32_t)(n / 16);
    }
    n = std::min(n, bytes);
    if (n == 0) return RXG_OK;
    if (!device_copy || c->device == RXG_HOST_ONLY) {
        memcpy(dst, h, n);
        return RXG_OK;
    }
    DEVGUARD(c);
    int rc = bursts_drain(c);
    if (rc) return rc;
    HIPCHK(hipMemcpy(dst, d, n, hipMemcpyDeviceToHost));
    return RXG_OK;
}

uint32_t rxg_ft_lookup_udp(const rxg_ctx *c, uint32_t dip, uint16_t dport) {
    if (!c) return RXG_FLOW_NONE;
    const rx_flowset &fs = c->fs;
    uint32_t f;
    if (!fs.port.empty() && rx_udp_port_decide(fs.port[dport], dip, fs.udp_dip, &f)) return f;
    return fs.udp.tab.lookup(dip, dport, 17u);
}

uint32_t rxg_ft_lookup_tcp(const rxg_ctx *c, uint32_t sip, uint32_t dip, uint16_t sport,
                           uint16_t dport) {
    if (!c) return RXG_FLOW_NONE;
    const rx_flowset &fs = c->fs;
    uint32_t f = fs.tcp.tab.lookup(sip, dip, (uint32_t)sport | ((uint32_t)dport << 16));
    if (f == RXG_FLOW_NONE) f = fs.listen[dport];
    return f;
}

uint32_t rxg_rss_hash(uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport) {
    return rx_rss_hash(sip, dip, sport, dport);
}

// workspace regions (rxg_ctx::wu)
enum { WS_BUF0 = 0, WS_BUF1 = 1, WS_BUF2 = 2, WS_SLAB = 3 };

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
        // every use of the old workspace has finished (its events): it is freed
        // and the grown one allocated in stream order on s, without the
        // device-wide synchronisation of hipFree
        for (rxg_ctx::ws_use &u : c->wu)
            if (u.used) HIPCHK(hipEventSynchronize(u.ev));
        int rc = ensure_dev_async((void **)&c->d_ws, &c->d_ws_cap, ws, s);
        if (rc) return rc;
    } else if (layout != c->ws_layout) {
        for (int r = 0; r < 4; ++r) HIPCHK(ws_wait(c, r, s));
    }
    c->ws_layout = layout;
    return RXG_OK;
}

// one burst on the workspace: classify + count on s (count_stream null or s),
// or classify on s and the slab count on count_stream (double-buffered indices)
static int classify_ws_body(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                       const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t g,
                       uint32_t p, uint32_t fpg, uint32_t pipe, uint4 *d_out,
                       unsigned long long *d_counts, hipStream_t s, hipStream_t cs) {
    // three index buffers: burst k's classify writes buffer k % 3, which the
    // count of burst k - 3 read (long done), so it never waits for the count
    // of burst k - 2, whose slab blocks (a whole CU each) can only start once
    // burst k - 1's classify drains.  With two, every step waited for that
    // count (+2.5% per step at cfg4, rocprofv3 trace, profiles/r05b)
    const uint32_t nb = c->ws_nbuf;
    const size_t ws = rx_classify_ws_bytes(n, g, pipe, c->ft, d_counts != nullptr, nb);
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
    c->ft.bpc_cap = c->tune_bpc; // (read by this burst's launches only: they copy c->ft)
    // the verdict format of this burst (rxg_classify_dev8: c->ft.v8)
    const auto k1 = c->ft.v8 ? rx_classify_launch8 : rx_classify_launch;
    if (!ws) {
        HIPCHK(k1(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                                  d_out, d_counts, s, c->d_ws, RX_PH_ALL, 0, nb));
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
        HIPCHK(k1(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                                  d_out, d_counts, s, c->d_ws, RX_PH_ALL, 0, nb));
        HIPCHK(ws_mark(c, WS_BUF0, s));
        HIPCHK(ws_mark(c, WS_SLAB, s));
        return join_cs();
    }
    const uint32_t b = c->ws_flip % nb;
    c->ws_flip = (b + 1u) % nb;
    HIPCHK(ws_wait(c, b, s)); // the count that last read this index buffer
    HIPCHK(k1(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                              d_out, d_counts, s, c->d_ws, RX_PH_CLASSIFY, b, nb));
    HIPCHK(hipEventRecord(c->ev_k1, s));
    HIPCHK(hipStreamWaitEvent(cs, c->ev_k1, 0));
    HIPCHK(ws_wait(c, WS_SLAB, cs));
    HIPCHK(k1(d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, c->ft,
                              d_out, d_counts, cs, c->d_ws, RX_PH_COUNT, b, nb));
    HIPCHK(ws_mark(c, b, cs)); // covers the classify too (cs waited on it)
    HIPCHK(ws_mark(c, WS_SLAB, cs));
    return RXG_OK;
}

// a burst: pending flow-table changes first (stream-ordered on s), the
// stream tracked for later table writes, then the launches
static int classify_ws(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                       const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t g,
                       uint32_t p, uint32_t fpg, uint32_t pipe, uint4 *d_out,
                       unsigned long long *d_counts, hipStream_t s, hipStream_t cs) {
    // the context's own counts move when the commit burst_begin makes grows
    // the id space (counts_layout frees the old vector, stream-ordered, and
    // the same commit may allocate a table in its place): take the pointer
    // after the commit, never before
    const bool own = d_counts != nullptr && d_counts == c->d_counts;
    int rc = burst_begin(c, s);
    if (rc) return rc;
    if (own) d_counts = c->d_counts;
    return classify_ws_body(c, d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe, d_out,
                            d_counts, s, cs);
}

static int classify_dev_impl(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                             const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                             uint32_t len_hint, void *d_out, uint64_t *d_counts, hipStream_t s,
                             hipStream_t cs, uint32_t v8 = 0) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len || !d_out) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    DEVGUARD(c);
    uint32_t g = c->tune_g, p = c->tune_p, fpg = c->tune_fpg, pipe = c->tune_pipe;
    if (!g && pipe == ~0u) rx_pick_variant(len_hint, &g, &p, &fpg, &pipe, v8 != 0);
    c->ft.v8 = v8; // read by this burst's launches only (they copy c->ft)
    const int rc = classify_ws(c, d_pkts, d_off, d_len, n, off_unit_log2, g, p, fpg, pipe,
                               static_cast<uint4 *>(d_out),
                               reinterpret_cast<unsigned long long *>(d_counts), s, cs);
    c->ft.v8 = 0;
    return rc;
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

int rxg_classify_dev8(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                      const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t len_hint,
                      rxg_verdict8 *d_out, uint64_t *d_counts, void *stream, void *count_stream) {
    static_assert(sizeof(rxg_verdict8) == 8, "rxg_verdict8 is 8 bytes");
    if (d_out && (reinterpret_cast<uintptr_t>(d_out) & 7u)) return RXG_EINVAL;
    return classify_dev_impl(c, d_pkts, d_off, d_len, n, off_unit_log2, len_hint, d_out,
                             d_counts, (hipStream_t)stream, (hipStream_t)count_stream, 1u);
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
                       uint32_t off_unit_log2, rxg_verdict *out, uint64_t ticket,
                       bool pulled = false) {
    const bool reused = sl.ticket != 0;
    if (reused) HIPCHK(hipStreamWaitEvent(c->s_h2d, sl.ev_k, 0));
    if (!pulled) HIPCHK(copy_in_frames(c, sl, pkts, span));
    HIPCHK(hipMemcpyAsync(sl.d_off, off, n * 4ull, hipMemcpyHostToDevice, c->s_h2d));
    HIPCHK(hipMemcpyAsync(sl.d_len, len, n * 2ull, hipMemcpyHostToDevice, c->s_h2d));
    if (pulled) { // registered host frames: the device pulls them into the slot
        HIPCHK(hipMemcpyAsync(sl.d_src, sl.h_src, n * 8ull, hipMemcpyHostToDevice, c->s_h2d));
        HIPCHK(rx_ingest_launch(sl.d_src, sl.d_off, sl.d_len, n, sl.d_pkts, c->s_h2d));
    }
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
    DEVGUARD(c);
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
    DEVGUARD(c);
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

// frames of an mbuf burst into slot sl's pinned staging at 64-B aligned
// places (buf_addr + data_off, data_len bytes); *span = bytes used
// the device address of [p, p + bytes) when it lies in a registered region
static uint8_t *region_dev(rxg_ctx *c, const uint8_t *p, uint64_t bytes) {
    const uint32_t nr = (uint32_t)c->regions.size();
    for (uint32_t k = 0; k < nr; ++k) {
        const uint32_t j = (c->region_hint + k) % nr;
        const rxg_ctx::host_region &r = c->regions[j];
        if (p >= r.h && p + bytes <= r.h + r.bytes) {
            c->region_hint = j;
            return r.d + (p - r.h);
        }
    }
    return nullptr;
}

// how an mbuf burst reaches a staging slot
struct staged {
    const uint8_t *src = nullptr; // host bytes copied in by DMA (the pinned gather, or a
                                  // registered span); nullptr when the device pulls
    uint64_t span = 0;            // bytes of the slot used
    uint64_t bound = 0;           // bounds the 16-B padded payloads of the burst (results' copy out)
    uint32_t ul = 6;              // descriptor unit (log2 bytes)
    bool pulled = false;          // the device pulls each frame (rx_ingest_launch)
};

// an mbuf burst whose frames all lie in registered host memory, 16-B aligned:
// descriptors only.  Dense in one region (the covering span at most 1.4x the
// frames' 16-B rounded bytes, and it fits the slot): one DMA copy of the span,
// descriptors in 16-B units from its start (the copy engine moves ~55 GB/s,
// device loads of host memory ~38); else the device pulls frame by frame
// (device source addresses).  st->src / pulled unset: the host gather takes it.
static int pull_mbufs(rxg_ctx *c, rxg_ctx::slot &sl, rxg_mbuf *const *m, uint32_t n, staged *st) {
    if (c->regions.empty() || c->tune_ingest == RXG_INGEST_GATHER || n == 0) return RXG_OK;
    if (!sl.h_src) {
        HIPCHK(hipMalloc(&sl.d_src, (size_t)c->max_pkts * 8));
        HIPCHK(hipHostMalloc((void **)&sl.h_src, (size_t)c->max_pkts * 8, 0));
    }
    if (sl.ticket) HIPCHK(hipEventSynchronize(sl.ev_in)); // the slot's last copy-in read h_*
    // one pass over the mbufs: each frame's device address (h_src) and
    // length, the covering span, and whether all frames share one 64-B phase
    uintptr_t lo = UINTPTR_MAX, hi = 0, phase = 0;
    const uintptr_t ph0 = m[0] ? ((uintptr_t)m[0]->buf_addr + m[0]->data_off) & 63u : 0;
    uint64_t dense = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!m[i] || !m[i]->buf_addr) return RXG_EINVAL;
        const uintptr_t f = (uintptr_t)m[i]->buf_addr + m[i]->data_off;
        const uint32_t l = m[i]->data_len;
        const uint64_t l16 = (l + 15ull) & ~15ull;
        uint8_t *d = (f & 15u) ? nullptr : region_dev(c, (const uint8_t *)f, l16);
        if (!d) return RXG_OK; // (the host gather takes the burst)
        sl.h_src[i] = (unsigned long long)(uintptr_t)d;
        sl.h_len[i] = (uint16_t)l;
        lo = std::min(lo, f);
        hi = std::max<uintptr_t>(hi, f + l16);
        phase |= (f & 63u) ^ ph0;
        dense += l16;
    }
    const uint64_t span = hi - lo;
    uint8_t *dlo = region_dev(c, (const uint8_t *)lo, 16);
    if (c->tune_ingest != RXG_INGEST_PULL && span <= c->max_bytes && span <= dense + dense / 5 * 2 &&
        span >> 4 <= 0xFFFFFFFFull && region_dev(c, (const uint8_t *)lo, span)) {
        // one span: 64-B units when every frame sits on a 64-B boundary from
        // its start (mbuf data rooms usually do), else 16-B units; offsets
        // from the device addresses (the same region, so the same distances)
        const uint32_t ul = phase ? 4u : 6u;
        const uintptr_t dbase = (uintptr_t)dlo;
        for (uint32_t i = 0; i < n; ++i) sl.h_off[i] = (uint32_t)(((uintptr_t)sl.h_src[i] - dbase) >> ul);
        st->src = (const uint8_t *)lo;
        st->span = span;
        st->bound = std::min<uint64_t>(std::max(span, dense), c->max_bytes); // (frames may overlap)
        st->ul = ul;
        return RXG_OK;
    }
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t step = std::max<uint64_t>((sl.h_len[i] + 63ull) & ~63ull, 64);
        if (pos + step > c->max_bytes) return RXG_ERANGE;
        sl.h_off[i] = (uint32_t)(pos >> 6);
        pos += step;
    }
    st->span = st->bound = pos;
    st->ul = 6;
    st->pulled = true;
    return RXG_OK;
}

static int gather_mbufs(rxg_ctx *c, rxg_ctx::slot &sl, rxg_mbuf *const *m, uint32_t n, staged *st,
                        bool registered) {
    *st = staged();
    if (registered) {
        int rc = pull_mbufs(c, sl, m, n, st);
        if (rc || st->pulled || st->src) return rc;
    }
    if (sl.ticket) HIPCHK(hipEventSynchronize(sl.ev_in)); // the slot's last copy-in read h_stage
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
    st->src = sl.h_stage;
    st->span = st->bound = pos;
    st->ul = 6;
    return RXG_OK;
}

int rxg_process_mbufs(rxg_ctx *c, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!m || !out) return RXG_EINVAL;
    if (n > c->max_pkts || !c->slots[0].h_stage) return RXG_ERANGE;
    DEVGUARD(c);
    const uint64_t t = c->next_ticket++;
    rxg_ctx::slot &sl = c->slots[t % RXG_PIPE_DEPTH];
    staged st;
    int rc = gather_mbufs(c, sl, m, n, &st, true);
    if (rc) return rc;
    rc = submit_slot(c, sl, st.src, st.span, sl.h_off, sl.h_len, n, st.ul, out, t, st.pulled);
    return rc ? rc : rxg_wait(c, t);
}

static int compact_impl(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        const uint4 *d_v, rxg_dgram *d_dg, uint32_t *d_first, uint8_t *d_payload,
                        uint64_t cap, uint32_t *d_totals, hipStream_t s) {
    const uint32_t nf = c->fs.udp.id_space();
    if (nf == 0 || nf > RXG_COMPACT_MAX_FLOWS) return nf ? RXG_ERANGE : RXG_OK;
    const size_t ws = rx_compact_ws_bytes(n, nf);
    if (ws > c->d_cp_ws_cap) { // (its uses are all on s: freed and grown in stream order)
        int rc = ensure_dev_async(&c->d_cp_ws, &c->d_cp_ws_cap, ws, s);
        if (rc) return rc;
    }
    HIPCHK(rx_compact_launch(d_pkts, d_off, d_len, n, off_unit_log2, d_v, nf, d_dg, d_first,
                             d_payload, cap, d_totals, c->d_cp_ws, s));
    return RXG_OK;
}

int rxg_udp_compact_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        const rxg_verdict *d_v, rxg_dgram *d_dgram, uint32_t *d_first,
                        uint8_t *d_payload, uint64_t payload_cap, uint32_t *d_totals, void *stream) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (!d_first || !d_totals || (n && (!d_pkts || !d_off || !d_len || !d_v || !d_dgram ||
                                        !d_payload)))
        return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    DEVGUARD(c);
    if (c->fs.udp.id_space() > RXG_COMPACT_MAX_FLOWS) return RXG_ERANGE;
    return compact_impl(c, d_pkts, d_off, d_len, n, off_unit_log2,
                        reinterpret_cast<const uint4 *>(d_v), d_dgram, d_first, d_payload,
                        payload_cap, d_totals, (hipStream_t)stream);
}

int rxg_process_mbufs_udp(rxg_ctx *c, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out,
                          const rxg_dgram **dgram, const uint32_t **first, const uint8_t **payload,
                          uint32_t *ndgram, uint64_t *nbytes) {
    if (!c || !dgram || !first || !payload || !ndgram || !nbytes) return RXG_EINVAL;
    *ndgram = 0;
    *nbytes = 0;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n && (!m || !out)) return RXG_EINVAL;
    if (n > c->max_pkts || !c->slots[0].h_stage) return RXG_ERANGE;
    const uint32_t nf = c->fs.udp.id_space();
    if (nf > RXG_COMPACT_MAX_FLOWS) return RXG_ERANGE;
    DEVGUARD(c);
    if (!c->h_cp_totals) { // first use: results sized for a full staging slot
        // (h_cp_totals is set last: a failed allocation leaves the set
        // incomplete and the next call retries the missing pieces)
        if (!c->d_cp_dg) HIPCHK(hipMalloc(&c->d_cp_dg, (size_t)c->max_pkts * sizeof(rxg_dgram)));
        if (!c->d_cp_first)
            HIPCHK(hipMalloc(&c->d_cp_first, (RXG_COMPACT_MAX_FLOWS + 1) * sizeof(uint32_t)));
        if (!c->d_cp_payload) HIPCHK(hipMalloc(&c->d_cp_payload, c->max_bytes));
        if (!c->d_cp_totals) HIPCHK(hipMalloc(&c->d_cp_totals, 4 * sizeof(uint32_t)));
        if (!c->h_cp_dg)
            HIPCHK(hipHostMalloc((void **)&c->h_cp_dg, (size_t)c->max_pkts * sizeof(rxg_dgram), 0));
        if (!c->h_cp_first)
            HIPCHK(hipHostMalloc((void **)&c->h_cp_first,
                                 (RXG_COMPACT_MAX_FLOWS + 1) * sizeof(uint32_t), 0));
        if (!c->h_cp_payload) HIPCHK(hipHostMalloc((void **)&c->h_cp_payload, c->max_bytes, 0));
        HIPCHK(hipHostMalloc((void **)&c->h_cp_totals, 4 * sizeof(uint32_t), 0));
    }
    *dgram = c->h_cp_dg;
    *first = c->h_cp_first;
    *payload = c->h_cp_payload;
    memset(c->h_cp_first, 0, (nf + 1) * sizeof(uint32_t));
    if (n == 0) return RXG_OK;
    const uint64_t t = c->next_ticket++;
    rxg_ctx::slot &sl = c->slots[t % RXG_PIPE_DEPTH];
    staged st;
    int rc = gather_mbufs(c, sl, m, n, &st, true);
    if (rc) return rc;
    rc = submit_slot(c, sl, st.src, st.span, sl.h_off, sl.h_len, n, st.ul, out, t, st.pulled);
    if (rc) return rc;
    // the compaction follows the classify on the context's stream (its inputs:
    // the staged frames and the device verdicts of this slot)
    rc = compact_impl(c, sl.d_pkts, sl.d_off, sl.d_len, n, st.ul, sl.d_out, c->d_cp_dg, c->d_cp_first,
                      c->d_cp_payload, c->max_bytes, c->d_cp_totals, c->stream);
    if (rc) return rc;
    if (nf) {
        HIPCHK(hipMemcpyAsync(c->h_cp_totals, c->d_cp_totals, 3 * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->h_cp_totals[2]) return RXG_ERANGE; // (not reached: staging bounds the payloads)
        *ndgram = c->h_cp_totals[0];
        *nbytes = c->h_cp_totals[1];
        HIPCHK(hipMemcpyAsync(c->h_cp_first, c->d_cp_first, (nf + 1) * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, c->stream));
        if (*ndgram)
            HIPCHK(hipMemcpyAsync(c->h_cp_dg, c->d_cp_dg, (size_t)*ndgram * sizeof(rxg_dgram),
                                  hipMemcpyDeviceToHost, c->stream));
        if (*nbytes)
            HIPCHK(hipMemcpyAsync(c->h_cp_payload, c->d_cp_payload, *nbytes, hipMemcpyDeviceToHost,
                                  c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return rxg_wait(c, t);
}

static int segsort_impl(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, const uint4 *d_v,
                        rxg_segment *d_seg, uint8_t *d_payload, uint64_t cap, uint32_t *d_totals,
                        hipStream_t s) {
    const size_t ws = rx_segsort_ws_bytes(n);
    if (ws > c->d_ss_ws_cap) { // (its uses are all on s: freed and grown in stream order)
        int rc = ensure_dev_async(&c->d_ss_ws, &c->d_ss_ws_cap, ws, s);
        if (rc) return rc;
    }
    HIPCHK(rx_segsort_launch(d_pkts, d_off, d_len, n, off_unit_log2, d_v, c->fs.tcp.id_space(), d_seg,
                             d_payload, cap, d_totals, c->d_ss_ws, s));
    return RXG_OK;
}

int rxg_payload_hold(rxg_ctx *c, int32_t ref) {
    if (!c || ref < 0 || ref >= RXG_PAYLOAD_BUFS) return RXG_EINVAL;
    c->pl[ref].refs.fetch_add(1, std::memory_order_acq_rel);
    return RXG_OK;
}

int rxg_payload_release(rxg_ctx *c, int32_t ref) {
    if (!c || ref < 0 || ref >= RXG_PAYLOAD_BUFS) return RXG_EINVAL;
    c->pl[ref].refs.fetch_sub(1, std::memory_order_acq_rel);
    return RXG_OK;
}

int rxg_tcp_compact_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                        const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2,
                        const rxg_verdict *d_v, rxg_segment *d_seg, uint8_t *d_payload,
                        uint64_t payload_cap, uint32_t *d_totals, void *stream) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (!d_totals || (n && (!d_pkts || !d_off || !d_len || !d_v || !d_seg)))
        return RXG_EINVAL; // (d_payload null: records only, RXG_DLV_TCP_IN_PLACE)
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    DEVGUARD(c);
    return segsort_impl(c, d_pkts, d_off, d_len, n, off_unit_log2, reinterpret_cast<const uint4 *>(d_v),
                        d_seg, d_payload, payload_cap, d_totals, (hipStream_t)stream);
}

static double now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

int rxg_deliver_submit(rxg_ctx *c, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out,
                       rxg_delivery *d) {
    if (!c || !d) return RXG_EINVAL;
    memset(d, 0, sizeof(*d));
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n && (!m || !out)) return RXG_EINVAL;
    if (n > c->max_pkts || !c->slots[0].h_stage) return RXG_ERANGE;
    // the next set in turn, which must have been waited for
    const uint32_t si = c->dl_next;
    rxg_ctx::delivery_set &ds = c->dls[si];
    if (ds.on) return RXG_EINVAL; // (RXG_DELIVER_DEPTH bursts in flight already)
    const uint32_t nf = c->fs.udp.id_space();
    const bool udp = nf > 0 && nf <= RXG_COMPACT_MAX_FLOWS;
    DEVGUARD(c);
    const double t0 = now_ms();
    // results buffers, first use (each set last-allocated-first-checked: a
    // failed allocation leaves the rest for the next call to retry)
    if (udp && !ds.h_cp_totals) {
        if (!c->d_cp_dg) HIPCHK(hipMalloc(&c->d_cp_dg, (size_t)c->max_pkts * sizeof(rxg_dgram)));
        if (!c->d_cp_first)
            HIPCHK(hipMalloc(&c->d_cp_first, (RXG_COMPACT_MAX_FLOWS + 1) * sizeof(uint32_t)));
        if (!c->d_cp_payload) HIPCHK(hipMalloc(&c->d_cp_payload, c->max_bytes));
        if (!c->d_cp_totals) HIPCHK(hipMalloc(&c->d_cp_totals, 4 * sizeof(uint32_t)));
        if (!ds.h_cp_dg)
            HIPCHK(hipHostMalloc((void **)&ds.h_cp_dg, (size_t)c->max_pkts * sizeof(rxg_dgram), 0));
        if (!ds.h_cp_first)
            HIPCHK(hipHostMalloc((void **)&ds.h_cp_first, (RXG_COMPACT_MAX_FLOWS + 1) * sizeof(uint32_t), 0));
        if (!ds.h_cp_payload) HIPCHK(hipHostMalloc((void **)&ds.h_cp_payload, c->max_bytes, 0));
        HIPCHK(hipHostMalloc((void **)&ds.h_cp_totals, 4 * sizeof(uint32_t), 0));
    }
    if (!ds.h_ss_totals) {
        if (!c->d_ss_seg) HIPCHK(hipMalloc(&c->d_ss_seg, (size_t)c->max_pkts * sizeof(rxg_segment)));
        if (!c->d_ss_payload) HIPCHK(hipMalloc(&c->d_ss_payload, c->max_bytes));
        if (!c->d_ss_totals) HIPCHK(hipMalloc(&c->d_ss_totals, 4 * sizeof(uint32_t)));
        if (!ds.h_ss_seg)
            HIPCHK(hipHostMalloc((void **)&ds.h_ss_seg, (size_t)c->max_pkts * sizeof(rxg_segment), 0));
        HIPCHK(hipHostMalloc((void **)&ds.h_ss_totals, 4 * sizeof(uint32_t), 0));
    }
    for (hipEvent_t &e : ds.tev)
        if (!e) HIPCHK(hipEventCreate(&e));
    // the TCP payloads of this burst: a free pooled buffer (a hold the caller
    // can take, rxg_payload_hold), else the set's own one (valid until the
    // set is reused: tcp_payload_ref = -1).  The library's hold on the
    // buffer of this set's previous burst ends here.  In place
    // (RXG_DLV_TCP_IN_PLACE): no payload is gathered or copied back; the
    // payloads stay in the caller's frames.
    const bool inplace = (c->deliver_flags & RXG_DLV_TCP_IN_PLACE) != 0;
    if (ds.pl >= 0) c->pl[ds.pl].refs.fetch_sub(1, std::memory_order_acq_rel);
    ds.pl = -1;
    for (int k = 0; k < RXG_PAYLOAD_BUFS && ds.pl < 0 && !inplace; ++k) {
        rxg_ctx::pl_buf &b = c->pl[k];
        if (b.refs.load(std::memory_order_acquire) != 0) continue;
        if (!b.h && hipHostMalloc((void **)&b.h, c->max_bytes, 0) != hipSuccess) {
            b.h = nullptr; // (out of pinned memory: the set's own buffer)
            (void)hipGetLastError();
            break;
        }
        b.refs.store(1, std::memory_order_release);
        ds.pl = k;
    }
    if (ds.pl < 0 && !inplace && !ds.h_ss_payload)
        HIPCHK(hipHostMalloc((void **)&ds.h_ss_payload, c->max_bytes, 0));
    d->seg = ds.h_ss_seg;
    d->tcp_payload_ref = ds.pl;
    d->tcp_payload = inplace ? nullptr : ds.pl >= 0 ? c->pl[ds.pl].h : ds.h_ss_payload;
    d->set = si + 1;
    if (udp) {
        d->dgram = ds.h_cp_dg;
        d->first = ds.h_cp_first;
        d->udp_payload = ds.h_cp_payload;
        memset(ds.h_cp_first, 0, (nf + 1) * sizeof(uint32_t));
    }
    ds.on = ds.udp = ds.tcp = false;
    ds.ticket = 0;
    ds.t0 = t0;
    c->dl_next = (si + 1) % RXG_DELIVER_DEPTH;
    if (n == 0) return RXG_OK;
    const uint64_t t = c->next_ticket++;
    rxg_ctx::slot &sl = c->slots[t % RXG_PIPE_DEPTH];
    staged st;
    int rc = gather_mbufs(c, sl, m, n, &st, true);
    if (rc) return rc;
    const uint64_t pos = st.bound;
    const double t1 = now_ms();
    bool tcp = false;
    // every device step and copy of the burst; on an error after the first is
    // queued, the streams are drained so nothing still writes into the set
    auto enqueue = [&]() -> int {
        HIPCHK(hipEventRecord(ds.tev[0], c->s_h2d));
        rc = submit_slot(c, sl, st.src, st.span, sl.h_off, sl.h_len, n, st.ul, out, t, st.pulled);
        if (rc) return rc;
        HIPCHK(hipEventRecord(ds.tev[1], c->s_h2d)); // after the copy in
        HIPCHK(hipEventRecord(ds.tev[2], c->stream)); // after K1
        // the compactions follow the classify on the context's stream
        if (udp)
            if ((rc = compact_impl(c, sl.d_pkts, sl.d_off, sl.d_len, n, st.ul, sl.d_out, c->d_cp_dg,
                                   c->d_cp_first, c->d_cp_payload, c->max_bytes, c->d_cp_totals,
                                   c->stream)))
                return rc;
        tcp = c->fs.tcp.id_space() > 0;
        if (tcp)
            if ((rc = segsort_impl(c, sl.d_pkts, sl.d_off, sl.d_len, n, st.ul, sl.d_out, c->d_ss_seg,
                                   inplace ? nullptr : c->d_ss_payload, c->max_bytes,
                                   c->d_ss_totals, c->stream)))
                return rc;
        HIPCHK(hipEventRecord(ds.tev[3], c->stream)); // after K3 / K4
        // every result in one round trip: the counts with upper-bound copies of
        // the records (n of each) and payloads (the staged span bounds the sum of
        // the 16-B padded payloads), so no synchronisation sits between the
        // compactions and their copy out.  The next set's compactions reuse the
        // device buffers after these copies, in stream order.
        if (udp) {
            HIPCHK(hipMemcpyAsync(ds.h_cp_totals, c->d_cp_totals, 3 * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(ds.h_cp_first, c->d_cp_first, (nf + 1) * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(ds.h_cp_dg, c->d_cp_dg, (size_t)n * sizeof(rxg_dgram),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(ds.h_cp_payload, c->d_cp_payload, pos, hipMemcpyDeviceToHost,
                                  c->stream));
        }
        if (tcp) {
            HIPCHK(hipMemcpyAsync(ds.h_ss_totals, c->d_ss_totals, 3 * sizeof(uint32_t),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(ds.h_ss_seg, c->d_ss_seg, (size_t)n * sizeof(rxg_segment),
                                  hipMemcpyDeviceToHost, c->stream));
            if (!inplace)
                HIPCHK(hipMemcpyAsync(const_cast<uint8_t *>(d->tcp_payload), c->d_ss_payload, pos,
                                      hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(hipEventRecord(ds.tev[4], c->stream)); // after the results' copy out
        return RXG_OK;
    };
    if ((rc = enqueue())) {
        (void)hipStreamSynchronize(c->s_h2d);
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->s_d2h);
        return rc;
    }
    ds.on = true;
    ds.udp = udp;
    ds.tcp = tcp;
    ds.ticket = t;
    ds.t1 = t1;
    return RXG_OK;
}

// no field of the context's flow tables is read here: the control plane
// (rxg_flows_*) may run beside it, from another thread (rxgpu.h)
int rxg_deliver_wait(rxg_ctx *c, rxg_delivery *d, float ms[8]) {
    if (!c || !d) return RXG_EINVAL;
    if (ms) memset(ms, 0, 8 * sizeof(float));
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (d->set < 1 || d->set > RXG_DELIVER_DEPTH) return RXG_EINVAL;
    rxg_ctx::delivery_set &ds = c->dls[d->set - 1];
    if (!ds.on) return RXG_OK; // (an empty burst, or waited for already)
    ds.on = false;
    DEVGUARD(c);
    HIPCHK(hipEventSynchronize(ds.tev[4]));
    int rc = rxg_wait(c, ds.ticket); // (the verdicts' copy out, on s_d2h)
    if (rc) return rc;
    const bool udp = ds.udp, tcp = ds.tcp;
    if ((udp && ds.h_cp_totals[2]) || (tcp && ds.h_ss_totals[2]))
        return RXG_ERANGE; // (not reached: staging bounds the payloads)
    if (udp) d->ndgram = ds.h_cp_totals[0], d->udp_bytes = ds.h_cp_totals[1];
    if (tcp) d->nseg = ds.h_ss_totals[0], d->tcp_bytes = ds.h_ss_totals[1];
    if (ms) {
        ms[0] = (float)(ds.t1 - ds.t0);
        for (int k = 0; k < 4; ++k) HIPCHK(hipEventElapsedTime(&ms[k + 1], ds.tev[k], ds.tev[k + 1]));
        ms[5] = (float)(now_ms() - ds.t0);
    }
    return RXG_OK;
}

int rxg_process_mbufs_deliver(rxg_ctx *c, rxg_mbuf *const *m, uint32_t n, rxg_verdict *out,
                              rxg_delivery *d, float ms[8]) {
    int rc = rxg_deliver_submit(c, m, n, out, d);
    if (rc) {
        if (c && d && d->set) c->dls[d->set - 1].on = false;
        if (ms) memset(ms, 0, 8 * sizeof(float));
        return rc;
    }
    return rxg_deliver_wait(c, d, ms);
}

int rxg_tx_cksum_dev(rxg_ctx *c, uint8_t *d_pkts, const uint32_t *d_off, const uint16_t *d_len,
                     uint32_t n, uint32_t off_unit_log2, uint32_t len_hint, void *stream) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n == 0) return RXG_OK;
    if (!d_pkts || !d_off || !d_len) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    DEVGUARD(c);
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
    DEVGUARD(c);
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

// the split / gather workspace d_aux: a use on another stream than the last
// one waits for it (event), growth waits on the host for the last use only
static int aux_begin(rxg_ctx *c, size_t ws, hipStream_t s) {
    if (ws > c->d_aux_cap) {
        if (c->aux_used) HIPCHK(hipEventSynchronize(c->ev_aux));
        int rc = ensure_dev_async(&c->d_aux, &c->d_aux_cap, ws, s);
        if (rc) return rc;
    } else if (c->aux_used && c->aux_st != s) {
        HIPCHK(hipStreamWaitEvent(s, c->ev_aux, 0));
    }
    return RXG_OK;
}
static int aux_end(rxg_ctx *c, hipStream_t s) {
    HIPCHK(hipEventRecord(c->ev_aux, s));
    c->aux_st = s;
    c->aux_used = true;
    return RXG_OK;
}

int rxg_rss_split_dev(rxg_ctx *c, const uint8_t *d_pkts, const uint32_t *d_off,
                      const uint16_t *d_len, uint32_t n, uint32_t off_unit_log2, uint32_t n_shards,
                      uint32_t *d_first, uint32_t *d_perm, void *stream) {
    if (!c || !d_first || n_shards == 0 || n_shards > RXG_MAX_SHARDS) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    if (n && (!d_pkts || !d_off || !d_len || !d_perm)) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    DEVGUARD(c);
    const hipStream_t s = (hipStream_t)stream;
    const size_t ws = rx_split_ws_bytes(n, n_shards);
    int rc = aux_begin(c, ws, s);
    if (rc) return rc;
    HIPCHK(rx_split_launch(d_pkts, d_off, d_len, n, off_unit_log2, n_shards, d_first, d_perm,
                           c->d_aux, s));
    return aux_end(c, s);
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
    DEVGUARD(c);
    const hipStream_t s = (hipStream_t)stream;
    const size_t ws = rx_gather_ws_bytes(count);
    int rc = aux_begin(c, ws, s);
    if (rc) return rc;
    HIPCHK(rx_gather_launch(d_pkts, d_off, d_len, off_unit_log2, d_idx, count, d_dst, dst_cap,
                            d_dst_off, d_dst_len, c->d_aux, s));
    // the packed size (64-B units) sits after the per-chunk sums
    const size_t nchunks = (ws - 8) / 8;
    uint64_t units = 0;
    HIPCHK(hipMemcpyAsync(&units, reinterpret_cast<uint64_t *>(c->d_aux) + nchunks, 8,
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if ((rc = aux_end(c, s))) return rc;
    if (span) *span = units << 6;
    if ((units << 6) > dst_cap || units > 0xFFFFFFFFull) return RXG_ERANGE;
    return RXG_OK;
}

// the increment since the last call is all-reduced and folded into the
// running total, so repeated calls never multiply earlier traffic by the ranks
int rxg_ctx_counts_allreduce(rxg_ctx *c, rxg_group *g) {
    if (!c || !g) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    DEVGUARD(c);
    int rc = bursts_drain(c); // every burst counted; the counts' stream order
    if (rc) return rc;
    const uint32_t nf = c->ft.nu + c->ft.nt;
    if (!nf) return RXG_OK;
    rc = rx_group_allreduce_u64(g, c->d_counts, nf, c->stream);
    if (rc) return rc;
    hipLaunchKernelGGL(rx_counts_fold_kernel, dim3((nf + 255) / 256), dim3(256), 0, c->stream,
                       c->d_counts_base, c->d_counts, nf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RXG_OK;
}

int rxg_flow_counts(rxg_ctx *c, uint64_t *counts, uint32_t ncounts) {
    if (!c || (ncounts && !counts)) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    const uint32_t nf = c->ft.nu + c->ft.nt;
    if (ncounts < nf) return RXG_ERANGE;
    DEVGUARD(c);
    int rc = bursts_drain(c); // every submitted burst's kernel has counted
    if (rc) return rc;
    if (!nf) return RXG_OK;
    std::vector<uint64_t> base(nf);
    HIPCHK(hipMemcpy(counts, c->d_counts, nf * 8ull, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(base.data(), c->d_counts_base, nf * 8ull, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < nf; ++i) counts[i] += base[i];
    return RXG_OK;
}

int rxg_counts_reset(rxg_ctx *c) {
    if (!c) return RXG_EINVAL;
    if (c->device == RXG_HOST_ONLY) return RXG_ENODEV;
    DEVGUARD(c);
    int rc = bursts_drain(c);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(c->d_counts, 0, (size_t)c->counts_cap * 8, c->stream));
    HIPCHK(hipMemsetAsync(c->d_counts_base, 0, (size_t)c->counts_cap * 8, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RXG_OK;
}

} // extern "C"
