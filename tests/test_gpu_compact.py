"""UDP delivery through the GPU's per-socket payload compaction (-m gpu).

udp_process, once its lookup found the socket (udp.c:14-19), copies
dgram_len - 8 payload bytes from udp + 1 into an offload and enqueues it on
the socket's ring (udp.c:25-52); nrecvfrom returns offload.length = dgram_len
bytes (common.c:517-565).  K3 (csrc/rx_compact.hip) groups a burst's
delivered datagrams by socket, in burst order, and gathers their captured
payloads; libnstack then hands each socket its slice with one copy.

Checked: the device records and payload buffer against a numpy model of the
same grouping (every datagram, every byte), and the whole socket layer
(nstack_rx_burst -> nrecvfrom) against the delivery oracle
(oracle/ref_stack.c) on bursts with 1000 sockets, mixed sizes, captures that
end inside the payload, unknown ports and split reads."""
import ctypes as C

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

pytestmark = pytest.mark.gpu
L = "192.168.100.77"


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    return torch, torch.device("cuda", 0)


def _burst(rng, n, nsock, base=30000):
    """UDP frames to sockets :base.. (some to unbound ports), mixed payload
    sizes, 5% with captures cut inside the payload"""
    frames, caps = [], []
    ports = rng.integers(0, nsock + 20, n)
    sizes = rng.choice([0, 1, 5, 22, 100, 555, 1000, 1458], n)
    for k in range(n):
        pl = bytes(rng.integers(0, 256, int(sizes[k]), dtype=np.uint8))
        f = F.udp_frame(f"10.{k % 7}.{k % 200}.{k % 250 + 1}", 1000 + k % 50000, L,
                        base + int(ports[k]), pl)
        frames.append(f)
        caps.append(len(f) if rng.random() > 0.05 else int(rng.integers(20, len(f) + 1)))
    return frames, caps


def test_compaction_matches_model(torch_dev):
    torch, dev = torch_dev
    rng = np.random.default_rng(1)
    nsock = 700
    udp = np.zeros(nsock, R.UDP_SOCK_DTYPE)
    udp["localip"] = R.ip_raw(L)
    udp["localport"] = [R.port_raw(30000 + k) for k in range(nsock)]
    udp["protocol"] = 17
    frames, caps = _burst(rng, 6000, nsock)
    buf, off, lens = F.pack_frames(frames, 6, caplens=caps)
    n = len(frames)
    with R.Context(0) as ctx:
        ctx.flows_sync(udp, None)
        d_pk = torch.from_numpy(np.concatenate([buf, np.zeros(64, np.uint8)])).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        d_ln = torch.from_numpy(lens.view(np.int16)).to(dev)
        d_v = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        ctx.classify_dev(d_pk, d_off, d_ln, n, 6, 600, d_v, None, stream=sh)
        d_dg = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        d_first = torch.empty(nsock + 1, dtype=torch.int32, device=dev)
        cap = len(buf) + 4096
        d_pl = torch.full((cap,), 0xCD, dtype=torch.uint8, device=dev)
        d_tot = torch.empty(3, dtype=torch.int32, device=dev)
        ctx.udp_compact_dev(d_pk, d_off, d_ln, n, 6, d_v, d_dg, d_first, d_pl, cap, d_tot, stream=sh)
        torch.cuda.synchronize(dev)
        v = d_v.cpu().numpy().view(R.VERDICT_DTYPE)
        tot = d_tot.cpu().numpy().view(np.uint32)
        first = d_first.cpu().numpy().view(np.uint32)
        dg = d_dg.cpu().numpy().view(R.DGRAM_DTYPE)[:tot[0]]
        pl = d_pl.cpu().numpy()
    assert tot[2] == 0
    deliv = np.nonzero((v["cls"] == R.CLS_UDP) & (v["rc"] == 0))[0]
    order = deliv[np.argsort(v["flow_id"][deliv], kind="stable")]  # by socket, burst order inside
    assert tot[0] == len(order) and np.array_equal(dg["frame"], order)
    assert np.array_equal(first, np.searchsorted(v["flow_id"][order], np.arange(nsock + 1)))
    pos = 0
    for r, i in enumerate(order):
        f = frames[i][:caps[i]]
        plen = int(v["payload_len"][i])
        ncopy = max(0, min(plen, len(f) - 42))
        d = dg[r]
        assert d["offset"] == pos and d["len"] == plen, r
        assert d["sip"] == int.from_bytes((f + bytes(64))[26:30], "little")
        assert d["sport"] == int.from_bytes((f + bytes(64))[34:36], "little")
        assert pl[pos:pos + ncopy].tobytes() == f[42:42 + ncopy], r
        pad = (ncopy + 15) // 16 * 16
        assert not pl[pos + ncopy:pos + pad].any(), r
        pos += pad
    assert tot[1] == pos


def test_socket_layer_batches_match_oracle(torch_dev):
    """nstack_rx_burst (GPU classify + compaction + one copy per socket) then
    nrecvfrom with assorted lengths (split reads re-enqueue the rest at the
    ring's tail, common.c:542-556) — every return value, source address and
    byte equal to the delivery oracle's"""
    rng = np.random.default_rng(5)
    nsock = 1000
    ns = R.NStack(0, max_burst=8192, max_bytes=1 << 24)
    os_ = O.Stack()
    try:
        fds = []
        for k in range(nsock):
            a = ns.socket(R.SOCK_DGRAM)
            assert a == os_.socket(2)
            ns.bind(a, L, 30000 + k)
            os_.bind(a, R.ip_raw(L), R.port_raw(30000 + k))
            fds.append(a)
        for burst in range(4):
            frames, caps = _burst(rng, 3000, nsock)
            frames = [f[:c] for f, c in zip(frames, caps)]
            want = [os_.rx(f) for f in frames]
            r, rcs, _ = ns.rx_burst(frames)
            assert list(rcs) == want
            for fd in rng.permutation(fds)[:600]:  # leave some queued across bursts
                for n in (7, 2048, 4, 30, 65536):
                    r1, d1, a = ns.recvfrom(int(fd), n)
                    r2, d2, sip, sport = os_.recvfrom(int(fd), n)
                    if r2 == O.WOULD_BLOCK:
                        assert r1 == -1
                        continue
                    assert (r1, d1) == (r2, d2), (burst, fd, n)
                    assert (a.sin_addr, a.sin_port) == (sip, sport)
        for fd in fds:  # drain everything
            while True:
                r1, d1, _ = ns.recvfrom(fd, 65536)
                r2, d2, _, _ = os_.recvfrom(fd, 65536)
                assert (r1 == -1) == (r2 == O.WOULD_BLOCK)
                if r1 == -1:
                    break
                assert (r1, d1) == (r2, d2)
    finally:
        ns.fini()


# ---- TCP: the per-connection segment sort + payload gather (K4) -----------
def _seg_model(buf, off, lens, v, nt):
    """numpy/Python model of rxg_tcp_compact_dev over the oracle's verdicts:
    rc-0 TCP segments with a tcb id < nt, stable-sorted by id; header fields
    with bytes past the capture read as 0; PSH segments with plen > 0 keep
    min(plen, cap - 34 - 4*hl) payload bytes at 16-B aligned offsets in
    sorted order"""
    elig = np.nonzero((v["cls"] == R.CLS_TCP) & (v["rc"] == 0) & (v["flow_id"] < nt))[0]
    order = elig[np.argsort(v["flow_id"][elig], kind="stable")]
    recs, payload, pos = [], bytearray(), 0
    for i in order:
        o, cap = int(off[i]) << 6, int(lens[i])

        def b(k):
            return int(buf[o + k]) if k < cap else 0
        hl, fl = b(46) >> 4, b(47)
        plen = ((b(16) << 8) | b(17)) - 20 - 4 * hl
        src = 34 + 4 * hl
        keep = min(plen, max(cap - src, 0)) if (fl & 0x08 and plen > 0) else 0
        recs.append((int(i), int(v["flow_id"][i]),
                     (b(38) << 24) | (b(39) << 16) | (b(40) << 8) | b(41),
                     (b(42) << 24) | (b(43) << 16) | (b(44) << 8) | b(45),
                     plen, pos, b(34) | (b(35) << 8), b(36) | (b(37) << 8), keep, fl, hl))
        data = bytes(buf[o + src:o + src + keep])
        pad = (keep + 15) // 16 * 16
        payload += data + bytes(pad - keep)
        pos += pad
    out = np.zeros(len(recs), R.SEGMENT_DTYPE)
    for k, r in enumerate(recs):
        out[k] = r
    return out, bytes(payload)


def _tcp_burst(rng, n, keys, lis_port=9999):
    """TCP segments over the connections `keys` ((client ip, port) -> :9999):
    PSH data of assorted sizes, pure ACKs, FIN, PSH|FIN, 24-B headers, a
    total_length shorter than the header (negative plen), bad checksums, SYNs
    to the listener, 5% captures cut inside the segment, some UDP between"""
    frames, caps = [], []
    for k in range(n):
        cip, cport = keys[int(rng.integers(len(keys)))]
        r = rng.random()
        p = bytes(rng.integers(0, 256, int(rng.choice([0, 1, 7, 100, 555, 1446])), dtype=np.uint8))
        kw = dict(seq=int(rng.integers(0, 2 ** 32)), ack=int(rng.integers(0, 2 ** 32)))
        if r < 0.5:
            f = F.tcp_frame(cip, cport, L, lis_port, p, flags=0x18, **kw)
        elif r < 0.6:
            f = F.tcp_frame(cip, cport, L, lis_port, b"", flags=0x10, **kw)
        elif r < 0.65:
            f = F.tcp_frame(cip, cport, L, lis_port, b"", flags=0x11, **kw)
        elif r < 0.7:
            f = F.tcp_frame(cip, cport, L, lis_port, p, flags=0x19, **kw)  # PSH|FIN|ACK
        elif r < 0.75:
            f = F.tcp_frame(cip, cport, L, lis_port, p, flags=0x18, data_off=0x60, **kw)
        elif r < 0.8:
            f = F.tcp_frame(cip, cport, L, lis_port, p, flags=0x18, tl=30, tl_cksum=True,
                            **kw)  # plen < 0 (the checksum of 10 L4 bytes: rc 0)
        elif r < 0.85:
            f = F.tcp_frame(cip, cport, L, lis_port, p, flags=0x18, corrupt=len(p) > 0, **kw)
        elif r < 0.9:
            f = F.tcp_frame("10.200.0.1", 50000 + k, L, lis_port, b"", flags=0x02, **kw)  # SYN
        elif r < 0.95:
            f = F.udp_frame("10.1.1.1", 5000, L, 8889, p)
        else:
            f = F.tcp_frame(cip, cport, L, 7, p, flags=0x18, **kw)  # no tcb, no listener
        frames.append(f)
        caps.append(len(f) if rng.random() > 0.05 else int(rng.integers(20, len(f) + 1)))
    return frames, caps


@pytest.mark.parametrize("ntcb,passes", [(3000, 2), (300000, 3), (100, 1)])
def test_tcp_segment_sort_matches_model(torch_dev, ntcb, passes):
    """every record and every payload byte of K4 against the model, at id
    spaces that take 1, 2 and 3 radix passes; tcbs with consecutive ids get
    the traffic so that flows interleave in the burst"""
    torch, dev = torch_dev
    rng = np.random.default_rng(ntcb)
    tcb = np.zeros(ntcb + 1, R.TCB_DTYPE)
    tcb[0] = (0, R.ip_raw(L), 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)
    keys = []
    for k in range(1, ntcb + 1):
        cip, cport = f"10.{(k >> 16) & 255}.{(k >> 8) & 255}.{k & 255}", 1024 + k % 60000
        tcb[k] = (R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(9999), 4)
        keys.append((cip, cport))
    hot = keys[:50] + keys[-50:] + [keys[int(x)] for x in rng.integers(0, ntcb, 200)]
    frames, caps = _tcp_burst(rng, 5000, hot)
    buf, off, lens = F.pack_frames(frames, 6, caplens=caps)
    n = len(frames)
    want_v = O.Tables(np.zeros(0, R.UDP_SOCK_DTYPE), tcb).classify(buf, off, lens, 6)
    want_seg, want_pl = _seg_model(buf, off, lens, want_v, ntcb + 1)
    assert len(want_seg) > 2000
    with R.Context(0) as ctx:
        ctx.flows_sync(None, tcb)
        d_pk = torch.from_numpy(np.concatenate([buf, np.zeros(64, np.uint8)])).to(dev)
        d_off = torch.from_numpy(off.view(np.int32)).to(dev)
        d_ln = torch.from_numpy(lens.view(np.int16)).to(dev)
        d_v = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        sh = torch.cuda.current_stream(dev).cuda_stream
        ctx.classify_dev(d_pk, d_off, d_ln, n, 6, 1500, d_v, None, stream=sh)
        d_seg = torch.full((n * 32,), 0xEE, dtype=torch.uint8, device=dev)
        cap = len(buf) + 4096
        d_pl = torch.full((cap,), 0xCD, dtype=torch.uint8, device=dev)
        d_tot = torch.empty(3, dtype=torch.int32, device=dev)
        ctx.tcp_compact_dev(d_pk, d_off, d_ln, n, 6, d_v, d_seg, d_pl, cap, d_tot, stream=sh)
        torch.cuda.synchronize(dev)
        v = d_v.cpu().numpy().view(R.VERDICT_DTYPE)
        tot = d_tot.cpu().numpy().view(np.uint32)
        seg = d_seg.cpu().numpy().view(R.SEGMENT_DTYPE)[:tot[0]]
        pl = d_pl.cpu().numpy()
    assert v.tobytes() == want_v.tobytes()
    assert tot[2] == 0 and tot[0] == len(want_seg) and tot[1] == len(want_pl)
    bad = [k for k in range(len(seg)) if seg[k].tobytes() != want_seg[k].tobytes()]
    assert not bad, [(k, seg[k], want_seg[k]) for k in bad[:5]]
    assert pl[:len(want_pl)].tobytes() == want_pl
    assert np.all(pl[len(want_pl):] == 0xCD)  # nothing written past the used bytes
    assert any(s["plen"] < 0 for s in want_seg) and any((s["flags"] & 0x09) == 0x09
                                                         for s in want_seg)


def test_tcp_segment_sort_edge_bursts(torch_dev):
    """an empty burst, a burst without TCP, one connection taking every
    segment (one long run), and an id space of one listener"""
    torch, dev = torch_dev
    tcb = np.zeros(2, R.TCB_DTYPE)
    tcb[0] = (0, R.ip_raw(L), 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)
    tcb[1] = (R.ip_raw("10.0.0.1"), R.ip_raw(L), R.port_raw(4000), R.port_raw(9999), 4)
    rng = np.random.default_rng(9)
    cases = [[], [F.udp_frame("10.1.1.1", 5000, L, 8889, b"x" * 30)] * 5,
             [F.tcp_frame("10.0.0.1", 4000, L, 9999,
                          bytes(rng.integers(0, 256, int(rng.integers(0, 1400)), dtype=np.uint8)),
                          seq=k) for k in range(3000)]]
    with R.Context(0) as ctx:
        ctx.flows_sync(None, tcb)
        for frames in cases:
            n = len(frames)
            buf, off, lens = F.pack_frames(frames or [b"\0" * 64], 6)
            want_v = O.Tables(np.zeros(0, R.UDP_SOCK_DTYPE), tcb).classify(buf, off[:n], lens[:n], 6)
            want_seg, want_pl = _seg_model(buf, off, lens, want_v, 2)
            d_pk = torch.from_numpy(np.concatenate([buf, np.zeros(64, np.uint8)])).to(dev)
            d_off = torch.from_numpy(off.view(np.int32)).to(dev)
            d_ln = torch.from_numpy(lens.view(np.int16)).to(dev)
            d_v = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device=dev)
            sh = torch.cuda.current_stream(dev).cuda_stream
            ctx.classify_dev(d_pk, d_off, d_ln, n, 6, 1500, d_v, None, stream=sh)
            d_seg = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device=dev)
            cap = len(buf) + 4096
            d_pl = torch.zeros(cap, dtype=torch.uint8, device=dev)
            d_tot = torch.full((3,), 7, dtype=torch.int32, device=dev)
            ctx.tcp_compact_dev(d_pk, d_off, d_ln, n, 6, d_v, d_seg, d_pl, cap, d_tot, stream=sh)
            torch.cuda.synchronize(dev)
            tot = d_tot.cpu().numpy().view(np.uint32)
            assert tot[0] == len(want_seg) and tot[1] == len(want_pl) and tot[2] == 0
            seg = d_seg.cpu().numpy().view(R.SEGMENT_DTYPE)[:tot[0]]
            assert seg.tobytes() == want_seg.tobytes()
            assert d_pl.cpu().numpy()[:len(want_pl)].tobytes() == want_pl


def test_registered_pool_is_pulled_by_the_device(torch_dev):
    """rxg_register_host: a burst whose frames lie in registered memory is
    pulled by the GPU (no host gather); every output of
    rxg_process_mbufs_deliver equals the host-gathered burst's and the
    oracle's verdicts; one frame outside the registered memory sends the burst
    back to the host gather, with the same results"""
    torch, dev = torch_dev
    rng = np.random.default_rng(21)
    nsock = 300
    udp = np.zeros(nsock, R.UDP_SOCK_DTYPE)
    udp["localip"] = R.ip_raw(L)
    udp["localport"] = [R.port_raw(30000 + k) for k in range(nsock)]
    udp["protocol"] = 17
    tcb = np.zeros(401, R.TCB_DTYPE)
    tcb[0] = (0, R.ip_raw(L), 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)
    keys = []
    for k in range(1, 401):
        cip, cport = f"10.7.{k >> 8}.{k & 255}", 2000 + k
        tcb[k] = (R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(9999), 4)
        keys.append((cip, cport))
    uf, ucaps = _burst(rng, 1500, nsock)
    tf, tcaps = _tcp_burst(rng, 1500, keys)
    order = rng.permutation(3000)
    frames = [(uf + tf)[i] for i in order]
    caps = [(ucaps + tcaps)[i] for i in order]
    buf, off, lens = F.pack_frames(frames, 6, caplens=caps)
    buf = np.concatenate([buf, np.zeros(4096, np.uint8)])
    want_v = O.Tables(udp, tcb).classify(buf, off, lens, 6)
    arr, keep = R.NStack.mbufs_over(buf, off, lens, 6)
    with R.Context(0, max_pkts=4096, max_bytes=len(buf) + 65536) as ctx:
        ctx.flows_sync(udp, tcb)
        host = ctx.process_mbufs_deliver(arr)
        ctx.register_host(buf.ctypes.data, buf.nbytes)
        pulled = ctx.process_mbufs_deliver(arr)  # dense: one span copied (RXG_INGEST_AUTO)
        ctx.tune_ingest(R.INGEST_PULL)
        pulled_frames = ctx.process_mbufs_deliver(arr)  # frame by frame by the device
        ctx.tune_ingest(R.INGEST_AUTO)
        # one frame outside the registered memory: the burst is gathered on the host
        o5 = int(off[5]) << 6
        extra = np.zeros(2048, np.uint8)
        extra[:int(lens[5])] = buf[o5:o5 + int(lens[5])]
        keep[5].buf_addr = extra.ctypes.data
        mixed = ctx.process_mbufs_deliver(arr)
        ctx.unregister_host(buf.ctypes.data)
    assert host[0].tobytes() == want_v.tobytes()
    for got in (pulled, pulled_frames, mixed):
        for a, b in zip(host[:6], got[:6]):
            assert (a is None and b is None) or a.tobytes() == b.tobytes()
    assert len(host[4]) > 500 and host[6][1] >= 0


@pytest.mark.parametrize("layout", ["dense16", "sparse", "overlap"])
def test_registered_layouts_match_host_gather(torch_dev, layout):
    """rxg_tune_ingest's registered forms against the host gather on the same
    mbufs: frames packed at 16-B (not 64-B) boundaries (one span, 16-B
    descriptor units), frames 4 KiB apart (sparse: pulled frame by frame), and
    mbufs sharing data (the span smaller than the frames' bytes: the results
    copy-out bound); every output equal"""
    rng = np.random.default_rng({"dense16": 41, "sparse": 42, "overlap": 43}[layout])
    nsock = 200
    udp = np.zeros(nsock, R.UDP_SOCK_DTYPE)
    udp["localip"] = R.ip_raw(L)
    udp["localport"] = [R.port_raw(30000 + k) for k in range(nsock)]
    udp["protocol"] = 17
    tcb = np.zeros(201, R.TCB_DTYPE)
    tcb[0] = (0, R.ip_raw(L), 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)
    keys = []
    for k in range(1, 201):
        cip, cport = f"10.8.{k >> 8}.{k & 255}", 2000 + k
        tcb[k] = (R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(9999), 4)
        keys.append((cip, cport))
    uf, ucaps = _burst(rng, 700, nsock)
    tf, tcaps = _tcp_burst(rng, 700, keys)
    frames = [f[:c] for f, c in zip(uf + tf, ucaps + tcaps)]
    frames = [frames[i] for i in rng.permutation(len(frames))]
    n = len(frames)
    stride = 4096 if layout == "sparse" else 0
    pos, offs = 0, []
    for f in frames:
        offs.append(pos)
        pos += stride or ((len(f) + 15) & ~15)
    buf = np.zeros(pos + 8192, np.uint8)
    for o, f in zip(offs, frames):
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
    ms = (R.Mbuf * n)()
    for i in range(n):
        o = offs[i] if layout != "overlap" else offs[i % (n // 3)]  # a third of the data, reused
        f = frames[i] if layout != "overlap" else frames[i % (n // 3)]
        ms[i].buf_addr = buf.ctypes.data + o
        ms[i].data_len = len(f)
    arr = (C.POINTER(R.Mbuf) * n)(*[C.pointer(ms[i]) for i in range(n)])
    with R.Context(0, max_pkts=2048, max_bytes=(2048 * 1536 if layout != "sparse" else n * 4096 + 8192)) as ctx:
        ctx.flows_sync(udp, tcb)
        host = ctx.process_mbufs_deliver(arr)
        ctx.register_host(buf.ctypes.data, buf.nbytes)
        auto = ctx.process_mbufs_deliver(arr)
        ctx.tune_ingest(R.INGEST_PULL)
        pull = ctx.process_mbufs_deliver(arr)
        ctx.unregister_host(buf.ctypes.data)
    for got in (auto, pull):
        for a, b in zip(host[:6], got[:6]):
            assert (a is None and b is None) or a.tobytes() == b.tobytes(), layout
    assert len(host[4]) > 100 and len(host[1]) > 100
