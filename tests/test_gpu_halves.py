"""Two delivery bursts in flight at once (-m gpu; RXG_DELIVER_DEPTH).

rxg_deliver_submit keeps a set of pinned result buffers per burst in flight,
so burst k+1's frames cross PCIe while burst k's results come back;
nstack_rx_burst can send a burst as two halves that way (nstack_set_halves)
and deliver the first half while the second is on the GPU.  The reference
handles the frames one by one in order (netfamily.c:152-200, udp.c:14-52,
tcp.c:373-415), so the halves must not change anything an application sees:

  - library: every output of two overlapped deliveries (waited for in
    reverse order) equals the same bursts delivered one at a time, and a
    third submit while both sets are in flight is refused;
  - socket layer: bursts of 12,000 frames, whose first half creates tcbs
    (SYN) that the second half's segments complete (ACK) and use (data), so
    the second half's verdicts are stale by the time it is delivered, against
    oracle/ref_stack.c frame by frame: every return code, accepted
    connection, nrecv / nrecvfrom result and what the application drains;
  - the pipelined pair (nstack_rx_submit / nstack_rx_complete): whole bursts,
    burst k+1 on the GPU while burst k is delivered, against the same oracle
    run sequentially, and with an application thread draining beside it."""
import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R
from test_gpu_compact import _burst, _tcp_burst

pytestmark = pytest.mark.gpu
L = "192.168.100.77"


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a GPU (no fallback path exists)")
    return torch, torch.device("cuda", 0)


def _tables(nsock=300, ntcb=400):
    udp = np.zeros(nsock, R.UDP_SOCK_DTYPE)
    udp["localip"] = R.ip_raw(L)
    udp["localport"] = [R.port_raw(30000 + k) for k in range(nsock)]
    udp["protocol"] = 17
    tcb = np.zeros(ntcb + 1, R.TCB_DTYPE)
    tcb[0] = (0, R.ip_raw(L), 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)
    keys = []
    for k in range(1, ntcb + 1):
        cip, cport = f"10.7.{k >> 8}.{k & 255}", 2000 + k
        tcb[k] = (R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(9999), 4)
        keys.append((cip, cport))
    return udp, tcb, keys


def _mixed(rng, n, nsock, keys):
    uf, ucaps = _burst(rng, n // 2, nsock)
    tf, tcaps = _tcp_burst(rng, n - n // 2, keys)
    order = rng.permutation(n)
    frames = [(uf + tf)[i] for i in order]
    caps = [(ucaps + tcaps)[i] for i in order]
    buf, off, lens = F.pack_frames(frames, 6, caplens=caps)
    return np.concatenate([buf, np.zeros(4096, np.uint8)]), off, lens


def test_two_deliveries_in_flight_match_one_at_a_time(torch_dev):
    rng = np.random.default_rng(31)
    udp, tcb, keys = _tables()
    a = _mixed(rng, 3000, len(udp), keys)
    b = _mixed(rng, 2500, len(udp), keys)
    ma, ka = R.NStack.mbufs_over(a[0], a[1], a[2], 6)
    mb, kb = R.NStack.mbufs_over(b[0], b[1], b[2], 6)
    tables = O.Tables(udp, tcb)
    with R.Context(0, max_pkts=4096, max_bytes=len(a[0]) + 65536) as ctx:
        ctx.flows_sync(udp, tcb)
        one_a = ctx.process_mbufs_deliver(ma)
        one_b = ctx.process_mbufs_deliver(mb)
        ha = ctx.deliver_submit(ma)
        hb = ctx.deliver_submit(mb)
        with pytest.raises(Exception):  # both sets in flight
            ctx.deliver_submit(ma)
        got_b = ctx.deliver_wait(hb)  # any order
        got_a = ctx.deliver_wait(ha)
        again = ctx.process_mbufs_deliver(ma)  # the sets are free again
    assert one_a[0].tobytes() == tables.classify(a[0], a[1], a[2], 6).tobytes()
    assert one_b[0].tobytes() == tables.classify(b[0], b[1], b[2], 6).tobytes()
    for want, got in ((one_a, got_a), (one_b, got_b), (one_a, again)):
        for x, y in zip(want[:6], got[:6]):
            assert (x is None and y is None) or x.tobytes() == y.tobytes()
    assert len(one_a[4]) > 300 and len(one_a[1]) > 300  # TCP segments and UDP datagrams


class Stacks:
    def __init__(self, n_est):
        self.ns = R.NStack(0, max_burst=16384, max_bytes=16384 * 1536)
        self.ns.set_halves(4096)  # 12,000-frame bursts: two halves of 6,000
        self.os = O.Stack()
        a = self.ns.socket(R.SOCK_STREAM)
        assert a == self.os.socket(1)
        assert self.ns.bind(a, L, 9999) == self.os.bind(a, R.ip_raw(L), R.port_raw(9999)) == 0
        assert self.ns.listen(a) == self.os.listen(a) == 0
        self.lfd = a
        self.ufd = []
        for k in range(40):
            u = self.ns.socket(R.SOCK_DGRAM)
            assert u == self.os.socket(2)
            assert self.ns.bind(u, L, 30000 + k) == self.os.bind(u, R.ip_raw(L), R.port_raw(30000 + k)) == 0
            self.ufd.append(u)
        self.est = []
        for k in range(n_est):
            cip, cport = f"10.9.{k >> 8}.{k & 255}", 3000 + k
            t = (R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(9998))
            assert self.ns.lib.nstack_tcb_add(*t, 4) == 0 and self.os.tcb_add(*t, 4) == 0
            self.est.append((cip, cport))
        self.conns = {}

    def burst(self, frames):
        want = [self.os.rx(f) for f in frames]
        n, rcs, _ = self.ns.rx_burst(frames)
        bad = [(i, int(rcs[i]), want[i]) for i in range(len(want)) if rcs[i] != want[i]]
        assert not bad, bad[:10]
        return self.ns.last_burst_phases()

    def accept_all(self):
        while True:
            fd, sip, sport = self.os.accept(self.lfd)
            if fd == O.WOULD_BLOCK:
                break
            got, a = self.ns.accept(self.lfd)
            assert (got, a.sin_addr, a.sin_port) == (fd, sip, sport)
            self.conns[(sip, sport)] = fd

    def read_all(self, n):
        for key, fd in list(self.conns.items()):
            while True:
                r1, d1 = self.ns.recv(fd, n, full=True)
                r2, d2 = self.os.recv(fd, n)
                if r2 == O.WOULD_BLOCK:
                    assert r1 == -1, key
                    break
                assert (r1, d1) == (r2, d2), (key, r1, r2)
        for fd in self.ufd:
            while True:
                r1, d1, a1 = self.ns.recvfrom(fd, n)
                r2, d2, s2, p2 = self.os.recvfrom(fd, n)
                if r2 == O.WOULD_BLOCK:
                    assert r1 == -1, fd
                    break
                assert (r1, d1[:max(r1, 0)], a1.sin_addr, a1.sin_port) == (r2, d2[:max(r2, 0)], s2, p2)


def _est_seg(rng, cip, cport):
    p = bytes(rng.integers(0, 256, int(rng.choice([0, 9, 300, 1446])), dtype=np.uint8))
    kw = dict(seq=int(rng.integers(0, 2 ** 32)), ack=int(rng.integers(0, 2 ** 32)))
    r = rng.random()
    if r < 0.8:
        return F.tcp_frame(cip, cport, L, 9998, p, flags=0x18, **kw)
    if r < 0.9:
        return F.tcp_frame(cip, cport, L, 9998, b"", flags=0x10, **kw)
    return F.tcp_frame(cip, cport, L, 9998, p, flags=0x19, **kw)


def test_socket_layer_halves_match_oracle(torch_dev):
    rng = np.random.default_rng(32)
    st = Stacks(2000)
    try:
        n = 12000  # halves of 6000
        for b in range(3):
            frames = []
            for _ in range(n - 200):
                if rng.random() < 0.5:
                    frames.append(_est_seg(rng, *st.est[int(rng.integers(len(st.est)))]))
                else:
                    k = int(rng.integers(48))  # 8 ports without a socket
                    pl = bytes(rng.integers(0, 256, int(rng.choice([0, 5, 100, 1000])), np.uint8))
                    frames.append(F.udp_frame(f"10.5.{k}.1", 7000 + k, L, 30000 + k, pl))
            if b < 2:  # SYN in the first half, its ACK and data in the second
                for i in range(60):
                    cip, cport = f"10.250.{b}.{i + 1}", 61000 + i
                    frames.insert(int(rng.integers(0, 5000)),
                                  F.tcp_frame(cip, cport, L, 9999, b"", flags=0x02, seq=1000 + i))
                    frames.insert(int(rng.integers(6200, len(frames))),
                                  F.tcp_frame(cip, cport, L, 9999, b"", flags=0x10))
                    frames.append(F.tcp_frame(cip, cport, L, 9999, b"data %d" % i, flags=0x18))
            frames = frames[:n]
            stale0 = st.ns.stat(5)
            ph = st.burst(frames)
            if b < 2:  # the first half's SYNs changed the lists: the second half is stale
                assert st.ns.stat(5) == stale0 + 1
            else:  # both halves through the per-connection and per-socket batches
                assert st.ns.stat(5) == stale0
                assert ph["segments"] > 1000 and ph["datagrams"] > 1000, ph
            st.accept_all()
            st.read_all(int(rng.choice([7, 4096])))
            buf = np.zeros(65536, np.uint8)
            assert st.ns.drain_all(buf) == st.os.drain_all(buf), b
        assert len(st.conns) >= 100
    finally:
        st.ns.fini()


def _mixed_frames(rng, st, n, b, syn):
    """n frames to the stack of `st`: data to its established connections and
    datagrams to its sockets; with syn, 60 SYNs to the listener (burst b)
    whose ACK and first data come in the NEXT burst (made by _syn_followups)"""
    frames = []
    for _ in range(n - (60 if syn else 0)):
        if rng.random() < 0.5:
            frames.append(_est_seg(rng, *st.est[int(rng.integers(len(st.est)))]))
        else:
            k = int(rng.integers(48))  # 8 ports without a socket
            pl = bytes(rng.integers(0, 256, int(rng.choice([0, 5, 100, 1000])), np.uint8))
            frames.append(F.udp_frame(f"10.5.{k}.1", 7000 + k, L, 30000 + k, pl))
    if syn:
        for i in range(60):
            frames.insert(int(rng.integers(0, len(frames))),
                          F.tcp_frame(f"10.251.{b}.{i + 1}", 62000 + i, L, 9999, b"", flags=0x02,
                                      seq=2000 + i))
    return frames


def _syn_followups(rng, frames, b):
    for i in range(60):
        cip, cport = f"10.251.{b}.{i + 1}", 62000 + i
        frames.insert(int(rng.integers(0, len(frames) // 2)), F.tcp_frame(cip, cport, L, 9999, b"", flags=0x10))
        frames.append(F.tcp_frame(cip, cport, L, 9999, b"piped %d" % i, flags=0x18))
    return frames


def test_socket_layer_pipelined_match_oracle(torch_dev):
    """nstack_rx_submit / nstack_rx_complete with burst k+1 on the GPU while
    burst k is delivered: every return code of every burst equals the oracle's
    sequential run (burst k wholly before burst k+1, netfamily.c:147-200).
    Bursts 1 and 3 carry SYNs whose ACK and data arrive in bursts 2 and 4,
    which were classified before those SYNs were delivered: they must be
    delivered frame by frame on the live lists (stat 5, a stale part each);
    the others go through the per-connection and per-socket batches."""
    rng = np.random.default_rng(35)
    st = Stacks(2000)
    st.ns.set_halves(0)
    try:
        bursts = []
        for b in range(6):
            fr = _mixed_frames(rng, st, 6000, b, syn=b in (1, 3))
            if b in (2, 4):
                fr = _syn_followups(rng, fr, b - 1)
            bursts.append(fr)
        stale0 = st.ns.stat(5)
        st.ns.rx_submit(bursts[0])
        stale = []
        for b in range(6):
            if b + 1 < 6:
                st.ns.rx_submit(bursts[b + 1])
                assert st.ns.rx_pending() == 2
                with pytest.raises(R.RxgError):  # both delivery sets in flight
                    st.ns.rx_submit(bursts[b + 1][:10])
                with pytest.raises(R.RxgError):  # the one-shot call is refused meanwhile
                    st.ns.rx_burst(bursts[b][:10])
                with pytest.raises(R.RxgError):  # and so is host-verdict delivery
                    st.ns.deliver(bursts[b][:1], np.zeros(1, R.VERDICT_DTYPE))
            s0 = st.ns.stat(5)
            want = [st.os.rx(f) for f in bursts[b]]
            n, rcs, _ = st.ns.rx_complete()
            bad = [(i, int(rcs[i]), want[i]) for i in range(len(want)) if rcs[i] != want[i]]
            assert not bad, (b, bad[:10])
            stale.append(st.ns.stat(5) - s0)
            st.accept_all()
            st.read_all(int(rng.choice([7, 4096])))
            buf = np.zeros(65536, np.uint8)
            assert st.ns.drain_all(buf) == st.os.drain_all(buf), b
        assert st.ns.rx_pending() == 0
        assert st.ns.lib.nstack_rx_complete() == -22  # RXG_EINVAL: nothing pending
        assert stale == [0, 0, 1, 0, 1, 0], stale
        assert st.ns.stat(5) == stale0 + 2
        assert len(st.conns) >= 100
        # bursts left pending are dropped by fini (waited for, not delivered)
        st.ns.rx_submit(bursts[0][:100])
    finally:
        st.ns.fini()


def _split_model(lens, cap):
    """drain_all's count through nrecv's split path (common.c:483-496): a
    fragment longer than cap gives cap bytes, re-queues the rest at the tail
    and returns the REMAINING length; the last piece returns its length"""
    got = nb = 0
    for n in lens:
        while n > cap:
            n -= cap
            got, nb = got + 1, nb + n
        got, nb = got + 1, nb + n
    return got, nb


@pytest.mark.parametrize("cap", [256, 1000, 4096])
def test_drain_all_reads_long_fragments_through_the_split_path(torch_dev, cap):
    """drain_all takes whole ring items out of a tcb and reads them after the
    stack's lock is released, except an item holding a fragment longer than
    the buffer, which goes through nrecv's split path in place: the counts
    must be those of nrecv called until empty"""
    ns = R.NStack(0, max_burst=1024, max_bytes=1024 * 1536)
    try:
        conns = []
        for k in range(3):
            t = (R.ip_raw(f"10.9.0.{k + 1}"), R.ip_raw(L), R.port_raw(3000 + k), R.port_raw(9998))
            assert ns.lib.nstack_tcb_add(*t, 4) == 0
            conns.append((f"10.9.0.{k + 1}", 3000 + k))
        rng = np.random.default_rng(33)
        lens, frames = [], []
        for i in range(60):
            cip, cport = conns[i % 3]
            n = int(rng.choice([1446, 9, 300, 1000, 257, 77]))
            lens.append(n)
            frames.append(F.tcp_frame(cip, cport, L, 9998, bytes(rng.integers(0, 256, n, np.uint8)),
                                      flags=0x18, seq=1000 + i, ack=1))
        _, rcs, _ = ns.rx_burst(frames)
        assert (np.asarray(rcs) == 0).all()
        buf = np.zeros(cap, np.uint8)
        assert ns.drain_all(buf) == _split_model(lens, cap)
        assert ns.drain_all(buf) == (0, 0)
    finally:
        ns.fini()


def _fnv_sum(payloads):
    """sum mod 2^64 of FNV-1a 64 over each payload (nstack_drain_all_sum's
    check), vectorised over the payloads"""
    n = len(payloads)
    lens = np.array([len(p) for p in payloads], np.int64)
    m = np.zeros((n, int(lens.max(initial=1))), np.uint8)
    for i, p in enumerate(payloads):
        m[i, :len(p)] = np.frombuffer(p, np.uint8)
    h = np.full(n, 0xcbf29ce484222325, np.uint64)
    prime = np.uint64(0x100000001b3)
    with np.errstate(over="ignore"):
        for j in range(m.shape[1]):
            live = lens > j
            h[live] = (h[live] ^ m[live, j].astype(np.uint64)) * prime
        return int(h[lens > 0].sum(dtype=np.uint64))


@pytest.mark.parametrize("mode", ["pooled", "inplace", "inplace_pipelined", "pooled_pipelined"])
def test_two_threads_receive_every_byte(torch_dev, mode):
    """The reference's arrangement: the protocol loop on one thread
    (nstack_rx_burst), the application on another draining every socket
    (nstack_drain_all_sum) at the same time.  pooled: the payloads come back
    from the GPU into pooled pinned buffers that the fragments point into
    (rx_burst waits for one while the application still holds them all);
    inplace: the fragments point into the frames, which their mbufs' counts
    hold (nstack_set_rx_inplace).  Every payload byte of every burst must
    reach the application exactly once and unchanged: the sum of the FNV-1a
    hashes of what the reads returned equals that of the payloads sent, so a
    buffer reused early (a payload overwritten while still queued) fails it."""
    import threading
    ns = R.NStack(0, max_burst=4096, max_bytes=4096 * 1536)
    try:
        if mode.startswith("inplace"):
            ns.set_rx_inplace(True)
        conns = []
        for k in range(512):
            cip, cport = f"10.8.{k >> 8}.{k & 255}", 4000 + k
            t = (R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(9998))
            assert ns.lib.nstack_tcb_add(*t, 4) == 0
            conns.append((cip, cport))
        rng = np.random.default_rng(34)
        bursts, want_items, want_bytes, payloads = [], 0, 0, []
        for b in range(16):
            frames = []
            for i in range(4000):
                cip, cport = conns[int(rng.integers(len(conns)))]
                n = int(rng.choice([1446, 1446, 700, 33]))
                pl = bytes(rng.integers(0, 256, n, np.uint8))
                frames.append(F.tcp_frame(cip, cport, L, 9998, pl, flags=0x18, seq=i, ack=1))
                want_items, want_bytes = want_items + 1, want_bytes + n
                payloads.append(pl)
            buf, off, lens = F.pack_frames(frames, 6)
            arr, keep = R.NStack.mbufs_over(buf, off, lens, 6)
            bursts.append((arr, len(frames), keep, buf))
        want_sum = _fnv_sum(payloads)
        got = [0, 0, 0]
        stop = threading.Event()

        def app():
            buf = np.zeros(65536, np.uint8)
            while True:
                last = stop.is_set()
                g, nb, hs = ns.drain_all_sum(buf)
                got[0], got[1], got[2] = got[0] + g, got[1] + nb, (got[2] + hs) % (1 << 64)
                if last:
                    break

        c0, w0 = ns.stat(6), ns.stat(11)
        th = threading.Thread(target=app)
        th.start()
        try:
            if mode.endswith("pipelined"):  # burst k+1 on the GPU while burst k is delivered
                ns.rx_submit_mbufs(bursts[0][0], bursts[0][1])
                for k, (arr, n, _keep, _buf) in enumerate(bursts):
                    if k + 1 < len(bursts):
                        ns.rx_submit_mbufs(bursts[k + 1][0], bursts[k + 1][1])
                    assert ns.rx_complete_mbufs() >= 0
                    if mode.startswith("inplace"):
                        ns.mbufs_put(arr, n)
            else:
                for arr, n, _keep, _buf in bursts:
                    assert ns.rx_burst_mbufs(arr, n) >= 0
                    if mode == "inplace":
                        ns.mbufs_put(arr, n)  # the caller's reference
        finally:
            stop.set()
            th.join()
        ns.reclaim()  # (the application thread's reads are freed by the protocol side)
        assert (got[0], got[1]) == (want_items, want_bytes)
        assert got[2] == want_sum
        assert ns.stat(7) == 0  # no batch left holding a payload buffer
        if mode.startswith("inplace"):  # every hold on a frame let go, exactly once
            for _arr, _n, keep, _buf in bursts:
                assert all(keep[i].refcnt == 0 for i in range(len(keep)))
            assert ns.stat(6) == c0  # nothing copied
        print(mode, "copied bytes", ns.stat(6) - c0, "bursts that waited", ns.stat(11) - w0)
    finally:
        ns.fini()
