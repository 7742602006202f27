"""The delivery half against its oracle.

libnstack (host/nstack.c: verdict -> socket delivery and the verdict-driven
TCP state machine) is driven side by side with oracle/ref_stack.c, the
independent restatement of udp.c:25-52, tcp.c:3-331/:373-415 and the socket
layer common.c:262-666, on the same frame sequences: per-frame return codes,
naccept results, every nrecvfrom / nrecv return value and buffer, tcb states
(status, rcv_nxt, snd_nxt once an ACK has set it, fd) and every control
fragment queued for transmission (flags, acknum) must agree.

Explicit, tested exceptions (the oracle defines what the reference leaves
undefined, see ref_stack.c): bytes past a capture and the 8 bytes nrecvfrom
returns past a datagram's payload read as 0; the random initial sequence
number is not compared; the non-blocking outcome stands for a blocking wait
(nstack: MSG_DONTWAIT -> -1, oracle: -2).

CPU: verdicts from the oracle's front end (the GPU's are bit-identical,
test_gpu_parity.py) through nstack_deliver.  GPU: the same scenario through
nstack_rx_burst (GPU classify + delivery)."""
import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

L, L2 = "192.168.100.77", "10.9.9.9"
UDP_BINDS = [(L, 8889), (L, 8890), (L, 7000), (L2, 8889)]
LISTEN = [(L, 9999), (L, 8080)]


def _ip(s):
    return R.ip_raw(s)


def _port(p):
    return R.port_raw(p)


def _client_script(rng, k, dport):
    """one TCP client's segments in order: handshake, data, FIN, and (after the
    server closes: 'close' marker) the final ACK; with the edge cases mixed in"""
    cip, cport = f"10.0.{k // 200}.{1 + k % 200}", 40000 + k
    seq = int(rng.integers(1, 2 ** 31))
    seg = []

    def tcp(payload=b"", flags=0x18, **kw):
        return F.tcp_frame(cip, cport, L, dport, payload, flags=flags, seq=seq, **kw)
    seg.append(tcp(flags=0x02))            # SYN -> SYN_RCVD, SYN|ACK queued
    seq += 1
    if rng.random() < 0.2:
        seg.append(tcp(flags=0x02))        # a retransmitted SYN (SYN_RCVD: ignored)
    seg.append(tcp(flags=0x10))            # ACK -> ESTABLISHED
    for _ in range(int(rng.integers(1, 5))):
        n = int(rng.choice([0, 1, 7, 100, 600]))
        p = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        kind = rng.random()
        if kind < 0.1:
            seg.append(tcp(p, corrupt=len(p) > 0))               # bad checksum (if any payload)
        elif kind < 0.2:
            seg.append(tcp(p, data_off=0x60))                     # options: 24-B header
        elif kind < 0.25:
            seg.append(tcp(p, tl=30, tl_cksum=True))              # tl - 20 < hl: 0-length EOF
        elif kind < 0.3:
            seg.append(tcp(flags=0x02))                           # SYN while established
        elif kind < 0.35:
            seg.append(tcp(p, flags=0x19))                        # PSH|FIN|ACK in one segment
        else:
            seg.append(tcp(p))                                    # PSH|ACK data
        seq += n
    if rng.random() < 0.8:
        seg.append(tcp(flags=0x11))        # FIN|ACK -> CLOSE_WAIT, EOF queued
        seq += 1
        seg.append("close")                # the server closes: LAST_ACK, FIN|ACK queued
        seg.append(tcp(flags=0x10))        # ACK -> CLOSED, the tcb leaves the list
    return (cip, cport, dport), seg


def _udp_frames(rng, n):
    out = []
    for _ in range(n):
        r = rng.random()
        dst, port = UDP_BINDS[int(rng.integers(len(UDP_BINDS)))]
        if r < 0.1:
            port = 6000                                            # no socket
        sip = f"10.1.{int(rng.integers(0, 4))}.{int(rng.integers(1, 255))}"
        p = bytes(rng.integers(0, 256, int(rng.choice([0, 1, 22, 100, 700])), dtype=np.uint8))
        if r < 0.2:
            f = F.udp_frame(sip, 5000, dst, port, p, dgram_len=int(rng.integers(0, 9)))  # <= 8
        elif r < 0.3:
            f = F.udp_frame(sip, 5000, dst, port, p, dgram_len=len(p) + 8 + 40)  # claims more
        elif r < 0.35:
            f = F.udp_frame(sip, 5000, dst, port, p)[:int(rng.integers(14, 45))]  # cut capture
        else:
            f = F.udp_frame(sip, 5000, dst, port, p, corrupt=rng.random() < 0.1)
        out.append(f)
    return out


def _scenario(seed, n_clients=8, n_udp=60):
    """the frame sequence (per-client TCP order kept, interleaved at random)
    with the socket calls made between bursts"""
    rng = np.random.default_rng(seed)
    scripts = [_client_script(rng, k, LISTEN[k % 2][1] if k < n_clients - 1 else 7)
               for k in range(n_clients)]  # the last client has no listener
    streams = [list(s) for _, s in scripts] + [_udp_frames(rng, n_udp)] + \
        [[F.arp_frame("10.0.0.5", L), F.icmp_frame("10.0.0.5", L)] * 2]
    keys = [k for k, _ in scripts]
    events, burst = [], []
    while any(streams):
        i = int(rng.choice([j for j, s in enumerate(streams) if s]))
        item = streams[i].pop(0)
        if isinstance(item, str):                # the server closes this client's connection
            if burst:
                events.append(("burst", burst))
                burst = []
            events.append(("close_conn", keys[i]))
            continue
        burst.append(item)
        if len(burst) >= int(rng.integers(1, 12)):
            events.append(("burst", burst))
            burst = []
            for _ in range(int(rng.integers(0, 3))):
                events.append(("recv_any", int(rng.choice([1, 7, 30, 200, 4096]))))
            if rng.random() < 0.5:
                events.append(("accept_all", None))
    if burst:
        events.append(("burst", burst))
    return keys, events


class Pair:
    """nstack and the oracle stack side by side, socket by socket"""

    def __init__(self, ns, deliver):
        self.ns, self.os, self.deliver_mode = ns, O.Stack(), deliver
        self.udp_fds, self.listen_fds, self.conns = [], {}, {}  # conn key -> fd

    def setup(self):
        for ip, port in UDP_BINDS:
            a = self.ns.socket(R.SOCK_DGRAM)
            b = self.os.socket(2)
            assert a == b
            assert self.ns.bind(a, ip, port) == self.os.bind(b, _ip(ip), _port(port)) == 0
            self.udp_fds.append(a)
        for ip, port in LISTEN:
            a = self.ns.socket(R.SOCK_STREAM)
            assert a == self.os.socket(1)
            assert self.ns.bind(a, ip, port) == self.os.bind(a, _ip(ip), _port(port)) == 0
            assert self.ns.listen(a) == self.os.listen(a) == 0
            self.listen_fds[port] = a

    def check_tables(self, frames, v):
        """the library's host table images (what the device probes) give every
        frame's key the flow of the oracle's list walk (verdicts v, stable ids)"""
        for f, x in zip(frames, v):
            if len(f) < 38 or x["cls"] not in (R.CLS_UDP, R.CLS_TCP):
                continue
            sip, dip = int.from_bytes(f[26:30], "little"), int.from_bytes(f[30:34], "little")
            sport, dport = int.from_bytes(f[34:36], "little"), int.from_bytes(f[36:38], "little")
            if x["cls"] == R.CLS_UDP:
                assert self.ns.lookup_udp(dip, dport) == x["flow_id"], (f.hex(), x)
            elif x["cksum_ok"]:
                assert self.ns.lookup_tcp(sip, dip, sport, dport) == x["flow_id"], (f.hex(), x)

    def burst(self, frames):
        want = [self.os.rx(f) for f in frames]
        rcs = np.zeros(len(frames), np.int32)
        if self.deliver_mode == "gpu":
            # the verdicts the GPU must hand the delivery: the oracle's front
            # end over the lists as they stand before the burst, in stable ids
            u, t = self.ns.flows()
            buf, off, lens = F.pack_frames(frames)
            vw = self.ns.to_ids(O.Tables(u, t).classify(buf, off, lens, 6))
            self.check_tables(frames, vw)
            _, rcs, vg = self.ns.rx_burst(frames)
            assert vg.tobytes() == vw.tobytes(), [(i, vg[i], vw[i]) for i in range(len(frames))
                                                  if vg[i].tobytes() != vw[i].tobytes()]
        else:
            u, t, gen = self.ns.flows(with_gen=True)
            buf, off, lens = F.pack_frames(frames)
            v = self.ns.to_ids(O.Tables(u, t).classify(buf, off, lens, 6))
            self.check_tables(frames, v)
            self.ns.deliver(frames, v, rcs, gen)
        assert list(rcs) == want, (list(rcs), want)

    def accept_all(self):
        for port, lfd in self.listen_fds.items():
            while True:
                fd, sip, sport = self.os.accept(lfd)
                if fd == O.WOULD_BLOCK:
                    break
                got, a = self.ns.accept(lfd)
                assert (got, a.sin_addr, a.sin_port) == (fd, sip, sport)
                self.conns[(sip, sport, port)] = fd

    def recv_any(self, n):
        for fd in self.udp_fds:
            r1, d1, a = self.ns.recvfrom(fd, n)
            r2, d2, sip, sport = self.os.recvfrom(fd, n)
            if r2 == O.WOULD_BLOCK:
                assert r1 == -1
                continue
            assert (r1, d1) == (r2, d2), (fd, n, r1, r2)
            assert (a.sin_addr, a.sin_port) == (sip, sport)
        for key, fd in list(self.conns.items()):
            r1, d1 = self.ns.recv(fd, n, full=True)
            r2, d2 = self.os.recv(fd, n)
            if r2 == O.WOULD_BLOCK:
                assert r1 == -1
                continue
            assert (r1, d1) == (r2, d2), (key, n, r1, r2)

    def close_conn(self, key):
        cip, cport, dport = key
        k = (_ip(cip), _port(cport), dport)
        self.accept_all()
        fd = self.conns.pop(k, None)
        if fd is not None:
            assert self.ns.close(fd) == self.os.close(fd) == 0

    def compare_tcbs(self, keys):
        assert self.ns.tcb_count() == self.os.tcb_count()
        for cip, cport, dport in keys:
            t = (_ip(cip), _ip(L), _port(cport), _port(dport))
            want = self.os.tcb_state(*t)
            got = self.ns.tcb_state(*t)
            if want is None:
                assert got is None, t
                continue
            st, rn, sn, fd = want
            assert got is not None and (got[0], got[1], got[3]) == (st, rn, fd), (t, got, want)
            if sn is not None:
                assert got[2] == sn, (t, got, want)
            assert self.ns.tcb_sndq(*t) == self.os.tcb_sndq(*t), t


def _run(ns, mode, seed):
    keys, events = _scenario(seed)
    p = Pair(ns, mode)
    p.setup()
    for kind, arg in events:
        if kind == "burst":
            p.burst(arg)
        elif kind == "recv_any":
            p.recv_any(arg)
        elif kind == "accept_all":
            p.accept_all()
        elif kind == "close_conn":
            p.close_conn(arg)
    p.compare_tcbs(keys)
    p.accept_all()
    for n in (3, 64, 4096, 4096, 4096):
        p.recv_any(n)
    p.compare_tcbs(keys)
    return p


@pytest.fixture()
def ns_host():
    s = R.NStack(R.HOST_ONLY)
    yield s
    s.fini()


@pytest.mark.parametrize("inplace", [False, True], ids=["copy", "inplace"])
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6, 7, 8])
def test_delivery_matches_oracle(ns_host, seed, inplace):
    """inplace: receive fragments point into the frames (nstack_set_rx_inplace)
    instead of copies (tcp.c:133-185); every nrecv result is the same"""
    if inplace:
        ns_host.set_rx_inplace(True)
    _run(ns_host, "cpu", seed)


@pytest.mark.gpu
@pytest.mark.parametrize("inplace", [False, True], ids=["copy", "inplace"])
@pytest.mark.parametrize("seed", [1, 5])
def test_delivery_through_gpu_matches_oracle(seed, inplace):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    ns = R.NStack(0)
    try:
        if inplace:  # the GPU sends back segment records only (RXG_DLV_TCP_IN_PLACE)
            ns.set_rx_inplace(True)
        _run(ns, "gpu", seed)
    finally:
        ns.fini()


def test_stale_verdicts_after_close(ns_host):
    """a burst classified against one snapshot and delivered after a
    socket closed (which renumbers the later sockets) reaches the sockets the
    reference's per-frame lookups would pick, and the oracle's rcs"""
    ns, os_ = ns_host, O.Stack()
    fds = []
    for port in (1000, 1001, 1002):
        a = ns.socket(R.SOCK_DGRAM)
        assert a == os_.socket(2)
        ns.bind(a, L, port)
        os_.bind(a, _ip(L), _port(port))
        fds.append(a)
    frames = [F.udp_frame("10.0.0.1", 5555, L, port, bytes([port & 0xFF]) * 5)
              for port in (1001, 1002, 1000)]
    u, t, gen = ns.flows(with_gen=True)
    buf, off, lens = F.pack_frames(frames)
    v = ns.to_ids(O.Tables(u, t).classify(buf, off, lens, 6))   # flow ids 1, 2, 0
    assert list(v["flow_id"]) == [1, 2, 0]
    assert ns.close(fds[0]) == os_.close(fds[0]) == 0  # 1001 -> id 0, 1002 -> id 1
    rcs = np.zeros(3, np.int32)
    ns.deliver(frames, v, rcs, gen)
    assert list(rcs) == [os_.rx(f) for f in frames] == [0, 0, -3]
    for fd, port in ((fds[1], 1001), (fds[2], 1002)):
        r1, d1, _ = ns.recvfrom(fd, 64)
        r2, d2, _, _ = os_.recvfrom(fd, 64)
        assert (r1, d1) == (r2, d2) and d1[:5] == bytes([port & 0xFF]) * 5
