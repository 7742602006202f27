"""CPU tests of the socket layer (libnstack, host C): the reference's
socket-call semantics (common.c:262-666) and UDP delivery with offload
semantics (udp.c:25-52).  Verdicts for delivery come from the oracle here
(no GPU); test_gpu_parity.py drives the same path through the GPU."""
import struct

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

L = "192.168.100.77"


@pytest.fixture()
def ns():
    s = R.NStack(R.HOST_ONLY)
    yield s
    s.fini()


def _verdicts(ns, frames):
    """oracle verdicts against the stack's lists, flow ids as stable ids"""
    u, t = ns.flows()
    buf, off, lens = F.pack_frames(frames)
    return ns.to_ids(O.Tables(u, t).classify(buf, off, lens, 6))


def test_udp_echo_slice(ns):
    fd = ns.socket(R.SOCK_DGRAM)
    assert fd == 3  # first fd after D_DEFAULT_FD_NUM (common.c:72-85)
    assert ns.bind(fd, L, 8889) == 0
    frames = [F.udp_frame("10.0.0.1", 5555, L, 8889, b"HELLO"),
              F.udp_frame("10.0.0.1", 5555, L, 9, b"nobody"),
              F.udp_frame("10.0.0.2", 6666, L, 8889, b"x" * 100, corrupt=True)]
    v = _verdicts(ns, frames)
    assert list(v["rc"]) == [0, -3, 0]
    assert ns.deliver(frames, v) == 2
    r, data, a = ns.recvfrom(fd, 2048)
    # offload.length = dgram_len (udp.c:37): 5 payload bytes + 8 (zeros here)
    assert r == 13 and data == b"HELLO" + bytes(8)
    assert a.sin_port == R.port_raw(5555) and a.sin_addr == R.ip_raw("10.0.0.1")
    # split read (common.c:542-556): first len bytes, the rest stays queued
    r, data, _ = ns.recvfrom(fd, 30)
    assert r == 30 and data == b"x" * 30
    r, data, _ = ns.recvfrom(fd, 2048)
    assert r == 78 and data == b"x" * 69 + b"\x01"[:0] + data[69:]
    r, data, _ = ns.recvfrom(fd, 2048)
    assert r == -1  # empty + MSG_DONTWAIT
    assert ns.stat(0) == 2


def test_sendto_and_close(ns):
    fd = ns.socket(R.SOCK_DGRAM)
    ns.bind(fd, L, 8889)
    assert ns.sendto(fd, b"reply", "10.0.0.1", 5555) == 5
    assert ns.close(fd) == 0
    assert ns.close(fd) == -1
    assert ns.socket(R.SOCK_DGRAM) == fd  # fd released to the bitmap


def test_snapshot_creation_order_and_duplicates(ns):
    fds = [ns.socket(R.SOCK_DGRAM) for _ in range(3)]
    for fd, port in zip(fds, (100, 200, 100)):
        ns.bind(fd, L, port)
    u, _ = ns.flows()
    assert [R.port_raw(p) for p in (100, 200, 100)] == list(u["localport"])
    # newest of the duplicate key wins, exactly like the list walk
    v = _verdicts(ns, [F.udp_frame("1.1.1.1", 1, L, 100, b"dup")])
    assert v["flow_id"][0] == 2
    assert ns.deliver([F.udp_frame("1.1.1.1", 1, L, 100, b"dup")], v) == 1
    assert ns.recvfrom(fds[2], 64)[0] == 11
    assert ns.recvfrom(fds[0], 64)[0] == -1
    ns.close(fds[1])
    u, _ = ns.flows()
    assert [R.port_raw(p) for p in (100, 100)] == list(u["localport"])


def test_tcp_listen_accept(ns):
    lfd = ns.socket(R.SOCK_STREAM)
    assert ns.bind(lfd, L, 9999) == 0 and ns.listen(lfd) == 0
    _, t = ns.flows()
    assert len(t) == 1 and t["status"][0] == R.TCP_STATUS_LISTEN
    assert ns.tcb_add("10.0.0.9", L, 40000, 9999) == 0
    cfd, a = ns.accept(lfd)
    assert cfd > lfd and a.sin_port == R.port_raw(40000) and a.sin_addr == R.ip_raw("10.0.0.9")
    _, t = ns.flows()
    assert len(t) == 2
    frames = [F.tcp_frame("10.0.0.9", 40000, L, 9999, b"data"),
              F.tcp_frame("10.0.0.10", 1, L, 9999, b"syn to listener"),
              F.tcp_frame("10.0.0.9", 40000, L, 9999, b"bad", corrupt=True),
              F.tcp_frame("10.0.0.9", 40000, L, 80, b"closed port")]
    v = _verdicts(ns, frames)
    assert list(v["rc"]) == [0, 0, -1, -2]
    assert list(v["flow_id"][:2]) == [1, 0]
    rcs = np.zeros(len(frames), np.int32)
    ns.deliver(frames, v, rcs)
    assert list(rcs) == [0, 0, -1, -2]
    assert ns.stat(2) == 2          # dispatched to the state machine
    assert ns.recv(cfd, 64) == (4, b"data")   # ESTABLISHED + PSH (tcp.c:228-252)
    assert ns.recv(cfd, 64)[0] == -1
    assert ns.send(cfd, b"hi") == 2
    assert ns.close(cfd) == 0       # FIN queued, tcb stays until LAST_ACK
    _, t = ns.flows()
    assert len(t) == 2
    assert ns.close(lfd) == 0       # listener removed
    _, t = ns.flows()
    assert len(t) == 1


def test_rx_burst_needs_gpu(ns):
    ns.socket(R.SOCK_DGRAM)
    with pytest.raises(R.RxgError):
        ns.rx_burst([F.udp_frame("1.1.1.1", 1, L, 2, b"x")])


def test_pipelined_receive_needs_gpu(ns):
    """nstack_rx_submit on a host-only stack: the library refuses the burst
    (RXG_ENODEV), nothing is left pending, a complete has nothing to
    deliver (RXG_EINVAL) and host-verdict delivery still works"""
    ns.socket(R.SOCK_DGRAM)
    with pytest.raises(R.RxgError):
        ns.rx_submit([F.udp_frame("1.1.1.1", 1, L, 2, b"x")])
    assert ns.rx_pending() == 0
    assert ns.lib.nstack_rx_complete() == -22
    assert _deliver(ns, [F.udp_frame("1.1.1.1", 1, L, 2, b"x")]) == [-3]


def _deliver(ns, frames):
    v = _verdicts(ns, frames)
    rcs = np.zeros(len(frames), np.int32)
    ns.deliver(frames, v, rcs)
    return list(rcs)


def _status(ns):
    _, t = ns.flows()
    return {(int(x["sip"]), int(x["sport"])): int(x["status"]) for x in t}


SYN, ACK, PSH, FIN = 0x02, 0x10, 0x08, 0x01
C_IP, C_PORT = "10.0.0.9", 40000


def _seg(flags, payload=b"", seq=1000, ack=2000):
    return F.tcp_frame(C_IP, C_PORT, L, 9999, payload, flags=flags, seq=seq, ack=ack)


def test_tcp_handshake_in_one_burst(ns):
    """SYN and its ACK in the same burst: the ACK must see the tcb the SYN
    created (tcp.c:43-131 run frame by frame), though the burst was classified
    against the list without it"""
    lfd = ns.socket(R.SOCK_STREAM)
    ns.bind(lfd, L, 9999)
    ns.listen(lfd)
    key = (R.ip_raw(C_IP), R.port_raw(C_PORT))
    assert _deliver(ns, [_seg(SYN), _seg(ACK, seq=1001)]) == [0, 0]
    assert _status(ns)[key] == 4  # SYN_RCVD -> ESTABLISHED
    cfd, a = ns.accept(lfd)
    assert cfd > lfd and a.sin_port == R.port_raw(C_PORT)


def test_tcp_session_data_fin_close(ns):
    lfd = ns.socket(R.SOCK_STREAM)
    ns.bind(lfd, L, 9999)
    ns.listen(lfd)
    key = (R.ip_raw(C_IP), R.port_raw(C_PORT))
    assert _deliver(ns, [_seg(SYN)]) == [0]
    assert _status(ns)[key] == 2  # SYN_RCVD, SYN|ACK queued
    assert _deliver(ns, [_seg(ACK, seq=1001)]) == [0]
    cfd, _ = ns.accept(lfd)
    # two data segments and a FIN in one burst; a corrupted one is dropped (-1)
    burst = [_seg(PSH | ACK, b"hello ", seq=1001),
             F.tcp_frame(C_IP, C_PORT, L, 9999, b"bad", flags=PSH | ACK, corrupt=True),
             _seg(PSH | ACK, b"world", seq=1007), _seg(FIN | ACK, seq=1012)]
    assert _deliver(ns, burst) == [0, -1, 0, 0]
    assert _status(ns)[key] == 9              # CLOSE_WAIT
    assert ns.stat(4) == 3                    # two payloads + the EOF marker
    # split read (common.c:483-496): copies 3 bytes, returns the REMAINING
    # length, and re-enqueues the rest at the ring's tail
    r, data = ns.recv(cfd, 3)
    assert r == 3 and data == b"hel"
    assert ns.recv(cfd, 64) == (5, b"world")
    assert ns.recv(cfd, 64) == (0, b"")       # EOF marker of the FIN
    assert ns.recv(cfd, 64) == (3, b"lo ")


def test_tcp_last_ack_frees_tcb_mid_burst(ns):
    lfd = ns.socket(R.SOCK_STREAM)
    ns.bind(lfd, L, 9999)
    ns.listen(lfd)
    ns.tcb_add(C_IP, L, C_PORT, 9999)
    cfd, _ = ns.accept(lfd)
    assert ns.close(cfd) == 0                 # FIN queued, LAST_ACK
    key = (R.ip_raw(C_IP), R.port_raw(C_PORT))
    assert _status(ns)[key] == 10
    # the final ACK frees the tcb; the next segment of the same burst falls
    # through to the listener (no SYN: ignored), a segment to a port with no
    # listener is -2
    burst = [_seg(ACK), _seg(PSH | ACK, b"late"),
             F.tcp_frame(C_IP, C_PORT, L, 80, b"x", flags=PSH | ACK)]
    assert _deliver(ns, burst) == [0, 0, -2]
    assert key not in _status(ns)
    assert len(ns.flows()[1]) == 1            # the listener only


def test_tcp_nrecv_eof_after_fin(ns):
    lfd = ns.socket(R.SOCK_STREAM)
    ns.bind(lfd, L, 9999)
    ns.listen(lfd)
    ns.tcb_add(C_IP, L, C_PORT, 9999)
    cfd, _ = ns.accept(lfd)
    assert _deliver(ns, [_seg(PSH | ACK, b"abc"), _seg(FIN | ACK, seq=1003)]) == [0, 0]
    assert ns.recv(cfd, 64) == (3, b"abc")
    assert ns.recv(cfd, 64) == (0, b"")       # 0-length fragment = EOF (common.c:497-501)
    assert ns.recv(cfd, 64)[0] == -1


# ---- TX: udp_out / tcp_out (udp.c:59-164, tcp.c:420-555), ARP (common.c:145-260)
LMAC, PMAC = F.LOCAL_MAC, F.PEER_MAC


def _ipv4(tl, proto, src, dst):  # ng_encode_*: id 0, no DF, ttl 64, checksum left 0
    return struct.pack(">BBHHHBBH4s4s", 0x45, 0, tl, 0, 0, 64, proto, 0, F.ip4(src), F.ip4(dst))


def _arp_request(sip, tip):  # ng_encode_arp_pkt with the all-ones target MAC
    return (bytes(6) + LMAC + b"\x08\x06" + struct.pack(">HHBBH", 1, 0x0800, 6, 4, 1) + LMAC +
            F.ip4(sip) + b"\xff" * 6 + F.ip4(tip))


def test_tx_udp_arp_then_datagram(ns):
    ns.set_local(L, LMAC)
    fd = ns.socket(R.SOCK_DGRAM)
    ns.bind(fd, L, 8889)
    assert ns.sendto(fd, b"reply", "10.0.0.1", 5555) == 5
    assert ns.tx_burst() == [_arp_request(L, "10.0.0.1")]     # no ARP entry yet
    arp_in = F.arp_frame("10.0.0.1", L)                        # the peer's ARP frame teaches it
    _deliver(ns, [arp_in])
    want = (PMAC + LMAC + b"\x08\x00" + _ipv4(33, 17, L, "10.0.0.1") +
            struct.pack(">HHHH", 8889, 5555, 13, 0) + b"reply")
    fr = ns.tx_burst()
    assert fr == [want]
    assert ns.tx_burst() == []
    # the oracle's TX fill makes it a frame whose checksums verify on rx
    buf, off, lens = F.pack_frames(fr, 6)
    filled = O.tx_cksum(buf, off, lens, 6)
    v = O.Tables(np.zeros(0, R.UDP_SOCK_DTYPE), np.zeros(0, R.TCB_DTYPE)).classify(
        filled, off, lens, 6)
    assert v["cksum_ok"][0] == 1 and v["rc"][0] == -3


def test_tx_one_datagram_per_socket_per_pass(ns):
    ns.set_local(L, LMAC)
    ns.arp_insert("10.0.0.1", PMAC)
    a, b = ns.socket(R.SOCK_DGRAM), ns.socket(R.SOCK_DGRAM)
    ns.bind(a, L, 1000)
    ns.bind(b, L, 2000)
    for fd, p in ((a, b"a1"), (a, b"a2"), (b, b"b1")):
        ns.sendto(fd, p, "10.0.0.1", 7777)
    first = ns.tx_burst()
    assert [f[42:] for f in first] == [b"b1", b"a1"]           # newest socket first (LL_ADD)
    assert [f[42:] for f in ns.tx_burst()] == [b"a2"]


def test_tx_tcp_synack_and_data(ns):
    ns.set_local(L, LMAC)
    ns.arp_insert("10.0.0.9", PMAC)
    lfd = ns.socket(R.SOCK_STREAM)
    ns.bind(lfd, L, 9999)
    ns.listen(lfd)
    _deliver(ns, [_seg(SYN, seq=5000)])
    fr = ns.tx_burst()
    assert len(fr) == 1
    f = fr[0]
    assert f[:14] == PMAC + LMAC + b"\x08\x00"
    assert f[14:34] == _ipv4(40, 6, L, "10.0.0.9")
    sport, dport, seq, ack, doff, flags = struct.unpack(">HHIIBB", f[34:48])
    assert (sport, dport, ack, doff, flags) == (9999, 40000, 5001, 0x50, SYN | ACK)
    assert f[48:50] == (14600).to_bytes(2, "little")           # rx_win without htons (tcp.c:454)
    assert f[50:54] == bytes(4)                                 # checksum 0, urp 0
    _deliver(ns, [_seg(ACK, seq=5001, ack=seq + 1)])
    cfd, _ = ns.accept(lfd)
    assert ns.send(cfd, b"hi there") == 8
    f = ns.tx_burst()[0]
    assert f[47] == PSH | ACK and f[54:] == b"hi there" and len(f) == 62
    assert struct.unpack(">I", f[42:46])[0] == 5001             # acknum = rcv_nxt
