"""CPU tests of the socket layer (libnstack, host C): the reference's
socket-call semantics (common.c:262-666) and UDP delivery with offload
semantics (udp.c:25-52).  Verdicts for delivery come from the oracle here
(no GPU); test_gpu_parity.py drives the same path through the GPU."""
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
    u, t = ns.flows()
    buf, off, lens = F.pack_frames(frames)
    return O.Tables(u, t).classify(buf, off, lens, 6)


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
    ns.deliver(frames, v)
    assert ns.stat(2) == 2          # classified, TCP state machine out of scope
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
