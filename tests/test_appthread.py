"""bench.py's application lcore in C (tools/libappthread.so): it binds the
stack bench.py loaded (the same libnstack.so instance) and reads every
datagram the protocol thread delivers while it runs — what the two-thread
socket rows of the bench line count.  Host-only stack, oracle verdicts."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = "192.168.100.77"


@pytest.mark.skipif(bool(os.environ.get("NSTACK_LIB")),
                    reason="tools/libappthread.so binds the in-tree libnstack.so, not NSTACK_LIB's")
def test_c_application_thread_reads_everything():
    sys.path.insert(0, ROOT)
    import bench  # noqa: E402  (the loader and the result layout bench.py uses)
    ns = R.NStack(R.HOST_ONLY)
    try:
        lib = bench._appthread_lib()
        ports = list(range(20000, 20064))
        for p in ports:
            assert ns.bind(ns.socket(R.SOCK_DGRAM), L, p) == 0
        rng = np.random.default_rng(5)
        want_items = want_bytes = 0
        r = bench.AppResult()
        d0 = ns.stat(12)
        assert lib.app_start(-1, 0) == 0
        try:
            for _ in range(20):
                frames = []
                for k in range(256):
                    n = int(rng.integers(1, 600))
                    frames.append(F.udp_frame("10.0.0.%d" % (k % 200 + 1), 5555, L,
                                              ports[int(rng.integers(0, len(ports)))],
                                              bytes(rng.integers(0, 256, n, dtype=np.uint8))))
                    want_items += 1
                    want_bytes += n + 8  # nrecvfrom's length is the UDP length (udp.c:31-46)
                u, t, gen = ns.flows(with_gen=True)
                buf, off, lens = F.pack_frames(frames)
                v = ns.to_ids(O.Tables(u, t).classify(buf, off, lens, 6))
                rcs = np.zeros(len(frames), np.int32)
                ns.deliver(frames, v, rcs, gen)
                assert (rcs == 0).all()
        finally:
            assert lib.app_stop(C.byref(r)) == 0
        assert r.err == 0
        assert (r.items, r.bytes) == (want_items, want_bytes)
        assert ns.stat(12) - d0 == 20  # one per delivered burst (lock-free counter)
        assert r.passes >= 1
        assert lib.app_stop(C.byref(r)) == -1  # not running
    finally:
        ns.fini()


if __name__ == "__main__":
    pytest.main([__file__, "-q"])


def _fnv(b: bytes) -> int:
    h = 0xcbf29ce484222325
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def _udp_burst(ns, rng, ports, n):
    frames, pays = [], []
    for k in range(n):
        m = int(rng.integers(1, 200))
        pay = bytes(rng.integers(0, 256, m, dtype=np.uint8))
        frames.append(F.udp_frame("10.0.0.%d" % (k % 200 + 1), 5555, L,
                                  ports[int(rng.integers(0, len(ports)))], pay))
        pays.append(pay)
    u, t, gen = ns.flows(with_gen=True)
    buf, off, lens = F.pack_frames(frames)
    v = ns.to_ids(O.Tables(u, t).classify(buf, off, lens, 6))
    ns.deliver(frames, v, None, gen)
    return pays


@pytest.mark.parametrize("cap", [65536, 100], ids=["whole", "split"])
def test_drain_all_udp_reads_what_nrecvfrom_reads(cap):
    """drain_all takes a socket's datagrams out under one hold of its mutex
    and reads them after (drain_udp); what it returns is what nrecvfrom with
    the same buffer returns, socket by socket: the payload then zeros to
    dgram_len, a datagram longer than the buffer split (common.c:542-564)"""
    ports = list(range(21000, 21016))
    res = []
    for mode in ("drain", "recvfrom"):
        ns = R.NStack(R.HOST_ONLY)
        try:
            fds = [ns.socket(R.SOCK_DGRAM) for _ in ports]
            for fd, p in zip(fds, ports):
                assert ns.bind(fd, L, p) == 0
            rng = np.random.default_rng(9)
            pays = _udp_burst(ns, rng, ports, 600)
            if mode == "drain":
                g, nb, hs = ns.drain_all_sum(np.zeros(cap, np.uint8))
            else:
                g = nb = hs = 0
                for fd in fds:
                    while True:
                        r, d, _ = ns.recvfrom(fd, cap)
                        if r < 0:
                            break
                        g, nb = g + 1, nb + r
                        hs = (hs + _fnv(d[:min(r, cap)])) & 0xFFFFFFFFFFFFFFFF
            res.append((g, nb, hs))
            if cap == 65536:  # every datagram whole: payload + 8 zero bytes
                want = sum(_fnv(p + bytes(8)) for p in pays) & 0xFFFFFFFFFFFFFFFF
                assert (g, nb, hs) == (len(pays), sum(len(p) + 8 for p in pays), want)
        finally:
            ns.fini()
    assert res[0] == res[1], res
