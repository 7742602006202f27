"""The socket layer at scale, against its oracle (-m gpu; SURVEY.md §8(f)
ranks 2-3).

262,144 established tcbs (installed in the same order in both stacks, as a
SYN / ACK handshake would leave them: nstack_tcb_add / oracle_tcb_add) plus a
listener.  Every burst mixes, in one frame sequence:
  - data segments to the established tcbs: PSH data of assorted sizes, PSH|FIN
    in one segment, FIN, pure ACKs, a total_length shorter than the header
    (negative payload length: a 0-length EOF fragment), bad checksums;
  - SYNs from new clients (a tcb created mid-burst), the ACKs completing the
    previous burst's handshakes, FINs of connections established earlier, and
    the final ACKs of connections the application closed (LAST_ACK: the tcb
    freed mid-burst);
so the burst's own segments change the tcb list (g_burst_mutated: every later
segment is looked up again, now through the host image of the flow tables in
O(1) instead of the reference's list walks) while the established tcbs' data
takes the GPU's per-connection path (K4 segment sort + one batch per
connection).  Every per-frame return code, every accepted connection, every
nrecv result on the accepted connections, the tcb states (status, rcv_nxt,
snd_nxt, every queued ACK) of a sample of the established tcbs and of every
client, and what the application drains from all 262K tcbs are compared with
oracle/ref_stack.c (the reference's list walks, frame by frame).  Then the
time of a mutated burst is set against an unmutated one (printed)."""
import time

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

pytestmark = pytest.mark.gpu
L = "192.168.100.77"
N_EST = 262144
EST_PORT = 9998  # the established tcbs' local port (no listener on it)
LIS_PORT = 9999


def _est_key(k):
    return f"10.{(k >> 16) & 255}.{(k >> 8) & 255}.{k & 255}", 1024 + k % 50000


def _raw4(cip, cport, dport):
    return R.ip_raw(cip), R.ip_raw(L), R.port_raw(cport), R.port_raw(dport)


def _data_seg(rng, cip, cport, dport):
    p = bytes(rng.integers(0, 256, int(rng.choice([0, 1, 9, 120, 700, 1446])), dtype=np.uint8))
    kw = dict(seq=int(rng.integers(0, 2 ** 32)), ack=int(rng.integers(0, 2 ** 32)))
    r = rng.random()
    if r < 0.70:
        return F.tcp_frame(cip, cport, L, dport, p, flags=0x18, **kw)
    if r < 0.78:
        return F.tcp_frame(cip, cport, L, dport, b"", flags=0x10, **kw)
    if r < 0.83:
        return F.tcp_frame(cip, cport, L, dport, p, flags=0x19, **kw)       # PSH|FIN|ACK
    if r < 0.87:
        return F.tcp_frame(cip, cport, L, dport, b"", flags=0x11, **kw)     # FIN|ACK
    if r < 0.92:
        return F.tcp_frame(cip, cport, L, dport, p, flags=0x18, tl=30, tl_cksum=True,
                           **kw)  # plen < 0, checksum over tl - 20 bytes: rc 0
    if r < 0.96:
        return F.tcp_frame(cip, cport, L, dport, p, flags=0x18, data_off=0x60, **kw)
    return F.tcp_frame(cip, cport, L, dport, p + b"z", flags=0x18, corrupt=True, **kw)


class Stacks:
    def __init__(self):
        self.ns = R.NStack(0, max_burst=8192, max_bytes=8192 * 1536)
        self.os = O.Stack()
        a = self.ns.socket(R.SOCK_STREAM)
        assert a == self.os.socket(1)
        assert self.ns.bind(a, L, LIS_PORT) == self.os.bind(a, R.ip_raw(L), R.port_raw(LIS_PORT)) == 0
        assert self.ns.listen(a) == self.os.listen(a) == 0
        self.lfd = a
        add_ns, add_os = self.ns.lib.nstack_tcb_add, self.os.tcb_add
        for k in range(N_EST):
            cip, cport = _est_key(k)
            t = _raw4(cip, cport, EST_PORT)
            assert add_ns(*t, 4) == 0 and add_os(*t, 4) == 0
        self.conns = {}  # client key -> fd

    def burst(self, frames):
        want = [self.os.rx(f) for f in frames]
        n, rcs, _ = self.ns.rx_burst(frames)
        assert list(rcs) == want, [(i, int(rcs[i]), want[i]) for i in range(len(want))
                                   if rcs[i] != want[i]][:10]

    def accept_all(self):
        while True:
            fd, sip, sport = self.os.accept(self.lfd)
            if fd == O.WOULD_BLOCK:
                break
            got, a = self.ns.accept(self.lfd)
            assert (got, a.sin_addr, a.sin_port) == (fd, sip, sport)
            self.conns[(sip, sport)] = fd

    def recv_conns(self, n):
        for key, fd in list(self.conns.items()):
            while True:
                r1, d1 = self.ns.recv(fd, n, full=True)
                r2, d2 = self.os.recv(fd, n)
                if r2 == O.WOULD_BLOCK:
                    assert r1 == -1, key
                    break
                assert (r1, d1) == (r2, d2), (key, n, r1, r2)

    def compare(self, keys):
        assert self.ns.tcb_count() == self.os.tcb_count()
        for t in keys:
            want, got = self.os.tcb_state(*t), self.ns.tcb_state(*t)
            if want is None:
                assert got is None, t
                continue
            st, rn, sn, fd = want
            assert got is not None and (got[0], got[1], got[3]) == (st, rn, fd), (t, got, want)
            if sn is not None:
                assert got[2] == sn, (t, got, want)
            assert self.ns.tcb_sndq(*t) == self.os.tcb_sndq(*t), t


def test_socket_layer_256k_tcbs_churn_matches_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    rng = np.random.default_rng(44)
    st = Stacks()
    try:
        syn_pending, est_clients, fin_clients, last_ack = [], [], [], []
        all_clients = []
        for b in range(6):
            frames = []
            hot = [int(k) for k in rng.integers(0, N_EST, 150)]
            for _ in range(600):  # established traffic (several segments per tcb, in order)
                k = hot[int(rng.integers(len(hot)))]
                frames.append(_data_seg(rng, *_est_key(k), EST_PORT))
            sample = [_raw4(*_est_key(k), EST_PORT) for k in hot[:100]]
            ctl = []
            for i in range(10):  # new clients: SYN (a tcb created mid-burst)
                cip, cport = f"10.250.{b}.{i + 1}", 60000 + i
                ctl.append(F.tcp_frame(cip, cport, L, LIS_PORT, b"", flags=0x02,
                                       seq=int(rng.integers(0, 2 ** 31))))
                all_clients.append((cip, cport))
            for cip, cport in syn_pending:  # the previous burst's handshakes complete
                ctl.append(F.tcp_frame(cip, cport, L, LIS_PORT, b"", flags=0x10))
            for cip, cport in est_clients:  # data, then the client's FIN
                ctl.append(F.tcp_frame(cip, cport, L, LIS_PORT, b"hello " * 20, flags=0x18))
                ctl.append(F.tcp_frame(cip, cport, L, LIS_PORT, b"", flags=0x11))
            for cip, cport in last_ack:  # LAST_ACK + ACK: the tcb is freed mid-burst
                ctl.append(F.tcp_frame(cip, cport, L, LIS_PORT, b"", flags=0x10))
            for f in ctl:  # the control segments at random places among the data
                frames.insert(int(rng.integers(0, len(frames) + 1)), f)
            st.burst(frames)
            st.accept_all()
            st.recv_conns(int(rng.choice([7, 100, 4096])))
            # the application closes the connections whose FIN came this burst
            last_ack = []
            for cip, cport in est_clients:
                key = (R.ip_raw(cip), R.port_raw(cport))
                fd = st.conns.pop(key, None)
                if fd is not None:
                    assert st.ns.close(fd) == st.os.close(fd) == 0
                    last_ack.append((cip, cport))
            est_clients, syn_pending = syn_pending, [c for c in all_clients[-10:]]
            st.compare(sample + [_raw4(c, p, LIS_PORT) for c, p in all_clients])
            buf = np.zeros(65536, np.uint8)
            assert st.ns.drain_all(buf) == st.os.drain_all(buf), b
        ph = st.ns.last_burst_phases()
        # a mutated burst against an unmutated one (same data traffic), timed
        # on nstack only: the stacks part ways here
        times = {"unmutated": [], "mutated": []}
        for r in range(6):
            hot = [int(k) for k in rng.integers(0, N_EST, 500)]
            frames = [_data_seg(rng, *_est_key(hot[int(rng.integers(len(hot)))]), EST_PORT)
                      for _ in range(4000)]
            kind = "mutated" if r % 2 else "unmutated"
            if kind == "mutated":
                for i in range(16):
                    frames.insert(int(rng.integers(0, len(frames))),
                                  F.tcp_frame(f"10.251.{r}.{i + 1}", 61000 + i, L, LIS_PORT, b"",
                                              flags=0x02))
            arr, keep = st.ns.mbufs(frames)
            t0 = time.perf_counter()
            st.ns.rx_burst_mbufs(arr, len(frames))
            times[kind].append(time.perf_counter() - t0)
            st.ns.drain_all(np.zeros(65536, np.uint8))
        med = {k: float(np.median(v)) * 1e3 for k, v in times.items()}
        import json
        import os
        out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
        if os.path.isdir(out):  # the session's record
            with open(os.path.join(out, "sockets_scale_256k.json"), "w") as f:
                json.dump(dict(tcbs=N_EST, frames_per_burst=4000, rx_burst_ms_median=med,
                               ratio=med["mutated"] / med["unmutated"],
                               times_ms={k: [t * 1e3 for t in v] for k, v in times.items()},
                               last_compared_burst_phases_ms=ph), f, indent=1)
        print(f"\n256K tcbs: rx_burst of 4000 data segments {med['unmutated']:.3f} ms, "
              f"with 16 SYNs mid-burst {med['mutated']:.3f} ms "
              f"(x{med['mutated'] / med['unmutated']:.2f}); last compared burst phases {ph}")
        assert med["mutated"] < 1.5 * med["unmutated"], med
    finally:
        st.ns.fini()
