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
