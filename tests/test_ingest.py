"""Host ingest: the C pcap reader/writer of librxgpu
(rxg_pcap_*) against the test-side Python pcap codec, and — on the GPU — the
pipelined host-buffer path (rxg_submit/rxg_wait, several bursts in flight)
fed from a pcap file, bit-exact against the oracle on the same file."""
import os
import struct

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxdist
import rxgpu as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _frames_of(pk, off, ln, unit_log2=6):
    return [pk[(int(o) << unit_log2):(int(o) << unit_log2) + int(n)].tobytes()
            for o, n in zip(off, ln)]


def _cfg4_frames(n, first=0):
    cfg = rxdist.gen_cfg("cfg4", n_udp=300, n_tcp=300)
    pk, off, ln = R.gen_host(cfg, first, n, 6)
    return cfg, _frames_of(pk, off, ln)


def test_pcap_write_matches_python_codec(tmp_path):
    _, frames = _cfg4_frames(500)
    buf, off, lens = F.pack_frames(frames, 6)
    p = str(tmp_path / "a.pcap")
    R.pcap_write(p, buf, off, lens, 6)
    assert F.read_pcap(p) == frames


@pytest.mark.parametrize("max_frames,cap_bytes,unit_log2", [(64, 1 << 20, 6), (1000, 40000, 4),
                                                            (7, 1 << 16, 5), (1, 2048, 6)])
def test_pcap_read_bursts(tmp_path, max_frames, cap_bytes, unit_log2):
    _, frames = _cfg4_frames(300)
    frames = frames + [b"", b"\x01" * 17] + F.read_pcap(os.path.join(GOLD, "edge.pcap"))
    p = str(tmp_path / "b.pcap")
    F.write_pcap(p, frames)
    pc = R.Pcap(p)
    got = []
    while True:
        pk, off, ln = pc.read_burst(max_frames, cap_bytes, unit_log2)
        if len(off) == 0:
            break
        assert len(off) <= max_frames
        unit = 1 << unit_log2
        for o, n in zip(off, ln):  # aligned starts, zero fill to the 16-B boundary
            s = int(o) << unit_log2
            assert s % unit == 0
            e16 = s + ((int(n) + 15) & ~15)
            assert not pk[s + int(n):e16].any()
        got += _frames_of(pk, off, ln, unit_log2)
    assert got == frames
    pc.rewind()
    pk, off, ln = pc.read_burst(3, 1 << 16, 6)
    assert _frames_of(pk, off, ln) == frames[:3]
    pc.close()


def test_pcap_big_endian_and_errors(tmp_path):
    frames = [F.udp_frame("10.0.0.1", 5555, "192.168.100.77", 8889, b"HELLO"), F.arp_frame(
        "1.1.1.1", "192.168.100.77")]
    p = str(tmp_path / "be.pcap")
    with open(p, "wb") as fh:  # big-endian file, nanosecond magic
        fh.write(struct.pack(">IHHiIII", 0xA1B23C4D, 2, 4, 0, 0, 65535, 1))
        for i, f in enumerate(frames):
            fh.write(struct.pack(">IIII", i, 0, len(f), len(f)) + f)
    pk, off, ln = R.Pcap(p).read_burst(16, 4096)
    assert _frames_of(pk, off, ln) == frames
    with open(p, "r+b") as fh:  # truncate the last record
        fh.truncate(os.path.getsize(p) - 3)
    with pytest.raises(R.RxgError):
        R.Pcap(p).read_burst(16, 4096)
    q = str(tmp_path / "raw.pcap")
    with open(q, "wb") as fh:  # LINKTYPE_RAW: not an Ethernet capture
        fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 101))
    with pytest.raises(R.RxgError):
        R.Pcap(q)
    with pytest.raises(R.RxgError):  # a frame larger than the whole buffer
        R.Pcap(os.path.join(GOLD, "edge.pcap")).read_burst(4, 32)


@pytest.mark.gpu
def test_pcap_pipeline_matches_oracle(tmp_path):
    """identical pcap input: the C reader + pipelined GPU bursts (5 in flight
    over 3 staging slots) give the oracle's verdicts and per-flow counts"""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    cfg, frames = _cfg4_frames(20000, first=777)
    frames += F.read_pcap(os.path.join(GOLD, "edge.pcap"))
    p = str(tmp_path / "c.pcap")
    F.write_pcap(p, frames)
    udp, tcb = R.gen_flows(cfg)
    fl = np.load(os.path.join(GOLD, "edge_flows.npz"))
    udp = np.concatenate([udp, fl["udp"]])
    tcb = np.concatenate([tcb, fl["tcb"]])
    buf, off, lens = F.pack_frames(frames, 6)
    want, wcnt = O.Tables(udp, tcb).classify(buf, off, lens, 6, counts=True)

    burst, cap = 4096, 4096 * 1536
    ctx = R.Context(0, max_pkts=burst, max_bytes=cap)
    try:
        ctx.flows_sync(udp, tcb)
        pc = R.Pcap(p)
        nb = (len(frames) + burst - 1) // burst
        bufs = [(torch.empty(cap, dtype=torch.uint8).pin_memory(),
                 torch.empty(burst, dtype=torch.int32).pin_memory(),
                 torch.empty(burst, dtype=torch.int16).pin_memory(),
                 torch.empty(burst * 16, dtype=torch.uint8).pin_memory()) for _ in range(nb)]
        tickets, sizes = [], []
        for b in bufs:  # every burst submitted before the first wait
            n, span = pc.read_burst_into(b[0].numpy(), b[1].numpy().view(np.uint32),
                                         b[2].numpy().view(np.uint16), 6)
            assert n > 0
            tickets.append(ctx.submit(b[0].data_ptr(), span, b[1].data_ptr(), b[2].data_ptr(), n,
                                      6, b[3].data_ptr()))
            sizes.append(n)
        assert tickets == sorted(tickets)
        for t in reversed(tickets):  # any wait order
            ctx.wait(t)
        got = np.concatenate([b[3].numpy()[:n * 16].view(R.VERDICT_DTYPE)
                              for b, n in zip(bufs, sizes)])
        assert got.tobytes() == want.tobytes()
        assert np.array_equal(ctx.flow_counts(), wcnt)
        pc.close()
    finally:
        ctx.close()


def test_cfg1_generator_is_one_flow():
    """BASELINE configs[0]: 100K x 64 B UDP, every frame the echo client's
    5-tuple 10.0.0.1:5555 -> 192.168.100.77:8889 (netfamily.c:227-229), every
    frame delivered to the one socket by the oracle"""
    cfg = rxdist.gen_cfg("cfg1")
    pk, off, ln = R.gen_host(cfg, 0, 5000, 6)
    fr = pk.reshape(5000, 64)
    assert np.all(ln == 64)
    assert np.all(fr[:, 26:30] == np.frombuffer(bytes([10, 0, 0, 1]), np.uint8))
    assert np.all(fr[:, 30:34] == np.frombuffer(bytes([192, 168, 100, 77]), np.uint8))
    assert np.all(fr[:, 34:36] == np.frombuffer((5555).to_bytes(2, "big"), np.uint8))
    assert np.all(fr[:, 36:38] == np.frombuffer((8889).to_bytes(2, "big"), np.uint8))
    udp, tcb = R.gen_flows(cfg)
    assert len(udp) == 1 and len(tcb) == 0
    v = O.Tables(udp, tcb).classify(pk, off, ln, 6)
    assert np.all(v["rc"] == 0) and np.all(v["flow_id"] == 0) and np.all(v["payload_len"] == 22)


@pytest.mark.gpu
def test_cfg1_pcap_through_gpu_matches_oracle(tmp_path):
    """cfg1 end to end: the 100K frames written with rxg_pcap_write, read back
    with rxg_pcap_read_burst into pinned memory, classified by rxg_classify
    (host-buffer path): every verdict equals the oracle's on the same bytes"""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    w = rxdist.WORKLOADS["cfg1"]
    cfg = rxdist.gen_cfg("cfg1")
    n = w["n"]
    pk, off, ln = R.gen_host(cfg, 0, n, 6)
    p = str(tmp_path / "cfg1.pcap")
    R.pcap_write(p, pk, off, ln, 6)
    pc = R.Pcap(p)
    buf = torch.zeros(n * 64 + 64, dtype=torch.uint8).pin_memory()
    po = torch.zeros(n, dtype=torch.int32).pin_memory()
    pl = torch.zeros(n, dtype=torch.int16).pin_memory()
    got_n, span = pc.read_burst_into(buf.numpy(), po.numpy().view(np.uint32),
                                     pl.numpy().view(np.uint16), 6)
    pc.close()
    assert got_n == n and span == n * 64
    udp, tcb = R.gen_flows(cfg)
    with R.Context(0, max_pkts=n, max_bytes=span) as ctx:
        ctx.flows_sync(udp, tcb)
        got = ctx.classify(buf.numpy()[:span], po.numpy().view(np.uint32),
                           pl.numpy().view(np.uint16), 6)
        want = O.Tables(udp, tcb).classify(buf.numpy()[:span], po.numpy().view(np.uint32),
                                           pl.numpy().view(np.uint16), 6)
        assert got.tobytes() == want.tobytes()
        assert np.all(got["rc"] == 0)
        assert np.array_equal(ctx.flow_counts(), np.array([n], np.uint64))


@pytest.mark.gpu
def test_host_buffers_end_exactly_at_the_last_frame():
    """a host burst whose buffer ends at the last frame's last byte (not on a
    16-B boundary): the copy in reads no byte past it, the TX copy back writes
    no byte past it (guard bytes after a view of exactly span bytes)"""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    frames = [F.udp_frame("10.0.0.1", 5555, "192.168.100.77", 8889, b"x" * k) for k in (5, 9, 30)]
    buf, off, lens = F.pack_frames(frames, 4)
    span = (int(off[-1]) << 4) + int(lens[-1])
    assert span % 16
    store = np.full(span + 32, 0xEE, np.uint8)  # guard bytes after the burst
    store[:span] = buf[:span]
    udp = np.zeros(1, R.UDP_SOCK_DTYPE)
    udp[0] = (R.ip_raw("192.168.100.77"), R.port_raw(8889), 17, 0)
    with R.Context(0, max_pkts=16, max_bytes=4096) as ctx:
        ctx.flows_sync(udp, None)
        got = ctx.classify(store[:span], off, lens, 4)
        want = O.Tables(udp, np.zeros(0, R.TCB_DTYPE)).classify(buf, off, lens, 4)
        assert got.tobytes() == want.tobytes()
        tx = store.copy()
        R._check(R._tx_cksum(ctx._h, tx.ctypes.data, span, off.ctypes.data, lens.ctypes.data,
                             len(off), 4), "rxg_tx_cksum")
        assert np.all(tx[span:] == 0xEE), "TX copy back wrote past the burst"
        assert np.array_equal(tx[:span], O.tx_cksum(buf, off, lens, 4)[:span])
