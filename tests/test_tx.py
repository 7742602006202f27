"""TX checksum generation: rte_ipv4_cksum + rte_ipv4_udptcp_cksum
filled into outgoing frames the way ng_encode_udp_apppkt (udp.c:84-95) and
ng_encode_tcp_apppkt (tcp.c:444-463) do.  The oracle's fill is pinned against
the pktgen's independently built checksums; the gfx950 kernel (K2) against
the oracle, bit-exact on whole buffers, and at BASELINE sizes through the
round trip "zero the fields -> K2 -> identical to the generated burst"."""
import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxdist
import rxgpu as R


def _zero_fields(pk, off, ln, unit_log2=6):
    z = pk.copy()
    for o, n in zip(off, ln):
        s = int(o) << unit_log2
        if n >= 34 and z[s + 12] == 8 and z[s + 13] == 0:
            z[s + 24:s + 26] = 0
            proto = z[s + 23]
            hole = 40 if proto == 17 else (50 if proto == 6 else None)
            if hole is not None and n >= hole + 2:
                z[s + hole:s + hole + 2] = 0
    return z


def _cfg(name):
    over = dict(bad_cksum_per10k=0)  # every generated checksum is then the correct one
    if name == "cfg5":
        over["n_tcp"] = 4096
    return rxdist.gen_cfg(name, **over)


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg4", "cfg5"])
def test_oracle_tx_restores_generated_frames(name):
    """the generator (rx_common.h) writes both checksums itself; zeroing them
    and running the oracle's TX fill must give the burst back byte for byte"""
    cfg = _cfg(name)
    n = {"cfg2": 3000, "cfg3": 800, "cfg4": 2000, "cfg5": 150}[name]
    pk, off, ln = R.gen_host(cfg, 4242, n, 6)
    z = _zero_fields(pk, off, ln)
    assert not np.array_equal(z, pk)
    assert np.array_equal(O.tx_cksum(z, off, ln, 6), pk)


def test_oracle_tx_reference_frames():
    """frames built like the reference's encoders (tests/frames.py) carry the
    checksums the oracle's fill computes; tl < 20 gives an L4 checksum of 0"""
    L = "192.168.100.77"
    fr = [F.udp_frame(L, 8889, "10.0.0.1", 5555, b"HELLO"),
          F.tcp_frame(L, 9999, "10.0.0.9", 40000, b"x" * 700, flags=0x18),
          F.udp_frame(L, 1, "10.0.0.1", 2, b""), F.arp_frame("1.1.1.1", L)]
    buf, off, lens = F.pack_frames(fr, 6)
    z = _zero_fields(buf, off, lens)
    assert np.array_equal(O.tx_cksum(z, off, lens, 6), buf)
    short = bytearray(F.udp_frame(L, 1, "10.0.0.1", 2, b"abc"))
    short[16:18] = (19).to_bytes(2, "big")
    buf, off, lens = F.pack_frames([bytes(short)], 6)
    t = O.tx_cksum(buf, off, lens, 6)
    assert t[40] == 0 and t[41] == 0


def _fuzz_burst(seed=3, n=4000):
    rng = np.random.default_rng(seed)
    L = "192.168.100.77"
    base = [F.udp_frame(L, 8889, "10.0.0.1", 5555, bytes(rng.integers(0, 256, 40, np.uint8))),
            F.tcp_frame(L, 9999, "10.0.0.9", 40000, bytes(rng.integers(0, 256, 1400, np.uint8))),
            F.tcp_frame(L, 9999, "10.0.0.9", 40000, b"y" * 17), F.arp_frame("1.2.3.4", L),
            F.icmp_frame(L, "1.2.3.4"), F.udp_frame(L, 1, "10.0.0.1", 2, b"z" * 8000)]
    frames, caps = [], []
    for _ in range(n):
        f = bytearray(base[rng.integers(len(base))])
        for _ in range(rng.integers(0, 3)):
            pos = int(rng.integers(0, min(len(f), 60)))
            f[pos] = int(rng.integers(0, 256))
        if rng.random() < 0.3:
            f[16:18] = int(rng.integers(0, 9100)).to_bytes(2, "big")
        frames.append(bytes(f))
        caps.append(len(f) if rng.random() < 0.85 else int(rng.integers(0, len(f) + 1)))
    return F.pack_frames(frames, 4, caplens=caps)


def test_oracle_tx_fuzz_is_idempotent():
    buf, off, lens = _fuzz_burst(n=600)
    once = O.tx_cksum(buf, off, lens, 4)
    assert not np.array_equal(once, buf)
    assert np.array_equal(O.tx_cksum(once, off, lens, 4), once)


@pytest.mark.gpu
def test_gpu_tx_cksum_matches_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    dev = torch.device("cuda", 0)
    buf, off, lens = _fuzz_burst()
    want = O.tx_cksum(buf, off, lens, 4)
    assert not np.array_equal(want, buf)
    with R.Context(0, max_pkts=len(off), max_bytes=len(buf) + 64) as ctx:
        got = ctx.tx_cksum(buf, off, lens, 4)                    # host path
        assert np.array_equal(got, want)
        # each default width (by len_hint), then every tuning variant of
        # tx_cksum.hip's k_tx table (forced through rxg_tune_tx)
        runs = [(hint, None) for hint in (64, 128, 354, 1500, 9000)] + \
            [(1500, v) for v in range(13)]
        with pytest.raises(R.RxgError):
            ctx.tune_tx(13)  # past the table
        try:
            for hint, v in runs:
                if v is not None:
                    ctx.tune_tx(v)
                d = torch.from_numpy(buf.copy()).to(dev)
                ctx.tx_cksum_dev(d, torch.from_numpy(off.view(np.int32)).to(dev),
                                 torch.from_numpy(lens.view(np.int16)).to(dev), len(off), 4, hint,
                                 torch.cuda.current_stream(dev).cuda_stream)
                torch.cuda.synchronize(dev)
                assert np.array_equal(d.cpu().numpy(), want), (hint, v)
        finally:
            ctx.tune_tx(R.TX_AUTO)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg5"])
def test_gpu_tx_round_trip_full_size(name):
    """BASELINE sizes: zero both checksum fields of every generated frame on
    the device, K2 fills them, the burst equals the generated one; K1 then
    verifies every L4 checksum (cksum_ok)"""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test needs a GPU (no fallback path exists)")
    dev = torch.device("cuda", 0)
    w = rxdist.WORKLOADS[name]
    cfg = _cfg(name)
    n = w["n"]
    pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n, dtype=torch.int32, device=dev)
    ln = torch.empty(n, dtype=torch.int16, device=dev)
    R.gen_dev(cfg, 0, n, pk, off, ln, w["unit_log2"])
    ref = pk.clone()
    slots = pk[:n * cfg.slot_bytes].view(n, cfg.slot_bytes)
    ipv4 = (slots[:, 12] == 8) & (slots[:, 13] == 0)
    slots[:, 24:26] = torch.where(ipv4[:, None], 0, slots[:, 24:26])
    udp = ipv4 & (slots[:, 23] == 17)
    tcp = ipv4 & (slots[:, 23] == 6)
    slots[:, 40:42] = torch.where(udp[:, None], 0, slots[:, 40:42])
    slots[:, 50:52] = torch.where(tcp[:, None], 0, slots[:, 50:52])
    assert not torch.equal(pk, ref)
    with R.Context(0) as ctx:
        ctx.tx_cksum_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"])
        torch.cuda.synchronize(dev)
        assert torch.equal(pk, ref)
        udp_f, tcb = R.gen_flows(cfg)
        ctx.flows_sync(udp_f, tcb)
        out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out)
        torch.cuda.synchronize(dev)
        v = out.view(n, 16)
        l4 = (v[:, 10] == R.CLS_UDP) | (v[:, 10] == R.CLS_TCP)
        assert bool((v[l4][:, 12] == 1).all())  # cksum_ok on every TCP/UDP frame
    del pk, ref, slots
    torch.cuda.empty_cache()
