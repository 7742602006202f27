"""The lane kernel's UDP decision from its LDS tables, restated on the host
and checked against the oracle (CPU; the kernel itself: test_gpu_parity.py
test_udp_port_window).

Small socket sets (<= 1024) give the lane kernel a compact UDP table (linear
probing under the context's hash seed) and, with the port tables, a port
window of the main address's bound ports (rx_flows.h small_rebuild).  The
kernel decides a UDP frame (csrc/rx_classify.hip lane_verdict, LDT branch):
  - with a window, on the window's address: the window entry, a miss outside;
  - with a window, elsewhere: a miss unless some compact key is bound off the
    window's address (udpc_other), else the probe;
  - without a window: the probe.
The tables are read back through rxg_ft_dump (which 3 / 4) from a host-only
context; every frame's flow must equal the oracle's lookup
(get_hostinfo_fromip_port, common.c:97-108: exact (dip, dport, proto),
newest socket wins).  Seeds: each context draws its own, so the probe
sequences differ per context; several contexts per case."""
import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

M32 = 0xFFFFFFFF
NONE = 0xFFFFFFFF


def _hash3s(seed, a, b, c):
    """rx_hash3s (csrc/rx_common.h)"""
    h = (seed ^ a) & M32
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 15
    h = (h + b) & M32
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 13
    h = (h + c) & M32
    h = (h * 0x27D4EB2F) & M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    return h


def _bswap16(x):
    return ((x & 0xFF) << 8) | (x >> 8)


def _lane_udp_flow(t3, i3, t4, dip, dport):
    """the LDT branch of lane_verdict: (flow, probes made)"""
    mask, probe, seed, other, wlo, wn, wdip = (int(x) for x in i3[:7])
    lt = t3.reshape(-1, 2)
    lw = t4.view(np.uint16)[:wn]
    k = (_bswap16(dport) - wlo) & M32
    win = wn != 0
    if win and dip == wdip:
        e = int(lw[k]) if k < wn else 0xFFFF
        return (NONE if e == 0xFFFF else e), 0
    if win and other == 0:
        return NONE, 0
    i = _hash3s(seed, dip, dport, 17) & mask
    for pr in range(probe):
        x, y = int(lt[i, 0]), int(lt[i, 1])
        if y == M32:
            return NONE, pr + 1
        if x == dip and (y & 0xFFFF) == dport:
            return y >> 16, pr + 1
        i = (i + 1) & mask
    return NONE, probe


def _case(kind):
    L, L2, L3 = "192.168.100.77", "10.9.9.9", "172.16.0.1"
    if kind == "one_address":  # cfg2's shape: 1024 sockets on one address
        return [(L, 20000 + k) for k in range(1024)]
    if kind == "one_address_sparse":
        return [(L, 30000 + 3 * k) for k in range(300)] + [(L, 30000 + 30 * k) for k in range(10)]
    if kind == "two_addresses":
        return ([(L, 30000 + 3 * k) for k in range(300)] + [(L2, 30000 + 21 * k) for k in range(20)]
                + [(L2, 5555)])
    if kind == "wide":  # ports span more than the 4096-port window: none built
        return [(L, 30000 + 3 * k) for k in range(300)] + [(L, 40000), (L3, 7)]
    raise ValueError(kind)


@pytest.mark.parametrize("tables", [0, R.TT_NO_UDP_PORT], ids=["port_tables", "no_port_tables"])
@pytest.mark.parametrize("kind", ["one_address", "one_address_sparse", "two_addresses", "wide"])
def test_lane_udp_rule_matches_oracle(kind, tables):
    L, L2, L3 = "192.168.100.77", "10.9.9.9", "172.16.0.1"
    socks = _case(kind)
    udp = np.zeros(len(socks), R.UDP_SOCK_DTYPE)
    for i, (ip, port) in enumerate(socks):
        udp[i] = (R.ip_raw(ip), R.port_raw(port), 17, 0)
    tcb = np.zeros(0, R.TCB_DTYPE)
    rng = np.random.default_rng(11)
    keys = []
    for _ in range(3000):
        r = rng.integers(0, 6)
        if r < 3:
            ip, port = socks[int(rng.integers(0, len(socks)))]
        elif r == 3:
            ip, port = L, int(rng.choice([7, 19999, 21024, 29999, 33001, 40000, 50000]))
        elif r == 4:
            ip, port = L2, int(rng.choice([5555, 30021, 30003, 7]))
        else:
            ip, port = L3, int(rng.choice([7, 30003, 20000]))
        keys.append((ip, port))
    frames = [F.udp_frame("10.0.0.1", 1000 + i, ip, port, b"p" * 18) for i, (ip, port) in enumerate(keys)]
    buf, off, lens = F.pack_frames(frames, 6)
    want = O.Tables(udp, tcb).classify(buf, off, lens, 6)
    probes_max = 0
    for _ in range(4):  # contexts: a seed each
        ctx = R.Context(R.HOST_ONLY)
        try:
            ctx.tune_tables(tables)
            ctx.flows_sync(udp, tcb)
            t3, i3 = R.ft_dump(ctx._h, 3, False)
            t4, i4 = R.ft_dump(ctx._h, 4, False)
        finally:
            ctx.close()
        assert int(i3[7]) > 0, "no compact table for a small socket set"
        assert (int(i4[5]) > 0) == (tables == 0 and kind != "wide"), (kind, tables, i4)
        for j, (ip, port) in enumerate(keys):
            flow, pr = _lane_udp_flow(t3, i3, t4, R.ip_raw(ip), R.port_raw(port))
            probes_max = max(probes_max, pr)
            assert flow == int(want["flow_id"][j]), (kind, tables, ip, port, flow, want[j])
    if tables == 0 and kind.startswith("one_address"):
        assert probes_max == 0  # every frame decided by the window or as a miss


if __name__ == "__main__":
    pytest.main([__file__, "-q"])
