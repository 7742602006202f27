"""Oracle pinning: the CPU restatement against every known-answer vector we
have (SURVEY.md §8(a) values recorded from the reference's compiled code,
RFC 1071, Microsoft RSS table) and the committed edge-case fixture."""
import json
import os

import numpy as np
import pytest

import frames as F
import oracle_bind as O
import rxgpu as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KATS = json.load(open(os.path.join(GOLD, "kats.json")))


@pytest.mark.parametrize("which", ["O2", "O0"])
@pytest.mark.parametrize("case", KATS["survey"] + KATS["rfc1071"], ids=lambda c: c["src"])
def test_cksum_kats(case, which):
    lib = O.lib if which == "O2" else O.lib_O0()
    b = bytes.fromhex(case["hex"])
    buf = np.frombuffer(b + bytes(8), np.uint8)
    if case["fn"] == "raw":
        got = lib.oracle_raw_cksum(buf.ctypes.data, len(b))
        assert got == case["expect"]
    elif case["fn"] == "udptcp":
        got = lib.oracle_ipv4_udptcp_cksum(buf.ctypes.data, buf.ctypes.data + 20)
        assert got == case["expect"], f"{case['src']}: {got:#06x} != {case['expect']:#06x}"
    else:  # IHL ignored: identical results for IHL 5 and 6
        b2 = np.frombuffer(bytes.fromhex(case["hex2"]) + bytes(8), np.uint8)
        assert lib.oracle_ipv4_udptcp_cksum(buf.ctypes.data, buf.ctypes.data + 20) == \
            lib.oracle_ipv4_udptcp_cksum(b2.ctypes.data, b2.ctypes.data + 20)


@pytest.mark.parametrize("case", KATS["ms_rss"], ids=lambda c: c["sip"])
def test_rss_kats(case):
    s, d = R.ip_raw(case["sip"]), R.ip_raw(case["dst"])
    sp, dp = R.port_raw(case["sport"]), R.port_raw(case["dport"])
    # zero ports contribute no input bits: the 12-byte hash equals the 8-byte IPv4 hash
    assert O.rss_hash(s, d, 0, 0) == case["ipv4"]
    assert O.rss_hash(s, d, sp, dp) == case["ipv4_tcp"]
    # the library's own (independently written) Toeplitz agrees
    assert R.rss_hash(s, d, 0, 0) == case["ipv4"]
    assert R.rss_hash(s, d, sp, dp) == case["ipv4_tcp"]


def _survey_flows():
    fl = KATS["survey_frames_flows"]
    udp = np.zeros(len(fl["udp"]), R.UDP_SOCK_DTYPE)
    for i, (ip, port) in enumerate(fl["udp"]):
        udp[i] = (R.ip_raw(ip), R.port_raw(port), 17, 0)
    tcb = np.zeros(len(fl["tcp"]), R.TCB_DTYPE)
    for i, (sip, dip, sport, dport, st) in enumerate(fl["tcp"]):
        tcb[i] = (R.ip_raw(sip), R.ip_raw(dip), R.port_raw(sport), R.port_raw(dport), st)
    return udp, tcb


def test_survey_frame_kats_oracle():
    udp, tcb = _survey_flows()
    frames = [bytes.fromhex(c["hex"]) for c in KATS["survey_frames"]]
    buf, off, lens = F.pack_frames(frames)
    v = O.Tables(udp, tcb).classify(buf, off, lens, 6)
    for c, vi in zip(KATS["survey_frames"], v):
        for k, want in c["expect"].items():
            if k == "dgram_len":
                assert vi["payload_len"] + 8 == want
            else:
                assert vi[k] == want, (c["src"], k, vi)


def test_edge_fixture_oracle_regression():
    flows = np.load(os.path.join(GOLD, "edge_flows.npz"))
    frames = F.read_pcap(os.path.join(GOLD, "edge.pcap"))
    buf, off, lens = F.pack_frames(frames)
    want = np.load(os.path.join(GOLD, "edge_verdicts.npy"))
    for which in (O.lib, O.lib_O0()):
        got = O.Tables(flows["udp"], flows["tcb"], which).classify(buf, off, lens, 6)
        assert got.tobytes() == want.tobytes()


def test_oracle_list_semantics():
    """first match in head-inserted order == newest creation index; listener
    pass ignores dst ip; exact pass ignores status (common.c:31-55, 97-108)"""
    L = R.ip_raw("192.168.100.77")
    udp = np.zeros(3, R.UDP_SOCK_DTYPE)
    udp[:] = [(L, R.port_raw(5), 17, 0), (L, R.port_raw(5), 17, 0), (L, R.port_raw(6), 17, 0)]
    tcb = np.zeros(3, R.TCB_DTYPE)
    tcb[:] = [(0, L, 0, R.port_raw(80), 1), (0, 0, 0, R.port_raw(80), 1),
              (7, L, 9, R.port_raw(80), 0)]
    t = O.Tables(udp, tcb)
    assert t.lookup_udp(L, R.port_raw(5)) == 1
    assert t.lookup_udp(L, R.port_raw(5), proto=6) == R.FLOW_NONE
    assert t.lookup_tcp(7, L, 9, R.port_raw(80)) == 2          # CLOSED still exact-matches
    assert t.lookup_tcp(8, 12345, 9, R.port_raw(80)) == 1      # newest listener, any dst ip
    assert t.lookup_tcp(8, L, 9, R.port_raw(81)) == R.FLOW_NONE


def test_pcap_roundtrip(tmp_path):
    fr = [F.udp_frame("1.2.3.4", 1, "5.6.7.8", 2, b"x" * n) for n in (0, 1, 17, 1000)]
    p = tmp_path / "t.pcap"
    F.write_pcap(str(p), fr, caplens=[len(f) - (i == 3) * 10 for i, f in enumerate(fr)])
    back = F.read_pcap(str(p))
    assert back[:3] == fr[:3] and back[3] == fr[3][:-10]
