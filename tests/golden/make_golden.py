#!/usr/bin/env python3
"""Writes the committed golden fixtures of tests/golden/.

1. kats.json — known-answer vectors whose EXPECTED values are transcribed
   literals, never computed here:
     * "survey"  : values SURVEY.md §8(a) ("Known-answer edge cases", lines
                   295-307) records from the reference's own compiled
                   rte_ipv4_udptcp_cksum / udp_process / tcp_process;
     * "rfc1071" : RFC 1071 §3 numerical example;
     * "ms_rss"  : Microsoft "Verifying the RSS Hash Calculation" IPv4 table
                   (standard 40-byte key).
   The inputs are built below from the SURVEY's description of each case.
2. edge.pcap + edge_flows.npz + edge_verdicts.npy — a regression fixture of
   edge-case frames (truncation, IHL, negative TCP payload, short UDP,
   duplicates, listeners, ARP/ICMP/VLAN).  Its verdicts are produced by the
   oracle (oracle/ref_cpu.c) and are labelled "oracle-derived": they pin the
   GPU path and future oracle edits to today's restatement, not to the
   reference (which cannot be run here).

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)),
                                "dpdk-tcp-udp_protocol_stack_amd"))

import frames as F  # noqa: E402


def ipbuf(tl: int, proto: int, l4: bytes, *, ver_ihl=0x45, fill=0, size=None) -> bytes:
    """IPv4 header at offset 0 followed by L4 bytes; all other bytes = fill."""
    size = size if size is not None else 20 + max(len(l4), 2) + 8
    b = bytearray([fill]) * size
    b[0] = ver_ihl
    b[2:4] = struct.pack(">H", tl)
    b[9] = proto
    b[20:20 + len(l4)] = l4
    return bytes(b)


def survey_kats():
    out = []
    # SURVEY.md:296  tl=19 -> 0x0000 (rte_ip.h:330-331 early return)
    out.append(dict(src="survey:296", fn="udptcp", hex=ipbuf(19, 6, b"").hex(), expect=0x0000))
    # SURVEY.md:297  tl=20 TCP, zero L4 -> 0xF9FF
    out.append(dict(src="survey:297", fn="udptcp", hex=ipbuf(20, 6, b"").hex(), expect=0xF9FF))
    # SURVEY.md:298  TCP L4 bytes ff f7, tl=22, zero addresses -> 0x0000 (stays 0)
    out.append(dict(src="survey:298", fn="udptcp", hex=ipbuf(22, 6, b"\xff\xf7").hex(),
                    expect=0x0000))
    # SURVEY.md:299  UDP L4 bytes ff ec, tl=22 -> 0xFFFF; same bytes proto 6 -> 0x0B00
    out.append(dict(src="survey:299", fn="udptcp", hex=ipbuf(22, 17, b"\xff\xec").hex(),
                    expect=0xFFFF))
    out.append(dict(src="survey:299", fn="udptcp", hex=ipbuf(22, 6, b"\xff\xec").hex(),
                    expect=0x0B00))
    # SURVEY.md:300  IHL=6 vs IHL=5, same bytes -> identical (IHL ignored)
    a = ipbuf(40, 6, bytes(range(1, 21)), ver_ihl=0x45)
    b = ipbuf(40, 6, bytes(range(1, 21)), ver_ihl=0x46)
    out.append(dict(src="survey:300", fn="udptcp_same", hex=a.hex(), hex2=b.hex(), expect=None))
    # SURVEY.md:301  odd L4 {0x12}, tl=21, TCP -> 0xF8ED
    out.append(dict(src="survey:301", fn="udptcp", hex=ipbuf(21, 6, b"\x12").hex(),
                    expect=0xF8ED))
    # SURVEY.md:302  9000-B buffer, every byte 0xA5 except ver_ihl=0x45, tl=8986,
    # proto=6 (cksum field left at 0xA5A5) -> 0x9982
    big = bytearray([0xA5]) * 9000
    big[0] = 0x45
    big[2:4] = struct.pack(">H", 8986)
    big[9] = 6
    out.append(dict(src="survey:302", fn="udptcp", hex=bytes(big).hex(), expect=0x9982))
    return out


def rfc_kats():
    # RFC 1071 §3 example: 00 01 f2 03 f4 f5 f6 f7 -> sum 0xddf2 in big-endian
    # order; the native little-endian word view used by the reference gives the
    # byte-swapped sum 0xf2dd (RFC 1071 §2(B), byte-order independence).
    return [dict(src="rfc1071:3", fn="raw", hex="0001f203f4f5f6f7", expect=0xF2DD)]


def rss_kats():
    # Microsoft RSS verification table, IPv4 (dst, src -> IPv4 hash, IPv4+TCP hash)
    rows = [
        ("161.142.100.80", 1766, "66.9.149.187", 2794, 0x323E8FC2, 0x51CCC178),
        ("65.69.140.83", 4739, "199.92.111.2", 14230, 0xD718262A, 0xC626B0EA),
        ("12.22.207.184", 38024, "24.19.198.95", 12898, 0xD2D0A5DE, 0x5C2B394A),
        ("209.142.163.6", 2217, "38.27.205.30", 48228, 0x82989176, 0xAFC7327F),
        ("202.188.127.2", 1303, "153.39.163.191", 44251, 0x5D1809C5, 0x10E828A2),
    ]
    return [dict(src="ms_rss", dst=d, dport=dp, sip=s, sport=sp, ipv4=h4, ipv4_tcp=h4t)
            for d, dp, s, sp, h4, h4t in rows]


def frame_kats():
    """SURVEY.md:303-307 — verdict-level expectations on full frames."""
    L = "192.168.100.77"
    cases = []
    # :303 UDP with corrupted checksum on a bound port -> rc 0
    cases.append(dict(src="survey:303", hex=F.udp_frame("10.0.0.1", 5555, L, 8889, b"hello world",
                                                         corrupt=True).hex(),
                      expect=dict(rc=0, cls=3, payload_off=42, payload_len=11)))
    # :304 TCP with one flipped bit -> rc -1
    cases.append(dict(src="survey:304", hex=F.tcp_frame("10.0.0.9", 40000, L, 9999, b"abcdef",
                                                         corrupt=True).hex(),
                      expect=dict(rc=-1, cls=4)))
    # :305 TCP to a port with no listener -> rc -2
    cases.append(dict(src="survey:305", hex=F.tcp_frame("10.0.0.9", 40000, L, 1234, b"x").hex(),
                      expect=dict(rc=-2, cls=4)))
    # :306 UDP to an unbound port -> rc -3
    cases.append(dict(src="survey:306", hex=F.udp_frame("10.0.0.1", 5555, L, 1111, b"x").hex(),
                      expect=dict(rc=-3, cls=3)))
    # :307 UDP "HELLO" (dgram_len 13) -> offload.length 13, 5 payload bytes copied
    cases.append(dict(src="survey:307", hex=F.udp_frame("10.0.0.1", 5555, L, 8889, b"HELLO").hex(),
                      expect=dict(rc=0, cls=3, payload_off=42, payload_len=5, dgram_len=13)))
    # flow set for these frames: the reference's UDP echo socket (netfamily.c:227-229)
    # and a listener on :9999 (netfamily.c:270, tcp_server_entry)
    flows = dict(udp=[[L, 8889]], tcp=[["0.0.0.0", L, 0, 9999, 1]])
    return cases, flows


def edge_frames():
    L = "192.168.100.77"
    fr, caps = [], []

    def add(f, cap=None):
        fr.append(f)
        caps.append(len(f) if cap is None else cap)

    add(F.udp_frame("10.0.0.1", 5555, L, 8889, b"HELLO"))
    add(F.udp_frame("10.0.0.1", 5555, L, 8889, b""))                  # dgram_len 8 -> rc -2
    add(F.udp_frame("10.0.0.1", 5555, L, 8889, b"abc", dgram_len=5))  # dgram_len < 8
    add(F.udp_frame("10.0.0.1", 5555, L, 8889, b"abc", dgram_len=200))  # copy past frame
    add(F.udp_frame("10.0.0.1", 5555, L, 8889, bytes(range(100)), corrupt=True))
    add(F.udp_frame("10.0.0.2", 6000, L, 20001, b"dup"))              # duplicate key -> newest
    add(F.udp_frame("10.0.0.2", 6000, "192.168.100.78", 8889, b"other ip"))
    add(F.tcp_frame("10.0.0.9", 40000, L, 9999, b"payload"))          # exact tcb
    add(F.tcp_frame("10.0.0.10", 40001, L, 9999, b"to listener"))     # listener fallback
    add(F.tcp_frame("10.0.0.10", 40001, "1.2.3.4", 9999, b"dst ignored"))  # listener, dst ip ignored
    add(F.tcp_frame("10.0.0.9", 40000, L, 9999, b"bad", corrupt=True))
    add(F.tcp_frame("10.0.0.9", 40000, L, 7777, b"no tcb"))
    add(F.tcp_frame("10.0.0.9", 40000, L, 9999, b"", data_off=0xF0, pad_options=False))  # tl-20-hl < 0
    add(F.tcp_frame("10.0.0.9", 40000, L, 9999, bytes(1400)))
    add(F.tcp_frame("10.0.0.9", 40000, L, 9999, b"odd!!"))            # odd L4 length
    f = bytearray(F.tcp_frame("10.0.0.9", 40000, L, 9999, b"ihl6"))
    f[14] = 0x46                                                      # IHL ignored
    add(bytes(f))
    add(F.tcp_frame("10.0.0.9", 40000, L, 9999, bytes(range(200))), cap=100)  # truncated capture
    add(F.udp_frame("10.0.0.1", 5555, L, 8889, b"x" * 40, tl=15))    # tl < 20
    add(F.arp_frame("192.168.100.1", L))
    add(F.icmp_frame("192.168.100.1", L))
    vl = F.ether(b"\x00\x64\x08\x00" + bytes(46), ethertype=0x8100)   # VLAN tagged -> KNI
    add(vl)
    add(bytes(10), cap=10)                                            # runt
    add(F.tcp_frame("0.0.0.0", 0, L, 9999, b"hits listener exactly"))  # exact match on listener
    return fr, caps


def edge_flows():
    import rxgpu as R
    L = R.ip_raw("192.168.100.77")
    udp = np.zeros(4, R.UDP_SOCK_DTYPE)
    udp[0] = (L, R.port_raw(8889), 17, 0)
    udp[1] = (L, R.port_raw(20001), 17, 0)
    udp[2] = (L, R.port_raw(20001), 17, 0)   # same key, newer -> wins
    udp[3] = (L, R.port_raw(20002), 6, 0)    # not UDP: never matches
    tcb = np.zeros(4, R.TCB_DTYPE)
    tcb[0] = (0, L, 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)
    tcb[1] = (R.ip_raw("10.0.0.9"), L, R.port_raw(40000), R.port_raw(9999), 4)
    tcb[2] = (0, L, 0, R.port_raw(9999), R.TCP_STATUS_LISTEN)   # newer listener wins
    tcb[3] = (R.ip_raw("10.0.0.9"), L, R.port_raw(40000), R.port_raw(7777), 0)  # CLOSED
    return udp, tcb


def main():
    kats = dict(survey=survey_kats(), rfc1071=rfc_kats(), ms_rss=rss_kats())
    fk, fl = frame_kats()
    kats["survey_frames"] = fk
    kats["survey_frames_flows"] = fl
    with open(os.path.join(HERE, "kats.json"), "w") as fh:
        json.dump(kats, fh, indent=1)

    import oracle_bind as O
    fr, caps = edge_frames()
    F.write_pcap(os.path.join(HERE, "edge.pcap"), fr, caps)
    udp, tcb = edge_flows()
    np.savez(os.path.join(HERE, "edge_flows.npz"), udp=udp, tcb=tcb)
    frames = F.read_pcap(os.path.join(HERE, "edge.pcap"))
    buf, off, lens = F.pack_frames(frames, 6)
    v = O.Tables(udp, tcb).classify(buf, off, lens, 6)
    np.save(os.path.join(HERE, "edge_verdicts.npy"), v)
    print(f"wrote kats.json, edge.pcap ({len(frames)} frames), edge_verdicts.npy")


if __name__ == "__main__":
    main()
