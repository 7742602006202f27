"""Small frame builder for tests (Ether / IPv4 / UDP / TCP / ARP), plus a
classic-pcap reader/writer (LINKTYPE_ETHERNET).  Test infrastructure."""
from __future__ import annotations

import struct

import numpy as np

LOCAL_MAC = bytes.fromhex("000c296a014d")
PEER_MAC = bytes.fromhex("02aabbccddee")


def ip4(dotted: str) -> bytes:
    return bytes(int(x) for x in dotted.split("."))


def fold_cksum(data: bytes) -> int:
    """RFC 1071 one's-complement sum of little-endian 16-bit words (native view)."""
    if len(data) & 1:
        data = data + b"\0"
    s = int(np.frombuffer(data, "<u2").astype(np.uint64).sum()) if data else 0
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def l4_cksum(ip_hdr: bytes, l4: bytes, proto: int) -> int:
    """value rte_ipv4_udptcp_cksum stores (native LE u16), l4 cksum field already 0"""
    psd = ip_hdr[12:20] + bytes([0, proto]) + struct.pack(">H", len(l4))
    c = (~fold_cksum(psd + l4)) & 0xFFFF
    if c == 0 and proto == 17:
        c = 0xFFFF
    return c


def ipv4_header(src: str, dst: str, proto: int, l4_len: int, ident: int = 1, tl=None,
                ver_ihl: int = 0x45) -> bytes:
    tl = 20 + l4_len if tl is None else tl
    h = bytearray(struct.pack(">BBHHHBBH4s4s", ver_ihl, 0, tl, ident, 0x4000, 64, proto, 0,
                              ip4(src), ip4(dst)))
    c = (~fold_cksum(bytes(h))) & 0xFFFF
    h[10:12] = struct.pack("<H", c)
    return bytes(h)


def ether(payload: bytes, ethertype: int = 0x0800, dst=LOCAL_MAC, src=PEER_MAC) -> bytes:
    return dst + src + struct.pack(">H", ethertype) + payload


def udp_frame(src: str, sport: int, dst: str, dport: int, payload: bytes, *, corrupt=False,
              dgram_len=None, tl=None) -> bytes:
    dl = 8 + len(payload) if dgram_len is None else dgram_len
    udp = bytearray(struct.pack(">HHHH", sport, dport, dl, 0) + payload)
    ip = ipv4_header(src, dst, 17, len(udp), tl=tl)
    c = l4_cksum(ip, bytes(udp), 17)
    udp[6:8] = struct.pack("<H", c)
    if corrupt:
        udp[-1] ^= 0x01
    return ether(ip + bytes(udp))


def tcp_frame(src: str, sport: int, dst: str, dport: int, payload: bytes, *, flags=0x18,
              seq=1000, ack=2000, corrupt=False, data_off=0x50, tl=None,
              pad_options=True, tl_cksum=False) -> bytes:
    """tl_cksum: with an explicit tl, the checksum the reference computes for
    it (over tl - 20 bytes from ip + 20, rte_ip.h:333), so the segment passes
    tcp_process's check (tcp.c:349-357) whatever tl says"""
    tcp = bytearray(struct.pack(">HHIIBBHHH", sport, dport, seq, ack, data_off, flags, 14600, 0,
                                0))
    hl = (data_off >> 4) * 4
    if hl > 20 and pad_options:
        tcp += bytes(hl - 20)
    tcp += payload
    ip = ipv4_header(src, dst, 6, len(tcp), tl=tl)
    if tl is not None and tl_cksum:
        n = max(tl - 20, 0)
        c = l4_cksum(ip, bytes(tcp[:n]) + bytes(max(n - len(tcp), 0)), 6) if tl >= 20 else 0
    else:
        c = l4_cksum(ip, bytes(tcp), 6)
    tcp[16:18] = struct.pack("<H", c)
    if corrupt:
        tcp[-1] ^= 0x01
    return ether(ip + bytes(tcp))


def arp_frame(sip: str, tip: str) -> bytes:
    body = struct.pack(">HHBBH6s4s6s4s", 1, 0x0800, 6, 4, 1, PEER_MAC, ip4(sip), bytes(6),
                       ip4(tip))
    return ether(body + bytes(18), ethertype=0x0806, dst=b"\xff" * 6)


def icmp_frame(src: str, dst: str) -> bytes:
    icmp = bytearray(struct.pack(">BBHHH", 8, 0, 0, 1, 1) + bytes(32))
    icmp[2:4] = struct.pack("<H", (~fold_cksum(bytes(icmp))) & 0xFFFF)
    return ether(ipv4_header(src, dst, 1, len(icmp)) + bytes(icmp))


def pack_frames(frames: list[bytes], unit_log2: int = 6, caplens=None):
    """Packed device layout: frame i at off[i] << unit_log2 (16-B aligned slots)."""
    unit = 1 << unit_log2
    offs, pos = [], 0
    for f in frames:
        offs.append(pos // unit)
        pos += max(unit, (len(f) + unit - 1) // unit * unit)
    pos = (pos + 15) // 16 * 16 + 16
    buf = np.zeros(pos, np.uint8)
    lens = []
    for i, f in enumerate(frames):
        o = offs[i] * unit
        buf[o:o + len(f)] = np.frombuffer(f, np.uint8)
        lens.append(len(f) if caplens is None else caplens[i])
    return buf, np.array(offs, np.uint32), np.array(lens, np.uint16)


# ---- classic pcap ---------------------------------------------------------
def write_pcap(path: str, frames: list[bytes], caplens=None):
    with open(path, "wb") as fh:
        fh.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1))
        for i, f in enumerate(frames):
            cap = len(f) if caplens is None else caplens[i]
            fh.write(struct.pack("<IIII", i, 0, cap, len(f)))
            fh.write(f[:cap])


def read_pcap(path: str) -> list[bytes]:
    with open(path, "rb") as fh:
        data = fh.read()
    magic = struct.unpack_from("<I", data, 0)[0]
    endian = "<" if magic in (0xA1B2C3D4, 0xA1B23C4D) else ">"
    linktype = struct.unpack_from(endian + "I", data, 20)[0]
    assert linktype == 1, "LINKTYPE_ETHERNET only"
    pos, out = 24, []
    while pos + 16 <= len(data):
        _, _, incl, _orig = struct.unpack_from(endian + "IIII", data, pos)
        pos += 16
        out.append(data[pos:pos + incl])
        pos += incl
    return out


# ---- vectorized builders (many frames at once, numpy) ----------------------
def tcp64_frames(sip, dip, sport, dport, seq=1000) -> np.ndarray:
    """n x 64-B TCP/IPv4 frames (PSH|ACK, 10 payload bytes) for raw
    network-order (sip, dip, sport, dport) arrays, L4 checksum as
    rte_ipv4_udptcp_cksum computes it (tl = 50, L4 = bytes [34, 64))"""
    n = len(sip)
    f = np.zeros((n, 64), np.uint8)
    f[:, 0:6] = np.frombuffer(LOCAL_MAC, np.uint8)
    f[:, 6:12] = np.frombuffer(PEER_MAC, np.uint8)
    f[:, 12:14] = (0x08, 0x00)
    f[:, 14:24] = np.frombuffer(bytes([0x45, 0, 0, 50, 0, 1, 0x40, 0, 64, 6]), np.uint8)
    f32 = f
    f32[:, 26:30] = np.asarray(sip, np.uint32).view(np.uint8).reshape(n, 4)
    f32[:, 30:34] = np.asarray(dip, np.uint32).view(np.uint8).reshape(n, 4)
    f32[:, 34:36] = np.asarray(sport, np.uint16).view(np.uint8).reshape(n, 2)
    f32[:, 36:38] = np.asarray(dport, np.uint16).view(np.uint8).reshape(n, 2)
    f32[:, 38:42] = np.frombuffer(struct.pack(">I", seq), np.uint8)
    f32[:, 46] = 0x50
    f32[:, 47] = 0x18
    f32[:, 48:50] = (0x39, 0x08)
    f32[:, 54:64] = np.arange(10, dtype=np.uint8)
    ip = f32[:, 14:34].copy().view("<u2").astype(np.uint64)
    s = ip.sum(axis=1)
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    f32[:, 24:26] = ((~s) & 0xFFFF).astype("<u2").view(np.uint8).reshape(n, 2)
    wd = f32.view("<u2").astype(np.uint64)  # 32 LE words; L4 = words 17..31, field = word 25
    s = wd[:, 13:17].sum(axis=1) + wd[:, 17:32].sum(axis=1) - wd[:, 25] + 0x0600 + 0x1E00
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    f32[:, 50:52] = ((~s) & 0xFFFF).astype("<u2").view(np.uint8).reshape(n, 2)
    return f
