"""ctypes binding of the oracle (oracle/ref_cpu.c) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")


def _load(name: str):
    path = os.path.join(ORACLE_DIR, name)
    if not os.path.exists(path):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    lib = C.CDLL(path)
    vp, u32, u16, u8 = C.c_void_p, C.c_uint32, C.c_uint16, C.c_uint8
    lib.oracle_raw_cksum.restype = u16
    lib.oracle_raw_cksum.argtypes = [vp, u32]
    lib.oracle_ipv4_udptcp_cksum.restype = u16
    lib.oracle_ipv4_udptcp_cksum.argtypes = [vp, vp]
    lib.oracle_ipv4_cksum.restype = u16
    lib.oracle_ipv4_cksum.argtypes = [vp]
    lib.oracle_tables_new.restype = vp
    lib.oracle_tables_new.argtypes = [vp, u32, vp, u32]
    lib.oracle_tables_free.restype = None
    lib.oracle_tables_free.argtypes = [vp]
    lib.oracle_lookup_udp.restype = u32
    lib.oracle_lookup_udp.argtypes = [vp, u32, u16, u8]
    lib.oracle_lookup_tcp.restype = u32
    lib.oracle_lookup_tcp.argtypes = [vp, u32, u32, u16, u16]
    lib.oracle_classify.restype = None
    lib.oracle_classify.argtypes = [vp, vp, vp, vp, u32, u32, vp, vp]
    lib.oracle_rss_hash.restype = u32
    lib.oracle_rss_hash.argtypes = [u32, u32, u16, u16]
    lib.oracle_tx_cksum.restype = None
    lib.oracle_tx_cksum.argtypes = [vp, vp, vp, u32, u32]
    return lib


lib = _load("liboracle.so")
_lib_O0 = None


def lib_O0():
    global _lib_O0
    if _lib_O0 is None:
        _lib_O0 = _load("liboracle_O0.so")
    return _lib_O0


def _p(a):
    return None if a is None or len(a) == 0 else a.ctypes.data


def raw_cksum(b: bytes) -> int:
    buf = np.frombuffer(bytes(b) + b"\0", np.uint8)
    return lib.oracle_raw_cksum(buf.ctypes.data, len(b))


def udptcp_cksum(ip_and_l4: bytes) -> int:
    """rte_ipv4_udptcp_cksum(ip, ip + 20) on a buffer that starts at the IPv4 header"""
    buf = np.frombuffer(bytes(ip_and_l4) + b"\0" * 8, np.uint8)
    return lib.oracle_ipv4_udptcp_cksum(buf.ctypes.data, buf.ctypes.data + 20)


def ipv4_cksum(hdr20: bytes) -> int:
    buf = np.frombuffer(bytes(hdr20), np.uint8)
    return lib.oracle_ipv4_cksum(buf.ctypes.data)


class Tables:
    """the reference's head-inserted control-block lists"""

    def __init__(self, udp: np.ndarray, tcb: np.ndarray, which=None):
        self.lib = which or lib
        self.udp, self.tcb = udp, tcb
        self.h = self.lib.oracle_tables_new(_p(udp), len(udp), _p(tcb), len(tcb))

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.oracle_tables_free(self.h)
            self.h = None

    def lookup_udp(self, dip, dport, proto=17):
        return self.lib.oracle_lookup_udp(self.h, dip, dport, proto)

    def lookup_tcp(self, sip, dip, sport, dport):
        return self.lib.oracle_lookup_tcp(self.h, sip, dip, sport, dport)

    def classify(self, pkts, off, lens, off_unit_log2, counts: bool = False):
        from rxgpu import VERDICT_DTYPE  # noqa: E402 (types only)
        n = len(off)
        out = np.zeros(n, VERDICT_DTYPE)
        cnt = np.zeros(max(len(self.udp) + len(self.tcb), 1), np.uint64) if counts else None
        pkts = np.ascontiguousarray(pkts, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        lens = np.ascontiguousarray(lens, np.uint16)
        self.lib.oracle_classify(self.h, pkts.ctypes.data, off.ctypes.data, lens.ctypes.data, n,
                                 off_unit_log2, out.ctypes.data,
                                 None if cnt is None else cnt.ctypes.data)
        if counts:
            return out, cnt[: len(self.udp) + len(self.tcb)]
        return out


def tx_cksum(pkts: np.ndarray, off: np.ndarray, lens: np.ndarray, off_unit_log2: int) -> np.ndarray:
    """TX checksum fill (udp.c:84-95, tcp.c:444-463) on a copy of the burst"""
    out = np.array(pkts, np.uint8, copy=True)
    off = np.ascontiguousarray(off, np.uint32)
    lens = np.ascontiguousarray(lens, np.uint16)
    lib.oracle_tx_cksum(_p(out), _p(off), _p(lens), len(off), off_unit_log2)
    return out


def rss_hash(sip, dip, sport, dport):
    return lib.oracle_rss_hash(sip, dip, sport, dport)
