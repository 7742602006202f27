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


# ---- the delivery half (oracle/ref_stack.c) -------------------------------
def _stack_sigs(l):
    vp, u32, u16, i32, sz, lng = C.c_void_p, C.c_uint32, C.c_uint16, C.c_int32, C.c_size_t, C.c_long
    for name, res, args in [
            ("oracle_stack_new", vp, []), ("oracle_stack_free", None, [vp]),
            ("oracle_nsocket", C.c_int, [vp, C.c_int]),
            ("oracle_nbind", C.c_int, [vp, C.c_int, u32, u16]),
            ("oracle_nlisten", C.c_int, [vp, C.c_int]),
            ("oracle_naccept", C.c_int, [vp, C.c_int, vp, vp]),
            ("oracle_nclose", C.c_int, [vp, C.c_int]),
            ("oracle_rx", C.c_int, [vp, vp, u32]),
            ("oracle_nrecvfrom", lng, [vp, C.c_int, vp, sz, vp, vp]),
            ("oracle_nrecv", lng, [vp, C.c_int, vp, sz]),
            ("oracle_tcb_state", C.c_int, [vp, u32, u32, u16, u16, vp, vp, vp, vp]),
            ("oracle_tcb_sndq", C.c_int, [vp, u32, u32, u16, u16, u32, vp, vp]),
            ("oracle_tcb_count", u32, [vp]),
            ("oracle_tcb_add", C.c_int, [vp, u32, u32, u16, u16, C.c_int]),
            ("oracle_rx_burst", None, [vp, vp, vp, vp, u32, u32, vp]),
            ("oracle_drain_all", lng, [vp, vp, sz, vp])]:
        f = getattr(l, name)
        f.restype, f.argtypes = res, args


_stack_sigs(lib)
WOULD_BLOCK = -2


class Stack:
    """the reference's socket layer + per-frame udp_process/tcp_process effects
    (oracle/ref_stack.c); a blocking call returns WOULD_BLOCK (-2)"""

    def __init__(self):
        self.h = lib.oracle_stack_new()

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:
            lib.oracle_stack_free(self.h)
            self.h = None

    def socket(self, type_):
        return lib.oracle_nsocket(self.h, type_)

    def bind(self, fd, ip_raw, port_raw):
        return lib.oracle_nbind(self.h, fd, ip_raw, port_raw)

    def listen(self, fd):
        return lib.oracle_nlisten(self.h, fd)

    def accept(self, fd):
        sip, sport = C.c_uint32(), C.c_uint16()
        r = lib.oracle_naccept(self.h, fd, C.byref(sip), C.byref(sport))
        return r, sip.value, sport.value

    def close(self, fd):
        return lib.oracle_nclose(self.h, fd)

    def rx(self, frame: bytes):
        b = C.create_string_buffer(bytes(frame), len(frame) + 1)
        return lib.oracle_rx(self.h, b, len(frame))

    def recvfrom(self, fd, n):
        buf = C.create_string_buffer(max(n, 1))
        sip, sport = C.c_uint32(), C.c_uint16()
        r = lib.oracle_nrecvfrom(self.h, fd, buf, n, C.byref(sip), C.byref(sport))
        return r, buf.raw[:max(r, 0)], sip.value, sport.value

    def recv(self, fd, n):
        """(return value, the whole n-byte buffer: a split read returns the
        REMAINING length, common.c:493, after copying n bytes)"""
        buf = C.create_string_buffer(max(n, 1))
        r = lib.oracle_nrecv(self.h, fd, buf, n)
        return r, buf.raw[:n]

    def tcb_state(self, sip, dip, sport, dport):
        """(status, rcv_nxt, snd_nxt or None while it is the random ISN, fd) or None"""
        st, rn, sn, fd = C.c_int32(), C.c_uint32(), C.c_uint32(), C.c_int32()
        r = lib.oracle_tcb_state(self.h, sip, dip, sport, dport, C.byref(st), C.byref(rn),
                                 C.byref(sn), C.byref(fd))
        if r < 0:
            return None
        return st.value, rn.value, (sn.value if r == 1 else None), fd.value

    def tcb_sndq(self, sip, dip, sport, dport):
        out, k = [], 0
        fl, ack = C.c_uint8(), C.c_uint32()
        while lib.oracle_tcb_sndq(self.h, sip, dip, sport, dport, k, C.byref(fl),
                                  C.byref(ack)) == 0:
            out.append((fl.value, ack.value))
            k += 1
        return out

    def tcb_count(self):
        return lib.oracle_tcb_count(self.h)

    def tcb_add(self, sip, dip, sport, dport, status):
        """test hook: install a tcb (raw network-order key) as a SYN would"""
        return lib.oracle_tcb_add(self.h, sip, dip, sport, dport, status)

    def rx_burst(self, pkts, off, lens, off_unit_log2, rcs=None):
        """frames through oracle_rx in burst order (one C call)"""
        lib.oracle_rx_burst(self.h, pkts.ctypes.data, off.ctypes.data, lens.ctypes.data, len(off),
                            off_unit_log2, None if rcs is None else rcs.ctypes.data)

    def drain_all(self, buf):
        nb = C.c_uint64()
        r = lib.oracle_drain_all(self.h, buf.ctypes.data, buf.nbytes, C.byref(nb))
        return r, nb.value
