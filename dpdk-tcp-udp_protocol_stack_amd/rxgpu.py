"""ctypes binding of librxgpu.so (include/rxgpu.h) and libnstack.so (include/nstack.h).

This module is plumbing for tests and bench.py: every verdict it returns is
computed by the gfx950 kernel in librxgpu.so.  There is no Python or CPU
fallback — if the shared library is missing, importing this module raises.

Reference interface mirrored (see include/rxgpu.h for file:line citations):
  pkt_process loop body (netfamily.c:152-200) -> Context.classify* / process_mbufs
  udp_process / tcp_process return codes       -> verdict['rc']
  get_hostinfo_fromip_port / tcp_stream_search -> verdict['flow_id'], lookup_udp/lookup_tcp
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RXGPU_LIB: another build of the same library (A/B of compile-time variants)
LIB_PATH = os.environ.get("RXGPU_LIB") or os.path.join(_HERE, "librxgpu.so")
# NSTACK_LIB: another build of the socket layer (e.g. a sanitizer build, host code only)
NSTACK_PATH = os.environ.get("NSTACK_LIB") or os.path.join(_HERE, "libnstack.so")

# One HIP runtime per process: PyTorch (the plumbing for device memory, streams
# and torch.distributed) ships its own libamdhip64.so.7 with the same SONAME as
# /opt/rocm's.  Loading torch first makes librxgpu bind to that copy; loading
# librxgpu first would bring a second HIP/HSA runtime into the process, and the
# two then contend for the device (observed: hipGetDeviceCount fails in one).
try:
    import torch  # noqa: F401
except ImportError:  # a pure-C deployment links /opt/rocm's runtime directly
    pass

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make -C {_HERE}` (or __graft_entry__.build()); "
        "there is no fallback path")
_lib = C.CDLL(LIB_PATH)

# ---- constants (mirror include/rxgpu.h) -----------------------------------
FLOW_NONE = 0xFFFFFFFF
CLS_ARP, CLS_NON_IP, CLS_IPV4_OTHER, CLS_UDP, CLS_TCP = 0, 1, 2, 3, 4
RC_OK, RC_TCP_BAD_CKSUM, RC_TCP_NO_TCB, RC_UDP_NOMEM, RC_UDP_NO_SOCKET, RC_KNI = 0, -1, -2, -2, -3, 1
F_TRUNC, F_TCP_NEGLEN, F_UDP_SHORT = 0x1, 0x2, 0x4
TCP_STATUS_LISTEN, TCP_STATUS_ESTABLISHED = 1, 4
HOST_ONLY = -1
# (lanes per frame, passes up front, frames per group, pipeline) compiled in
# rx_classify.hip (verdict-exact ones; the >= 100 pipeline ids are ablations)
# the product library's classify variants (csrc/rx_classify.hip k_variants):
# (lanes per frame, passes, frames per group, pipeline); every one gives the
# reference's verdicts (tests/test_gpu_parity.py runs each)
KERNEL_VARIANTS = [(1, 4, 1, 12), (1, 4, 1, 5), (1, 4, 1, 14), (1, 4, 1, 19), (1, 4, 1, 25), (1, 4, 1, 16),
                   (1, 4, 1, 0),
                   (4, 1, 1, 1), (8, 2, 2, 0), (8, 2, 2, 40), (8, 2, 2, 41), (8, 2, 2, 42), (8, 2, 2, 48),
                   (8, 2, 1, 0), (16, 2, 2, 0),
                   (32, 3, 2, 0), (64, 4, 1, 0),
                   (0, 0, 0, 20),  # size-class binned: lane kernel + G=8 kernel
                   (0, 0, 0, 30), (0, 0, 0, 38), (0, 0, 0, 738), (0, 0, 0, 938),  # stream kernel
                   (0, 0, 0, 60), (0, 0, 0, 64), (0, 0, 0, 67)]  # SH kernel
# compiled only into the RX_DIAG build (librxgpu_diag.so, RXGPU_LIB=...):
# tuning shapes with correct verdicts ...
DIAG_TUNING_VARIANTS = [(1, 4, 1, 13), (1, 4, 1, 18), (1, 4, 1, 23), (1, 4, 1, 24), (1, 4, 1, 21), (1, 4, 1, 22), (8, 2, 2, 1), (16, 2, 1, 0),
                        (8, 2, 2, 43), (8, 2, 2, 44), (8, 2, 2, 45), (8, 2, 2, 46),
                        (8, 2, 2, 47), (8, 2, 2, 49), (8, 2, 2, 50), (8, 2, 2, 51), (8, 2, 2, 52), (8, 2, 2, 53), (8, 2, 2, 54), (8, 2, 2, 55), (8, 2, 2, 56), (0, 0, 0, 54), (0, 0, 0, 66),
                        (0, 0, 0, 68), (0, 0, 0, 75), (0, 0, 0, 65),
                        (0, 0, 0, 80), (0, 0, 0, 81), (0, 0, 0, 82), (0, 0, 0, 83)]  # WC kernel
# ... and ablations, wrong verdicts (or counts) by construction
DIAG_ABLATIONS = [(1, 4, 1, 101), (1, 4, 1, 104), (1, 4, 1, 108), (1, 4, 1, 113), (1, 4, 1, 201),
                  (1, 4, 1, 204), (1, 4, 1, 213), (0, 0, 0, 130), (0, 0, 0, 46), (0, 0, 0, 146),
                  (0, 0, 0, 246), (0, 0, 0, 446), (0, 0, 0, 646), (0, 0, 0, 438), (0, 0, 0, 838),
                  (0, 0, 0, 1238), (0, 0, 0, 160), (0, 0, 0, 264), (0, 0, 0, 1064),
                  (0, 0, 0, 2064), (0, 0, 0, 167),
                  (1, 4, 1, 1401), (1, 4, 1, 1404), (1, 4, 1, 1408), (1, 4, 1, 1413), (1, 4, 1, 1604), (0, 0, 0, 1667), (0, 0, 0, 6467)]

VERDICT_DTYPE = np.dtype([
    ("flow_id", "<u4"), ("payload_off", "<u2"), ("payload_len", "<u2"), ("l4_cksum", "<u2"),
    ("cls", "u1"), ("rc", "i1"), ("cksum_ok", "u1"), ("flags", "u1"), ("stored_cksum", "<u2"),
])
assert VERDICT_DTYPE.itemsize == 16
# rxg_verdict8 (rxg_classify_dev8): off_neg = payload_off | TCP_NEGLEN << 7,
# status = cls | (rc & 7) << 3 | cksum_ok << 6 | TRUNC << 7
VERDICT8_DTYPE = np.dtype([("flow_id", "<u4"), ("payload_len", "<u2"), ("off_neg", "u1"),
                           ("status", "u1")])
assert VERDICT8_DTYPE.itemsize == 8


def verdict8_of(v: np.ndarray) -> np.ndarray:
    """the 8-B verdicts of 16-B ones (rxg_verdict8_of in include/rxgpu.h)"""
    v = np.ascontiguousarray(v).view(VERDICT_DTYPE)
    r = np.empty(v.shape, VERDICT8_DTYPE)
    r["flow_id"] = v["flow_id"]
    r["payload_len"] = v["payload_len"]
    r["off_neg"] = (v["payload_off"] & 0x7F) | np.where(v["flags"] & 0x02, 0x80, 0)
    r["status"] = ((v["cls"] & 7) | ((v["rc"].view(np.uint8) & 7) << 3) | ((v["cksum_ok"] & 1) << 6)
                   | np.where(v["flags"] & 0x01, 0x80, 0)).astype(np.uint8)
    return r


UDP_SOCK_DTYPE = np.dtype([("localip", "<u4"), ("localport", "<u2"), ("protocol", "u1"),
                           ("_pad", "u1")])
TCB_DTYPE = np.dtype([("sip", "<u4"), ("dip", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
                      ("status", "<u4")])
DGRAM_DTYPE = np.dtype([("frame", "<u4"), ("offset", "<u4"), ("sip", "<u4"), ("sport", "<u2"),
                        ("len", "<u2")])
assert DGRAM_DTYPE.itemsize == 16
COMPACT_MAX_FLOWS = 1024
SEGMENT_DTYPE = np.dtype([("frame", "<u4"), ("flow", "<u4"), ("seq", "<u4"), ("ack", "<u4"),
                          ("plen", "<i4"), ("offset", "<u4"), ("sport", "<u2"), ("dport", "<u2"),
                          ("ncopy", "<u2"), ("flags", "u1"), ("hl", "u1")])
assert SEGMENT_DTYPE.itemsize == 32


class Delivery(C.Structure):
    """rxg_delivery (rxg_process_mbufs_deliver's results)"""
    _fields_ = [("dgram", C.c_void_p), ("first", C.c_void_p), ("udp_payload", C.c_void_p),
                ("ndgram", C.c_uint32), ("nseg", C.c_uint32), ("udp_bytes", C.c_uint64),
                ("seg", C.c_void_p), ("tcp_payload", C.c_void_p), ("tcp_bytes", C.c_uint64),
                ("tcp_payload_ref", C.c_int32), ("set", C.c_uint32)]


class GenCfg(C.Structure):
    """rxg_gen_cfg"""
    _fields_ = [
        ("seed", C.c_uint64), ("size_mode", C.c_uint32), ("frame_len", C.c_uint32),
        ("slot_bytes", C.c_uint32), ("proto_mode", C.c_uint32), ("n_udp", C.c_uint32),
        ("n_tcp", C.c_uint32), ("local_ip", C.c_uint32), ("udp_base_port", C.c_uint16),
        ("tcp_port", C.c_uint16), ("bad_cksum_per10k", C.c_uint32),
        ("unknown_per10k", C.c_uint32), ("other_per10k", C.c_uint32), ("shard", C.c_uint32),
        ("n_shards", C.c_uint32), ("packed", C.c_uint32), ("src_ip", C.c_uint32),
        ("src_port", C.c_uint16), ("_pad", C.c_uint16),
    ]


class Mbuf(C.Structure):
    """rxg_mbuf: rte_mbuf-shaped descriptor (buf_addr@0, data_off@16, refcnt@18,
    data_len@40)."""
    _fields_ = [("buf_addr", C.c_void_p), ("_r0", C.c_uint8 * 8), ("data_off", C.c_uint16),
                ("refcnt", C.c_uint16), ("_r1", C.c_uint8 * 20), ("data_len", C.c_uint16),
                ("_r2", C.c_uint8 * 86)]


assert C.sizeof(Mbuf) == 128

_vp, _u32, _u64, _i32, _u16 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_uint16


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_open = _sig("rxg_open", _i32, C.POINTER(_vp), _i32, _u32, _u64)
_close = _sig("rxg_close", None, _vp)
_strerror = _sig("rxg_strerror", C.c_char_p, _i32)
_last_hip = _sig("rxg_last_hip_error", C.c_char_p)
_flows_sync = _sig("rxg_flows_sync", _i32, _vp, _vp, _u32, _vp, _u32)
_flows_add = _sig("rxg_flows_add", _i32, _vp, _vp, _u32, _vp, _u32, _vp, _vp)
_flows_remove = _sig("rxg_flows_remove", _i32, _vp, _vp, _u32, _vp, _u32)
_flows_update_udp = _sig("rxg_flows_update_udp", _i32, _vp, _u32, _vp)
_flows_update_tcb = _sig("rxg_flows_update_tcb", _i32, _vp, _u32, _vp)
_flows_commit = _sig("rxg_flows_commit", _i32, _vp, _vp)
_num_udp_ids = _sig("rxg_num_udp_ids", _u32, _vp)
_udp_compact_dev = _sig("rxg_udp_compact_dev", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp,
                        _vp, _u64, _vp, _vp)
_flows_rebuilds = _sig("rxg_flows_rebuilds", _u32, _vp)
_tcp_compact_dev = _sig("rxg_tcp_compact_dev", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp,
                        _u64, _vp, _vp)
_process_mbufs_deliver = _sig("rxg_process_mbufs_deliver", _i32, _vp, _vp, _u32, _vp, _vp, _vp)
_deliver_submit = _sig("rxg_deliver_submit", _i32, _vp, _vp, _u32, _vp, _vp)
_tune_ingest = _sig("rxg_tune_ingest", _i32, _vp, _u32)
INGEST_AUTO, INGEST_PULL, INGEST_GATHER = 0, 1, 2
_deliver_wait = _sig("rxg_deliver_wait", _i32, _vp, _vp, _vp)
_register_host = _sig("rxg_register_host", _i32, _vp, _vp, _u64)
_payload_hold = _sig("rxg_payload_hold", _i32, _vp, _i32)
_payload_release = _sig("rxg_payload_release", _i32, _vp, _i32)
_unregister_host = _sig("rxg_unregister_host", _i32, _vp, _vp)
_classify_dev = _sig("rxg_classify_dev", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp)
_classify_dev_cs = _sig("rxg_classify_dev_cs", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp,
                        _vp, _vp)
# (older builds, e.g. an A/B against a previous library, lack it: classify_dev8 then raises)
_classify_dev8 = (_sig("rxg_classify_dev8", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp,
                       _vp, _vp) if hasattr(_lib, "rxg_classify_dev8") else None)
_classify = _sig("rxg_classify", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _vp)
_classify_span = _sig("rxg_classify_span", _i32, _vp, _vp, _u64, _vp, _vp, _u32, _u32, _vp)
_process_mbufs = _sig("rxg_process_mbufs", _i32, _vp, _vp, _u32, _vp)
_flow_counts = _sig("rxg_flow_counts", _i32, _vp, _vp, _u32)
_counts_reset = _sig("rxg_counts_reset", _i32, _vp)
_num_flows = _sig("rxg_num_flows", _u32, _vp)
_tune = _sig("rxg_tune", _i32, _vp, _u32, _u32, _u32, _u32)
_tune_grid = _sig("rxg_tune_grid", _i32, _vp, _u32)
_kernel_variant = (_sig("rxg_kernel_variant", _i32, _vp, _u32, _vp, C.c_char_p, _u32)
                   if hasattr(_lib, "rxg_kernel_variant") else None)
_tune_tx = _sig("rxg_tune_tx", _i32, _vp, _u32, _u32)
_tune_flow_load = _sig("rxg_tune_flow_load", _i32, _vp, _u32)
_tune_tables = _sig("rxg_tune_tables", _i32, _vp, _u32)
TT_NO_UDP_PORT = 0x1
TT_COUNT_4B = 0x2
TT_COUNT_2BUF = 0x4
TT_SLAB_HALF = 0x8     # the slab pass on half / a quarter of the CUs (fewer, larger slabs)
TT_SLAB_QUARTER = 0x10
TX_AUTO = 0xFFFFFFFF
_lk_udp = _sig("rxg_ft_lookup_udp", _u32, _vp, _u32, _u16)
_lk_tcp = _sig("rxg_ft_lookup_tcp", _u32, _vp, _u32, _u32, _u16, _u16)
_ft_dump = _sig("rxg_ft_dump", _i32, _vp, _u32, _i32, _vp, _u64, _vp)
_rss = _sig("rxg_rss_hash", _u32, _u32, _u32, _u16, _u16)
_gen_flows = _sig("rxg_gen_flows", _i32, C.POINTER(GenCfg), _vp, _vp)
_gen_host = _sig("rxg_gen_host", _i32, C.POINTER(GenCfg), _u64, _u32, _vp, _vp, _vp, _u32)
_gen_dev = _sig("rxg_gen_dev", _i32, C.POINTER(GenCfg), _u64, _u32, _vp, _vp, _vp, _u32, _vp)
_submit = _sig("rxg_submit", _i32, _vp, _vp, _u64, _vp, _vp, _u32, _u32, _vp, C.POINTER(_u64))
_wait = _sig("rxg_wait", _i32, _vp, _u64)
_pcap_open = _sig("rxg_pcap_open", _i32, C.POINTER(_vp), C.c_char_p)
_pcap_close = _sig("rxg_pcap_close", None, _vp)
_pcap_rewind = _sig("rxg_pcap_rewind", _i32, _vp)
_pcap_read = _sig("rxg_pcap_read_burst", _i32, _vp, _vp, _u64, _vp, _vp, _u32, _u32,
                  C.POINTER(_u32), C.POINTER(_u64))
_pcap_write = _sig("rxg_pcap_write", _i32, C.c_char_p, _vp, _vp, _vp, _u32, _u32)
_tx_cksum_dev = _sig("rxg_tx_cksum_dev", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp)
_tx_cksum = _sig("rxg_tx_cksum", _i32, _vp, _vp, _u64, _vp, _vp, _u32, _u32)
_rss_split = _sig("rxg_rss_split", _i32, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp)
_rss_split_dev = _sig("rxg_rss_split_dev", _i32, _vp, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp,
                      _vp)
_gather_dev = _sig("rxg_gather_dev", _i32, _vp, _vp, _vp, _vp, _u32, _vp, _u32, _vp, _u64, _vp, _vp,
                   C.POINTER(_u64), _vp)
_group_id = _sig("rxg_group_id", _i32, _vp)
_group_open = _sig("rxg_group_open", _i32, C.POINTER(_vp), _i32, _u32, _u32, _vp)
_group_close = _sig("rxg_group_close", None, _vp)
_group_size = _sig("rxg_group_size", _i32, _vp, C.POINTER(_u32), C.POINTER(_u32))
_counts_allreduce = _sig("rxg_counts_allreduce", _i32, _vp, _vp, _u32, _vp)
_ctx_counts_allreduce = _sig("rxg_ctx_counts_allreduce", _i32, _vp, _vp)
PIPE_DEPTH = 3
SLAB_MIN_FLOWS = 8193  # from here up the per-flow counts are slab passes after the classify kernel
MAX_SHARDS = 64
GROUP_ID_BYTES = 128

EXPORTED = ["rxg_open", "rxg_close", "rxg_strerror", "rxg_last_hip_error", "rxg_flows_sync",
            "rxg_flows_add", "rxg_flows_remove", "rxg_flows_update_udp", "rxg_flows_update_tcb",
            "rxg_flows_commit", "rxg_num_udp_ids", "rxg_flows_rebuilds", "rxg_udp_compact_dev",
            "rxg_process_mbufs_udp", "rxg_tcp_compact_dev", "rxg_process_mbufs_deliver",
            "rxg_deliver_submit", "rxg_deliver_wait", "rxg_tune_ingest",
            "rxg_register_host", "rxg_unregister_host", "rxg_payload_hold", "rxg_payload_release",
            "rxg_classify_dev", "rxg_classify_dev_cs", "rxg_classify_dev8", "rxg_classify", "rxg_classify_span", "rxg_process_mbufs", "rxg_flow_counts",
            "rxg_counts_reset", "rxg_num_flows", "rxg_tune", "rxg_kernel_variant", "rxg_tune_grid", "rxg_tune_tx", "rxg_tune_flow_load", "rxg_tune_tables", "rxg_ft_lookup_udp", "rxg_ft_lookup_tcp", "rxg_ft_dump",
            "rxg_rss_hash", "rxg_gen_flows", "rxg_gen_host", "rxg_gen_dev", "rxg_submit", "rxg_wait",
            "rxg_pcap_open", "rxg_pcap_close", "rxg_pcap_rewind", "rxg_pcap_read_burst",
            "rxg_pcap_write", "rxg_tx_cksum_dev", "rxg_tx_cksum", "rxg_rss_split",
            "rxg_rss_split_dev", "rxg_gather_dev", "rxg_group_id", "rxg_group_open",
            "rxg_group_close", "rxg_group_size", "rxg_counts_allreduce", "rxg_ctx_counts_allreduce"]


class RxgError(RuntimeError):
    def __init__(self, rc: int, what: str):
        msg = _strerror(rc).decode()
        if rc in (-1000, -1001):
            msg += " [" + _last_hip().decode() + "]"
        super().__init__(f"{what}: {msg} ({rc})")
        self.rc = rc


def _check(rc: int, what: str):
    if rc != 0:
        raise RxgError(rc, what)


def _ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to librxgpu must be contiguous"
    return a.ctypes.data


def _tptr(t):
    """device pointer of a torch tensor (or None)"""
    return None if t is None else t.data_ptr()


# ---- byte-order helpers (raw network-order values as the reference stores them)
def ip_raw(dotted: str) -> int:
    b = bytes(int(x) for x in dotted.split("."))
    return int.from_bytes(b, "little")


def port_raw(port: int) -> int:
    return int.from_bytes(port.to_bytes(2, "big"), "little")


class Context:
    """rxg_ctx: one per rx thread (device = HIP ordinal, or HOST_ONLY)."""

    def __init__(self, device: int = 0, max_pkts: int = 0, max_bytes: int = 0):
        h = _vp()
        _check(_open(C.byref(h), device, max_pkts, max_bytes), "rxg_open")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            _close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def flows_sync(self, udp: np.ndarray | None = None, tcb: np.ndarray | None = None):
        udp = np.ascontiguousarray(udp if udp is not None else np.zeros(0, UDP_SOCK_DTYPE),
                                   UDP_SOCK_DTYPE)
        tcb = np.ascontiguousarray(tcb if tcb is not None else np.zeros(0, TCB_DTYPE), TCB_DTYPE)
        _check(_flows_sync(self._h, _ptr(udp) if len(udp) else None, len(udp),
                           _ptr(tcb) if len(tcb) else None, len(tcb)), "rxg_flows_sync")
        self.nu, self.nt = len(udp), len(tcb)

    def flows_add(self, udp: np.ndarray | None = None, tcb: np.ndarray | None = None):
        """add control blocks as the newest ones (rxg_flows_add); returns
        (udp_ids, tcp_ids, count_layout_moved)"""
        udp = np.ascontiguousarray(udp if udp is not None else np.zeros(0, UDP_SOCK_DTYPE),
                                   UDP_SOCK_DTYPE)
        tcb = np.ascontiguousarray(tcb if tcb is not None else np.zeros(0, TCB_DTYPE), TCB_DTYPE)
        uid = np.zeros(max(len(udp), 1), np.uint32)
        tid = np.zeros(max(len(tcb), 1), np.uint32)
        rc = _flows_add(self._h, _ptr(udp) if len(udp) else None, len(udp),
                        _ptr(tcb) if len(tcb) else None, len(tcb), _ptr(uid), _ptr(tid))
        if rc < 0:
            _check(rc, "rxg_flows_add")
        return uid[:len(udp)], tid[:len(tcb)], rc == 1

    def flows_remove(self, udp_ids=None, tcp_ids=None):
        u = np.ascontiguousarray(udp_ids if udp_ids is not None else [], np.uint32)
        t = np.ascontiguousarray(tcp_ids if tcp_ids is not None else [], np.uint32)
        _check(_flows_remove(self._h, _ptr(u) if len(u) else None, len(u),
                             _ptr(t) if len(t) else None, len(t)), "rxg_flows_remove")

    def flows_update_udp(self, fid: int, sock):
        a = np.ascontiguousarray(np.asarray(sock, UDP_SOCK_DTYPE).reshape(1))
        _check(_flows_update_udp(self._h, fid, _ptr(a)), "rxg_flows_update_udp")

    def flows_update_tcb(self, fid: int, tcb):
        a = np.ascontiguousarray(np.asarray(tcb, TCB_DTYPE).reshape(1))
        _check(_flows_update_tcb(self._h, fid, _ptr(a)), "rxg_flows_update_tcb")

    def flows_commit(self, stream=None):
        _check(_flows_commit(self._h, stream), "rxg_flows_commit")

    @property
    def num_udp_ids(self) -> int:
        return _num_udp_ids(self._h)

    @property
    def flows_rebuilds(self) -> int:
        return _flows_rebuilds(self._h)

    def tune(self, lanes_per_frame: int = 0, passes: int = 0, frames_per_group: int = 0,
             pipeline: int = 0xFFFFFFFF):
        """force a kernel variant (lanes_per_frame 0 = automatic); see KERNEL_VARIANTS"""
        _check(_tune(self._h, lanes_per_frame, passes, frames_per_group, pipeline), "rxg_tune")

    def kernel_variant(self, len_hint: int):
        """(kernel name as a trace shows it, [g, p, fpg, pipe]) of the classify
        dispatch a burst with this len_hint runs (rxg_kernel_variant)"""
        if _kernel_variant is None:
            return None, None
        v = np.zeros(4, np.uint32)
        buf = C.create_string_buffer(128)
        _check(_kernel_variant(self._h, len_hint, _ptr(v), buf, 128), "rxg_kernel_variant")
        return buf.value.decode(), [int(x) for x in v]

    def tune_grid(self, blocks_per_cu: int = 0):
        """cap resident blocks per CU (0 = occupancy)"""
        _check(_tune_grid(self._h, blocks_per_cu), "rxg_tune_grid")

    def tune_tx(self, variant: int = TX_AUTO, blocks_per_cu: int = 0):
        """force a TX checksum kernel variant (tx_cksum.hip k_tx index; TX_AUTO =
        by len_hint) and cap its resident blocks per CU (0 = its default)"""
        _check(_tune_tx(self._h, variant, blocks_per_cu), "rxg_tune_tx")

    def tune_flow_load(self, load_log2: int = 0):
        """exact-key flow tables at load <= 2**-load_log2 from the next
        flows_sync (0 = default); verdicts do not depend on it"""
        _check(_tune_flow_load(self._h, load_log2), "rxg_tune_flow_load")

    def tune_tables(self, flags: int = 0):
        """flow-table layout flags (TT_*) from the next flows_sync; verdicts do
        not depend on them"""
        _check(_tune_tables(self._h, flags), "rxg_tune_tables")

    @property
    def num_flows(self) -> int:
        return _num_flows(self._h)

    def lookup_udp(self, dip: int, dport: int) -> int:
        return _lk_udp(self._h, dip, dport)

    def lookup_tcp(self, sip: int, dip: int, sport: int, dport: int) -> int:
        return _lk_tcp(self._h, sip, dip, sport, dport)

    def classify(self, pkts: np.ndarray, off: np.ndarray, lens: np.ndarray,
                 off_unit_log2: int) -> np.ndarray:
        """Host buffers in, verdicts out (PCIe-inclusive, synchronous)."""
        pkts = np.ascontiguousarray(pkts, np.uint8)
        off = np.ascontiguousarray(off, np.uint32)
        lens = np.ascontiguousarray(lens, np.uint16)
        out = np.zeros(len(off), VERDICT_DTYPE)
        _check(_classify(self._h, _ptr(pkts), _ptr(off), _ptr(lens), len(off), off_unit_log2,
                         _ptr(out)), "rxg_classify")
        return out

    def classify_span(self, pkts_ptr: int, span: int, off_ptr: int, len_ptr: int, n: int,
                      off_unit_log2: int, out_ptr: int):
        """raw-pointer host burst (pinned buffers from the caller), PCIe-inclusive"""
        _check(_classify_span(self._h, pkts_ptr, span, off_ptr, len_ptr, n, off_unit_log2,
                              out_ptr), "rxg_classify_span")

    def submit(self, pkts_ptr: int, span: int, off_ptr: int, len_ptr: int, n: int,
               off_unit_log2: int, out_ptr: int) -> int:
        """raw-pointer pipelined burst (pinned host buffers); returns the ticket"""
        t = _u64()
        _check(_submit(self._h, pkts_ptr, span, off_ptr, len_ptr, n, off_unit_log2, out_ptr,
                       C.byref(t)), "rxg_submit")
        return t.value

    def wait(self, ticket: int):
        _check(_wait(self._h, ticket), "rxg_wait")

    def classify_dev(self, d_pkts, d_off, d_len, n: int, off_unit_log2: int, len_hint: int,
                     d_out, d_counts=None, stream=None, count_stream=None):
        """Device tensors in/out (torch tensors or raw ints), asynchronous on
        `stream`; with count_stream (a raw hipStream_t), d_counts is completed
        on that stream instead (rxg_classify_dev_cs)"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        if count_stream is None:
            _check(_classify_dev(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2,
                                 len_hint, p(d_out), p(d_counts), stream), "rxg_classify_dev")
        else:
            _check(_classify_dev_cs(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2,
                                    len_hint, p(d_out), p(d_counts), stream, count_stream),
                   "rxg_classify_dev_cs")

    def classify_dev8(self, d_pkts, d_off, d_len, n: int, off_unit_log2: int, len_hint: int,
                      d_out, d_counts=None, stream=None, count_stream=None):
        """classify_dev writing 8-B verdicts (VERDICT8_DTYPE, rxg_classify_dev8)
        into d_out (n x 8 bytes)"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        if _classify_dev8 is None:
            raise RuntimeError(f"{LIB_PATH} has no rxg_classify_dev8 (an older build)")
        _check(_classify_dev8(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2, len_hint,
                              p(d_out), p(d_counts), stream, count_stream), "rxg_classify_dev8")

    def udp_compact_dev(self, d_pkts, d_off, d_len, n: int, off_unit_log2: int, d_v, d_dgram,
                        d_first, d_payload, payload_cap: int, d_totals, stream=None):
        """K3: a classified burst's delivered datagrams grouped by socket and
        their payloads gathered (rxg_udp_compact_dev), async on stream"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        _check(_udp_compact_dev(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2, p(d_v),
                                p(d_dgram), p(d_first), p(d_payload), payload_cap, p(d_totals),
                                stream), "rxg_udp_compact_dev")

    def tcp_compact_dev(self, d_pkts, d_off, d_len, n: int, off_unit_log2: int, d_v, d_seg,
                        d_payload, payload_cap: int, d_totals, stream=None):
        """K4: a classified burst's rc-0 TCP segments sorted by tcb id and their
        PSH payloads gathered (rxg_tcp_compact_dev), async on stream"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        _check(_tcp_compact_dev(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2, p(d_v),
                                p(d_seg), p(d_payload), payload_cap, p(d_totals), stream),
               "rxg_tcp_compact_dev")

    def register_host(self, ptr: int, nbytes: int):
        """rxg_register_host: frames in [ptr, ptr + nbytes) are pulled by the
        device (keep the memory alive until unregister_host / close)"""
        _check(_register_host(self._h, ptr, nbytes), "rxg_register_host")

    def unregister_host(self, ptr: int):
        _check(_unregister_host(self._h, ptr), "rxg_unregister_host")

    def process_mbufs_deliver(self, mbufs):
        """rxg_process_mbufs_deliver over Mbuf structures: (verdicts, dgrams,
        first, udp payload, segments, tcp payload, phase ms) as numpy copies"""
        if not isinstance(mbufs, C.Array):
            mbufs = (C.POINTER(Mbuf) * len(mbufs))(*[C.pointer(m) for m in mbufs])
        arr = mbufs
        out = np.zeros(len(mbufs), VERDICT_DTYPE)
        d = Delivery()
        ms = (C.c_float * 8)()
        _check(_process_mbufs_deliver(self._h, C.cast(arr, _vp), len(mbufs), _ptr(out),
                                      C.byref(d), ms), "rxg_process_mbufs_deliver")
        return self._delivery_results(out, d, ms)

    def _delivery_results(self, out, d, ms):
        def grab(ptr, nbytes, dtype):
            if not ptr or nbytes == 0:
                return np.zeros(0, dtype)
            return np.frombuffer((C.c_uint8 * nbytes).from_address(ptr), np.uint8).copy().view(dtype)
        nf = _num_udp_ids(self._h)
        dg = grab(d.dgram, d.ndgram * 16, DGRAM_DTYPE)
        first = grab(d.first, (nf + 1) * 4, np.uint32) if d.first else None
        up = grab(d.udp_payload, d.udp_bytes, np.uint8)
        seg = grab(d.seg, d.nseg * 32, SEGMENT_DTYPE)
        tp = grab(d.tcp_payload, d.tcp_bytes, np.uint8)
        return out, dg, first, up, seg, tp, list(ms)

    def tune_ingest(self, mode: int):
        """rxg_tune_ingest: INGEST_AUTO / INGEST_PULL / INGEST_GATHER"""
        _check(_tune_ingest(self._h, mode), "rxg_tune_ingest")

    def deliver_submit(self, mbufs):
        """rxg_deliver_submit: a handle for deliver_wait (keeps the arrays alive)"""
        if not isinstance(mbufs, C.Array):
            mbufs = (C.POINTER(Mbuf) * len(mbufs))(*[C.pointer(m) for m in mbufs])
        out = np.zeros(len(mbufs), VERDICT_DTYPE)
        d = Delivery()
        _check(_deliver_submit(self._h, C.cast(mbufs, _vp), len(mbufs), _ptr(out), C.byref(d)),
               "rxg_deliver_submit")
        return (mbufs, out, d)

    def deliver_wait(self, handle):
        """rxg_deliver_wait: the results as process_mbufs_deliver returns them"""
        _, out, d = handle
        ms = (C.c_float * 8)()
        _check(_deliver_wait(self._h, C.byref(d), ms), "rxg_deliver_wait")
        return self._delivery_results(out, d, ms)

    def tx_cksum(self, pkts: np.ndarray, off: np.ndarray, lens: np.ndarray,
                 off_unit_log2: int) -> np.ndarray:
        """TX checksum fill of a host burst (PCIe round trip); returns the filled copy"""
        out = np.array(pkts, np.uint8, copy=True)
        off = np.ascontiguousarray(off, np.uint32)
        lens = np.ascontiguousarray(lens, np.uint16)
        span = max(((int(o) << off_unit_log2) + int(n) for o, n in zip(off, lens)), default=0)
        _check(_tx_cksum(self._h, _ptr(out), span, _ptr(off), _ptr(lens), len(off), off_unit_log2),
               "rxg_tx_cksum")
        return out

    def tx_cksum_dev(self, d_pkts, d_off, d_len, n: int, off_unit_log2: int, len_hint: int,
                     stream=None):
        """in-place TX checksum fill of a device burst (torch tensors or raw ints)"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        _check(_tx_cksum_dev(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2, len_hint,
                             stream), "rxg_tx_cksum_dev")

    def process_mbufs(self, mbufs) -> np.ndarray:
        arr = (C.POINTER(Mbuf) * len(mbufs))(*[C.pointer(m) for m in mbufs])
        out = np.zeros(len(mbufs), VERDICT_DTYPE)
        _check(_process_mbufs(self._h, C.cast(arr, _vp), len(mbufs), _ptr(out)),
               "rxg_process_mbufs")
        return out

    def rss_split_dev(self, d_pkts, d_off, d_len, n: int, off_unit_log2: int, n_shards: int,
                      d_first, d_perm, stream=None):
        """RSS split of a device burst: d_first (n_shards + 1 u32) and d_perm (n u32)"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        _check(_rss_split_dev(self._h, p(d_pkts), p(d_off), p(d_len), n, off_unit_log2, n_shards,
                              p(d_first), p(d_perm), stream), "rxg_rss_split_dev")

    def gather_dev(self, d_pkts, d_off, d_len, off_unit_log2: int, d_idx, count: int, d_dst,
                   dst_cap: int, d_dst_off, d_dst_len, stream=None) -> int:
        """pack frames d_idx[0..count) into d_dst (64-B units); returns the bytes used"""
        def p(x):
            return x if (x is None or isinstance(x, int)) else x.data_ptr()
        span = _u64()
        _check(_gather_dev(self._h, p(d_pkts), p(d_off), p(d_len), off_unit_log2, p(d_idx), count,
                           p(d_dst), dst_cap, p(d_dst_off), p(d_dst_len), C.byref(span), stream),
               "rxg_gather_dev")
        return span.value

    def counts_allreduce(self, group: "Group"):
        """sum the context-owned counts over the group's ranks (synchronous)"""
        _check(_ctx_counts_allreduce(self._h, group._h), "rxg_ctx_counts_allreduce")

    def flow_counts(self) -> np.ndarray:
        n = self.num_flows
        out = np.zeros(max(n, 1), np.uint64)
        _check(_flow_counts(self._h, _ptr(out), n), "rxg_flow_counts")
        return out[:n]

    def counts_reset(self):
        _check(_counts_reset(self._h), "rxg_counts_reset")


class Pcap:
    """rxg_pcap: a capture file read burst by burst into the packed layout."""

    def __init__(self, path: str):
        h = _vp()
        _check(_pcap_open(C.byref(h), path.encode()), "rxg_pcap_open")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _pcap_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rewind(self):
        _check(_pcap_rewind(self._h), "rxg_pcap_rewind")

    def read_burst_into(self, pkts: np.ndarray, off: np.ndarray, lens: np.ndarray,
                        off_unit_log2: int = 6):
        """fill caller arrays (e.g. pinned tensors' numpy views); returns (n, span)"""
        n, span = _u32(), _u64()
        _check(_pcap_read(self._h, _ptr(pkts), pkts.nbytes, _ptr(off), _ptr(lens), len(off),
                          off_unit_log2, C.byref(n), C.byref(span)), "rxg_pcap_read_burst")
        return n.value, span.value

    def read_burst(self, max_frames: int, cap_bytes: int, off_unit_log2: int = 6):
        pkts = np.zeros(cap_bytes, np.uint8)
        off = np.zeros(max_frames, np.uint32)
        lens = np.zeros(max_frames, np.uint16)
        n, span = self.read_burst_into(pkts, off, lens, off_unit_log2)
        return pkts[:span + 16], off[:n], lens[:n]


def pcap_write(path: str, pkts: np.ndarray, off: np.ndarray, lens: np.ndarray,
               off_unit_log2: int = 6):
    pkts = np.ascontiguousarray(pkts, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    lens = np.ascontiguousarray(lens, np.uint16)
    _check(_pcap_write(path.encode(), _ptr(pkts), _ptr(off), _ptr(lens), len(off), off_unit_log2),
           "rxg_pcap_write")


def rss_hash(sip: int, dip: int, sport: int, dport: int) -> int:
    return _rss(sip, dip, sport, dport)


def rss_split(pkts: np.ndarray, off: np.ndarray, lens: np.ndarray, off_unit_log2: int,
              n_shards: int):
    """host RSS split (rxg_rss_split): (first[n_shards + 1], perm[n])"""
    pkts = np.ascontiguousarray(pkts, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    lens = np.ascontiguousarray(lens, np.uint16)
    first = np.zeros(n_shards + 1, np.uint32)
    perm = np.zeros(max(len(off), 1), np.uint32)
    _check(_rss_split(_ptr(pkts), _ptr(off), _ptr(lens), len(off), off_unit_log2, n_shards,
                      _ptr(first), _ptr(perm)), "rxg_rss_split")
    return first, perm[:len(off)]


def group_id() -> bytes:
    """rank 0: a fresh communicator id to hand to every rank (rxg_group_id)"""
    b = (C.c_uint8 * GROUP_ID_BYTES)()
    _check(_group_id(b), "rxg_group_id")
    return bytes(b)


class Group:
    """rxg_group: the node's GPUs as one RCCL communicator (one rank per process)"""

    def __init__(self, device: int, nranks: int, rank: int, gid: bytes):
        assert len(gid) == GROUP_ID_BYTES
        h = _vp()
        buf = (C.c_uint8 * GROUP_ID_BYTES)(*gid)
        _check(_group_open(C.byref(h), device, nranks, rank, buf), "rxg_group_open")
        self._h = h

    def size(self):
        """rxg_group_size: (nranks, rank) as the RCCL communicator reports them"""
        nr, rk = C.c_uint32(), C.c_uint32()
        _check(_group_size(self._h, C.byref(nr), C.byref(rk)), "rxg_group_size")
        return nr.value, rk.value

    def allreduce(self, d_counts, n: int, stream=None):
        """in-place sum of a device u64[n] vector over the ranks, async on stream"""
        p = d_counts if isinstance(d_counts, int) else d_counts.data_ptr()
        _check(_counts_allreduce(self._h, p, n, stream), "rxg_counts_allreduce")

    def close(self):
        if getattr(self, "_h", None):
            _group_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_gen_cfg(**kw) -> GenCfg:
    d = dict(seed=0x5EED0001, size_mode=0, frame_len=64, slot_bytes=64, proto_mode=0, n_udp=1024,
             n_tcp=0, local_ip=ip_raw("192.168.100.77"), udp_base_port=20000, tcp_port=9999,
             bad_cksum_per10k=100, unknown_per10k=50, other_per10k=50, shard=0, n_shards=1,
             packed=0, src_ip=0, src_port=0)
    d.update(kw)
    return GenCfg(**d)


def gen_flows(cfg: GenCfg):
    udp = np.zeros(cfg.n_udp, UDP_SOCK_DTYPE)
    tcb = np.zeros(cfg.n_tcp + 1 if cfg.n_tcp else 0, TCB_DTYPE)
    _check(_gen_flows(C.byref(cfg), _ptr(udp) if len(udp) else None,
                      _ptr(tcb) if len(tcb) else None), "rxg_gen_flows")
    return udp, tcb


def gen_host(cfg: GenCfg, first: int, n: int, off_unit_log2: int = 6):
    pkts = np.zeros(n * cfg.slot_bytes, np.uint8)
    off = np.zeros(n, np.uint32)
    lens = np.zeros(n, np.uint16)
    _check(_gen_host(C.byref(cfg), first, n, _ptr(pkts), _ptr(off), _ptr(lens), off_unit_log2),
           "rxg_gen_host")
    return pkts, off, lens


def gen_dev(cfg: GenCfg, first: int, n: int, d_pkts, d_off, d_len, off_unit_log2: int = 6,
            stream=None):
    _check(_gen_dev(C.byref(cfg), first, n, _tptr(d_pkts), _tptr(d_off), _tptr(d_len),
                    off_unit_log2, stream), "rxg_gen_dev")


# ---- libnstack: the socket layer (include/nstack.h) ------------------------
AF_INET, SOCK_STREAM, SOCK_DGRAM, MSG_DONTWAIT = 2, 1, 2, 0x40


class SockaddrIn(C.Structure):
    _fields_ = [("sin_family", C.c_uint16), ("sin_port", C.c_uint16), ("sin_addr", C.c_uint32),
                ("sin_zero", C.c_uint8 * 8)]


def sockaddr(ip: str, port: int) -> SockaddrIn:
    return SockaddrIn(AF_INET, port_raw(port), ip_raw(ip))


def ft_dump(h, which: int, device: bool):
    """rxg_ft_dump of context handle h: (uint32 array of the table, info[8]);
    which 3 / 4: the compact UDP table / the port window (include/rxgpu.h)"""
    info = np.zeros(8, np.uint32)
    _check(_ft_dump(h, which, int(device), None, 0, _ptr(info)), "rxg_ft_dump")  # sizes
    words = {0: int(info[7]) * 4, 1: int(info[7]) * 4, 2: 65536, 3: int(info[7]) * 2,
             4: (int(info[7]) + 1) // 2}[which]
    buf = np.zeros(words, np.uint32)
    _check(_ft_dump(h, which, int(device), _ptr(buf), buf.nbytes, _ptr(info)), "rxg_ft_dump")
    return buf, info


class NStack:
    """Process-wide socket layer (one per process, like the reference's globals)."""
    _lib = None

    def __init__(self, device: int = HOST_ONLY, max_burst: int = 4096, max_bytes: int = 1 << 24):
        if NStack._lib is None:
            if not os.path.exists(NSTACK_PATH):
                raise ImportError(f"{NSTACK_PATH} missing: run make -C {_HERE}")
            lib = C.CDLL(NSTACK_PATH)
            ssz = C.c_ssize_t
            sig = [("nstack_init", _i32, [_i32, _u32, _u64]), ("nstack_fini", None, []),
                   ("nsocket", _i32, [_i32, _i32, _i32]), ("nbind", _i32, [_i32, _vp, _u32]),
                   ("nlisten", _i32, [_i32, _i32]), ("naccept", _i32, [_i32, _vp, _vp]),
                   ("nsend", ssz, [_i32, _vp, C.c_size_t, _i32]),
                   ("nrecv", ssz, [_i32, _vp, C.c_size_t, _i32]),
                   ("nrecvfrom", ssz, [_i32, _vp, C.c_size_t, _i32, _vp, _vp]),
                   ("nsendto", ssz, [_i32, _vp, C.c_size_t, _i32, _vp, _u32]),
                   ("nclose", _i32, [_i32]),
                   ("nstack_rx_burst", _i32, [_vp, _u32, _vp, _vp]),
                   ("nstack_rx_submit", _i32, [_vp, _u32, _vp, _vp]),
                   ("nstack_rx_complete", _i32, []),
                   ("nstack_rx_pending", _i32, []),
                   ("nstack_deliver", _i32, [_vp, _u32, _vp, _u64, _vp]),
                   ("nstack_tcb_add", _i32, [_u32, _u32, _u16, _u16, _i32]),
                   ("nstack_flows", _i32, [_vp, _u32, _vp, _vp, _u32, _vp, _vp]),
                   ("nstack_flow_ids", _i32, [_vp, _u32, _vp, _u32]),
                   ("nstack_drain_all", C.c_int64, [_vp, C.c_size_t, _vp]),
                   ("nstack_drain_all_sum", C.c_int64, [_vp, C.c_size_t, _vp, _vp]),
                   ("nstack_set_rx_inplace", _i32, [_i32, _vp, _vp]),
                   ("nstack_mbufs_put", None, [_vp, _u32]),
                   ("nstack_reclaim", None, []),
                   ("nstack_last_burst_phases", _i32, [_vp]),
                   ("nstack_tcb_state", _i32, [_u32, _u32, _u16, _u16, _vp, _vp, _vp, _vp]),
                   ("nstack_tcb_sndq", _i32, [_u32, _u32, _u16, _u16, _u32, _vp, _vp]),
                   ("nstack_tcb_count", _u32, []),
                   ("nstack_lookup_udp", _u32, [_u32, _u16]),
                   ("nstack_lookup_tcp", _u32, [_u32, _u32, _u16, _u16]),
                   ("nstack_ctx", _vp, []),
                   ("nstack_register_host", _i32, [_vp, _u64]),
                   ("nstack_set_halves", _i32, [_u32]),
                   ("nstack_stat", _u64, [_i32]),
                   ("nstack_set_local", _i32, [_u32, _vp]),
                   ("nstack_arp_insert", _i32, [_u32, _vp]),
                   ("nstack_tx_burst", _i32, [_vp, _u64, _vp, _vp, _u32, _i32, _vp])]
            for name, res, args in sig:
                f = getattr(lib, name)
                f.restype, f.argtypes = res, args
            NStack._lib = lib
        self.lib = NStack._lib
        _check(self.lib.nstack_init(device, max_burst, max_bytes), "nstack_init")

    def fini(self):
        self.lib.nstack_fini()
        self._held = []  # (in place: the stack let go of every frame)
        self._inplace = False

    # socket calls: thin pass-through with the reference's argument meaning
    def socket(self, type_):
        return self.lib.nsocket(AF_INET, type_, 0)

    def bind(self, fd, ip, port):
        a = sockaddr(ip, port)
        return self.lib.nbind(fd, C.byref(a), C.sizeof(a))

    def listen(self, fd):
        return self.lib.nlisten(fd, 10)

    def accept(self, fd):
        a = SockaddrIn()
        n = C.c_uint32(C.sizeof(a))
        r = self.lib.naccept(fd, C.byref(a), C.byref(n))
        return r, a

    def recvfrom(self, fd, n, flags=MSG_DONTWAIT):
        buf = C.create_string_buffer(max(n, 1))
        a = SockaddrIn()
        al = C.c_uint32(C.sizeof(a))
        r = self.lib.nrecvfrom(fd, buf, n, flags, C.byref(a), C.byref(al))
        return r, buf.raw[:max(r, 0)], a

    def recv(self, fd, n, flags=MSG_DONTWAIT, full=False):
        """(return value, bytes); full=True: the whole n-byte buffer (a split
        read returns the remaining length, common.c:493, after copying n bytes)"""
        buf = C.create_string_buffer(max(n, 1))
        r = self.lib.nrecv(fd, buf, n, flags)
        return r, (buf.raw[:n] if full else buf.raw[:max(r, 0)])

    def sendto(self, fd, data: bytes, ip, port):
        a = sockaddr(ip, port)
        return self.lib.nsendto(fd, data, len(data), 0, C.byref(a), C.sizeof(a))

    def send(self, fd, data: bytes):
        return self.lib.nsend(fd, data, len(data), 0)

    def close(self, fd):
        return self.lib.nclose(fd)

    def tcb_add(self, sip, dip, sport, dport, status=TCP_STATUS_ESTABLISHED):
        return self.lib.nstack_tcb_add(ip_raw(sip), ip_raw(dip), port_raw(sport),
                                       port_raw(dport), status)

    def flow_ids(self):
        """(udp_ids, tcp_ids): the stable flow id of each block of flows()"""
        u, t = self.flows()
        uid = np.zeros(max(len(u), 1), np.uint32)
        tid = np.zeros(max(len(t), 1), np.uint32)
        _check(self.lib.nstack_flow_ids(_ptr(uid), len(u), _ptr(tid), len(t)), "nstack_flow_ids")
        return uid[:len(u)], tid[:len(t)]

    def to_ids(self, v: np.ndarray) -> np.ndarray:
        """verdicts made against flows()'s arrays (creation-order indices, e.g. by
        the oracle) with their flow ids turned into the blocks' stable ids"""
        uid, tid = self.flow_ids()
        v = np.array(v, VERDICT_DTYPE, copy=True)
        for cls, ids in ((CLS_UDP, uid), (CLS_TCP, tid)):
            m = (v["cls"] == cls) & (v["flow_id"] != FLOW_NONE)
            v["flow_id"][m] = ids[v["flow_id"][m]]
        return v

    def lookup_udp(self, dip: int, dport: int) -> int:
        """the flow id the library's tables give a UDP key (raw network order)"""
        return self.lib.nstack_lookup_udp(dip, dport)

    def lookup_tcp(self, sip: int, dip: int, sport: int, dport: int) -> int:
        """the flow id the library's tables give a TCP 4-tuple (raw), listener included"""
        return self.lib.nstack_lookup_tcp(sip, dip, sport, dport)

    def tune_ingest(self, mode: int):
        """rxg_tune_ingest on the stack's context (INGEST_AUTO / _PULL / _GATHER)"""
        _check(_tune_ingest(self.lib.nstack_ctx(), mode), "rxg_tune_ingest")

    def set_halves(self, min_half: int):
        """nstack_set_halves: bursts of >= 2 * min_half frames as two halves in flight (0 = off)"""
        _check(self.lib.nstack_set_halves(min_half), "nstack_set_halves")

    def register_host(self, ptr: int, nbytes: int):
        """nstack_register_host: frames in this memory are pulled by the GPU"""
        _check(self.lib.nstack_register_host(ptr, nbytes), "nstack_register_host")

    def ft_dump(self, which: int, device: bool):
        """diagnostics: (table, info) of the socket layer's context (rxg_ft_dump)"""
        return ft_dump(self.lib.nstack_ctx(), which, device)

    def flows(self, with_gen: bool = False):
        """the lists in creation order (and, with_gen, their generation for deliver)"""
        nu, nt, gen = C.c_uint32(), C.c_uint32(), _u64()
        _check(self.lib.nstack_flows(None, 0, C.byref(nu), None, 0, C.byref(nt), None),
               "nstack_flows")
        u = np.zeros(nu.value, UDP_SOCK_DTYPE)
        t = np.zeros(nt.value, TCB_DTYPE)
        _check(self.lib.nstack_flows(_ptr(u) if len(u) else None, len(u), None,
                                     _ptr(t) if len(t) else None, len(t), None, C.byref(gen)),
               "nstack_flows")
        return (u, t, gen.value) if with_gen else (u, t)

    def tcb_state(self, sip, dip, sport, dport):
        """(status, rcv_nxt, snd_nxt, fd) of the tcb with this raw 4-tuple, or None"""
        st, rn, sn, fd = C.c_int32(), C.c_uint32(), C.c_uint32(), C.c_int32()
        if self.lib.nstack_tcb_state(sip, dip, sport, dport, C.byref(st), C.byref(rn),
                                     C.byref(sn), C.byref(fd)):
            return None
        return st.value, rn.value, sn.value, fd.value

    def tcb_sndq(self, sip, dip, sport, dport):
        """[(tcp_flags, acknum)] queued in the tcb's send ring, oldest first"""
        out, k = [], 0
        fl, ack = C.c_uint8(), C.c_uint32()
        while self.lib.nstack_tcb_sndq(sip, dip, sport, dport, k, C.byref(fl), C.byref(ack)) == 0:
            out.append((fl.value, ack.value))
            k += 1
        return out

    def tcb_count(self):
        return self.lib.nstack_tcb_count()

    PHASES = ("gather", "h2d", "classify", "compact", "d2h", "lib_call", "udp_deliver",
              "tcp_deliver", "frame_loop", "rx_burst", "segments", "datagrams")

    def last_burst_phases(self) -> dict:
        """where the last rx_burst's time went (nstack_last_burst_phases, ms)"""
        ms = (C.c_float * 12)()
        _check(self.lib.nstack_last_burst_phases(ms), "nstack_last_burst_phases")
        return dict(zip(self.PHASES, [float(x) for x in ms]))

    @staticmethod
    def mbufs(frames: list[bytes]):
        """rte_mbuf-shaped descriptors over the given frames (kept alive by the return)"""
        bufs = [C.create_string_buffer(f, len(f) + 16) for f in frames]
        ms = [Mbuf() for _ in frames]
        for m, b, f in zip(ms, bufs, frames):
            m.buf_addr = C.cast(b, C.c_void_p)
            m.data_off = 0
            m.data_len = len(f)
            m.refcnt = 1  # the caller's reference (rte_pktmbuf_alloc)
        arr = (C.POINTER(Mbuf) * len(ms))(*[C.pointer(m) for m in ms])
        return arr, (bufs, ms)

    STALE = 0xFFFFFFFFFFFFFFFF  # a generation no list state has: re-look every frame up

    def deliver(self, frames: list[bytes], verdicts: np.ndarray, rcs: np.ndarray | None = None,
                gen: int = STALE) -> int:
        """apply verdicts (flow ids = stable ids, see to_ids) made against the
        lists of generation `gen`; the default trusts no flow id and looks every
        frame up again on the live lists.  rcs (int32[n], optional) receives the
        per-frame return codes"""
        arr, keep = self.mbufs(frames)
        verdicts = np.ascontiguousarray(verdicts, VERDICT_DTYPE)
        r = self.lib.nstack_deliver(C.cast(arr, _vp), len(frames), _ptr(verdicts), gen, _ptr(rcs))
        self._let_go(arr, len(frames), keep)
        if r < 0:
            _check(r, "nstack_deliver")
        return r

    def rx_burst(self, frames: list[bytes]):
        arr, keep = self.mbufs(frames)
        rcs = np.zeros(len(frames), np.int32)
        v = np.zeros(len(frames), VERDICT_DTYPE)
        r = self.lib.nstack_rx_burst(C.cast(arr, _vp), len(frames), _ptr(rcs), _ptr(v))
        self._let_go(arr, len(frames), keep)
        if r < 0:
            _check(r, "nstack_rx_burst")
        return r, rcs, v

    def rx_submit(self, frames: list[bytes]):
        """nstack_rx_submit: the burst goes to the GPU; rx_complete delivers it"""
        arr, keep = self.mbufs(frames)
        rcs = np.zeros(len(frames), np.int32)
        v = np.zeros(len(frames), VERDICT_DTYPE)
        r = self.lib.nstack_rx_submit(C.cast(arr, _vp), len(frames), _ptr(rcs), _ptr(v))
        if r < 0:
            _check(r, "nstack_rx_submit")
        if not hasattr(self, "_pend"):
            self._pend = []
        self._pend.append((arr, len(frames), keep, rcs, v))
        return r

    def rx_complete(self):
        """nstack_rx_complete: deliver the oldest submitted burst: (delivered, rcs, verdicts)
        of that burst, as rx_burst returns them"""
        r = self.lib.nstack_rx_complete()
        arr, n, keep, rcs, v = self._pend.pop(0)
        self._let_go(arr, n, keep)
        if r < 0:
            _check(r, "nstack_rx_complete")
        return r, rcs, v

    def rx_pending(self) -> int:
        return int(self.lib.nstack_rx_pending())

    def rx_submit_mbufs(self, arr, n: int, rcs: np.ndarray | None = None) -> int:
        """nstack_rx_submit over prebuilt descriptors (mbufs_over); keep arr
        (and rcs) alive until rx_complete_mbufs"""
        r = self.lib.nstack_rx_submit(C.cast(arr, _vp), n, _ptr(rcs), None)
        if r < 0:
            _check(r, "nstack_rx_submit")
        return r

    def rx_complete_mbufs(self) -> int:
        r = self.lib.nstack_rx_complete()
        if r < 0:
            _check(r, "nstack_rx_complete")
        return r

    def _let_go(self, arr, n, keep):
        """after a burst call: in place, the frames stay alive while the stack
        holds them (kept here until fini) and the caller's references go"""
        if getattr(self, "_inplace", False):
            self._held.append((arr, keep))
            self.lib.nstack_mbufs_put(C.cast(arr, _vp), n)

    def set_rx_inplace(self, on: bool = True):
        """nstack_set_rx_inplace (no release callback: poll Mbuf.refcnt)"""
        self._inplace = bool(on)
        if not hasattr(self, "_held"):
            self._held = []
        _check(self.lib.nstack_set_rx_inplace(1 if on else 0, None, None), "nstack_set_rx_inplace")

    def reclaim(self):
        """nstack_reclaim: free what application threads let go of (protocol thread)"""
        self.lib.nstack_reclaim()

    def mbufs_put(self, arr, n: int):
        """nstack_mbufs_put: drop the caller's reference on n mbufs"""
        self.lib.nstack_mbufs_put(C.cast(arr, _vp), n)

    def drain_all_sum(self, buf: np.ndarray):
        """nstack_drain_all_sum: (items received, bytes, sum of FNV-1a 64 of what each read returned)"""
        nb, hs = _u64(), _u64()
        r = self.lib.nstack_drain_all_sum(_ptr(buf), buf.nbytes, C.byref(nb), C.byref(hs))
        if r < 0:
            _check(int(r), "nstack_drain_all_sum")
        return int(r), nb.value, hs.value

    @staticmethod
    def mbufs_over(pkts: np.ndarray, off: np.ndarray, lens: np.ndarray, off_unit_log2: int):
        """rte_mbuf-shaped descriptors over a packed burst (no copies; keep
        pkts alive while they are used): (array, n)"""
        n = len(off)
        ms = (Mbuf * n)()
        base = pkts.ctypes.data
        for i in range(n):
            ms[i].buf_addr = base + (int(off[i]) << off_unit_log2)
            ms[i].data_len = int(lens[i])
            ms[i].refcnt = 1  # the caller's reference (rte_pktmbuf_alloc)
        arr = (C.POINTER(Mbuf) * n)(*[C.pointer(ms[i]) for i in range(n)])
        return arr, ms

    def rx_burst_mbufs(self, arr, n: int, rcs: np.ndarray | None = None) -> int:
        """nstack_rx_burst over prebuilt descriptors (mbufs_over)"""
        r = self.lib.nstack_rx_burst(C.cast(arr, _vp), n, _ptr(rcs), None)
        if r < 0:
            _check(r, "nstack_rx_burst")
        # a two-half burst whose second half failed returns the first half's
        # count and reports the error per frame in rcs: raise it
        if rcs is not None and n and int(rcs[:n].min()) < -3:  # (the reference's own codes are -3..1)
            _check(int(rcs[:n].min()), "nstack_rx_burst (second half)")
        return r

    def drain_all(self, buf: np.ndarray):
        """nstack_drain_all: (items received, bytes)"""
        nb = _u64()
        r = self.lib.nstack_drain_all(_ptr(buf), buf.nbytes, C.byref(nb))
        if r < 0:
            _check(int(r), "nstack_drain_all")
        return int(r), nb.value

    def stat(self, which):
        return self.lib.nstack_stat(which)

    def set_local(self, ip: str, mac: bytes):
        """gLocalIp + port MAC (netfamily.c:11, 415)"""
        return self.lib.nstack_set_local(ip_raw(ip), (C.c_uint8 * 6)(*mac))

    def arp_insert(self, ip: str, mac: bytes) -> int:
        return self.lib.nstack_arp_insert(ip_raw(ip), (C.c_uint8 * 6)(*mac))

    def tx_burst(self, max_frames: int = 256, cap_bytes: int = 1 << 20, cksum: bool = False):
        """one udp_out + tcp_out pass: the frames (bytes) it produced"""
        pk = np.zeros(cap_bytes, np.uint8)
        off = np.zeros(max(max_frames, 1), np.uint32)
        ln = np.zeros(max(max_frames, 1), np.uint16)
        span = C.c_uint64()
        r = self.lib.nstack_tx_burst(_ptr(pk), cap_bytes, _ptr(off), _ptr(ln), max_frames,
                                     int(cksum), C.byref(span))
        if r < 0:
            _check(r, "nstack_tx_burst")
        return [pk[int(o) << 6:(int(o) << 6) + int(n)].tobytes() for o, n in zip(off[:r], ln[:r])]


_COMPILED = {}


def compiled_variants(vs):
    """the variants of `vs` the loaded library has compiled in, in order
    (the product library: KERNEL_VARIANTS; the RX_DIAG build, RXGPU_LIB=
    .../librxgpu_diag.so: also its tuning shapes and ablations).  A variant
    in none of the three lists is an error, not a silent skip"""
    known = set(map(tuple, KERNEL_VARIANTS + DIAG_TUNING_VARIANTS + DIAG_ABLATIONS))
    unknown = [tuple(v) for v in vs if tuple(v) not in known]
    if unknown:
        raise ValueError(f"variants in no build's table: {unknown}")
    out = []
    with Context(HOST_ONLY) as c:
        for v in vs:
            v = tuple(v)
            if v not in _COMPILED:
                try:
                    c.tune(*v)
                    _COMPILED[v] = True
                except RxgError:
                    _COMPILED[v] = False
            if _COMPILED[v]:
                out.append(v)
        c.tune(0)
    return out
