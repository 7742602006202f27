"""The compact 8-B verdict (rxg_verdict8, include/rxgpu.h; written by
rxg_classify_dev8).  CPU: the header's rxg_verdict8_of and RXG_V8_* decode
macros (compiled with gcc from include/rxgpu.h) agree with rxgpu.verdict8_of,
and decoding gives back every field the 8-B form keeps (flow id, payload
window, class, return code, checksum pass/fail, flags) for every verdict shape
the kernels produce.  The GPU side is in test_gpu_parity.py (every variant,
v8=True) and test_digest.py (whole bursts against verdict8_sha256)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import rxgpu as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include "rxgpu.h"
void conv(const rxg_verdict *v, rxg_verdict8 *o, int n) {
    for (int i = 0; i < n; ++i) o[i] = rxg_verdict8_of(&v[i]);
}
/* per verdict: payload_off, cls, rc, cksum_ok, flags */
void decode(const rxg_verdict8 *v, int *o, int n) {
    for (int i = 0; i < n; ++i) {
        o[5 * i + 0] = (int)RXG_V8_PAYLOAD_OFF(v[i]);
        o[5 * i + 1] = (int)RXG_V8_CLS(v[i]);
        o[5 * i + 2] = RXG_V8_RC(v[i]);
        o[5 * i + 3] = (int)RXG_V8_CKSUM_OK(v[i]);
        o[5 * i + 4] = (int)RXG_V8_FLAGS(v[i]);
    }
}
"""


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("v8")
    c = d / "v8.c"
    c.write_text(SRC)
    so = d / "libv8.so"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-O2", "-shared", "-fPIC",
                    "-I", os.path.join(ROOT, "include"), str(c), "-o", str(so)], check=True)
    return C.CDLL(str(so))


def _verdicts(rng, n):
    """16-B verdicts of the shapes the kernels write (rxgpu.h field rules)"""
    v = np.zeros(n, R.VERDICT_DTYPE)
    cls = rng.integers(0, 5, n)
    v["cls"] = cls
    v["flow_id"] = np.where(rng.random(n) < 0.2, 0xFFFFFFFF, rng.integers(0, 1 << 32, n))
    hl = rng.integers(0, 16, n)
    v["payload_off"] = np.select([cls == R.CLS_UDP, cls == R.CLS_TCP], [42, 34 + 4 * hl], 0)
    v["payload_len"] = np.where(cls >= R.CLS_UDP, rng.integers(0, 65536, n), 0)
    v["payload_len"][rng.random(n) < 0.1] = 0
    udp_rc = rng.choice([0, -2, -3], n)
    tcp_rc = rng.choice([0, -1, -2], n)
    v["rc"] = np.select([cls == R.CLS_UDP, cls == R.CLS_TCP], [udp_rc, tcp_rc], 1)
    v["cksum_ok"] = rng.integers(0, 2, n)
    trunc = rng.integers(0, 2, n)
    neglen = (cls == R.CLS_TCP) & (v["payload_len"] == 0) & (rng.random(n) < 0.5)
    short = (cls == R.CLS_UDP) & (v["payload_len"] == 0)
    v["flags"] = trunc | (neglen * 2) | (short * 4)
    v["l4_cksum"] = rng.integers(0, 65536, n)
    v["stored_cksum"] = rng.integers(0, 65536, n)
    return v


def test_header_projection_equals_numpy(lib):
    rng = np.random.default_rng(8)
    v = _verdicts(rng, 20000)
    o = np.zeros(len(v), R.VERDICT8_DTYPE)
    lib.conv(v.ctypes.data_as(C.c_void_p), o.ctypes.data_as(C.c_void_p), C.c_int(len(v)))
    assert o.tobytes() == R.verdict8_of(v).tobytes()


def test_torch_projection_equals_numpy():
    import torch

    import digest as D
    v = _verdicts(np.random.default_rng(10), 5000)
    t = D.verdict8_torch(torch.from_numpy(v.view(np.uint8).copy()))
    assert t.numpy().tobytes() == R.verdict8_of(v).tobytes()


def test_decode_recovers_every_kept_field(lib):
    rng = np.random.default_rng(9)
    v = _verdicts(rng, 20000)
    v8 = R.verdict8_of(v)
    d = np.zeros((len(v), 5), np.int32)
    lib.decode(v8.ctypes.data_as(C.c_void_p), d.ctypes.data_as(C.c_void_p), C.c_int(len(v)))
    assert np.array_equal(v8["flow_id"], v["flow_id"])
    assert np.array_equal(v8["payload_len"], v["payload_len"])
    assert np.array_equal(d[:, 0], v["payload_off"])
    assert np.array_equal(d[:, 1], v["cls"])
    assert np.array_equal(d[:, 2], v["rc"])
    assert np.array_equal(d[:, 3], v["cksum_ok"])
    assert np.array_equal(d[:, 4], v["flags"])


def test_oracle_edge_fixture_round_trips(lib):
    """the oracle's verdicts of the edge pcap (every class, return code and
    flag the kernels produce) survive the projection"""
    want = np.load(os.path.join(ROOT, "tests", "golden", "edge_verdicts.npy"))
    v8 = R.verdict8_of(want)
    d = np.zeros((len(want), 5), np.int32)
    lib.decode(v8.ctypes.data_as(C.c_void_p), d.ctypes.data_as(C.c_void_p), C.c_int(len(want)))
    for k, f in enumerate(("payload_off", "cls", "rc", "cksum_ok", "flags")):
        assert np.array_equal(d[:, k], want[f]), f
