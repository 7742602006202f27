"""Whole-burst verdict digests (test infrastructure: tests/, bench.py parity leg).

Two digests of one burst's verdict array (SURVEY.md §4 item 4, §8(c)
transport rule: "SHA-256 digests of full-config verdict arrays"):

- ``verdict_sha256``: SHA-256 of the n x 16 verdict bytes in frame order (the
  unsharded burst, 1 GPU);
- ``frame_digest``: an order-independent digest, sum over frames i of
  H(i, verdict_i) mod 2**64, so ranks that each hold an RSS shard of the burst
  (bench.py --gpus N) add their partial sums and compare the total.

H is a splitmix64-style mix of the frame index and the verdict's two
little-endian u64 halves; the numpy form (host) and the torch form (device,
int64 arithmetic that wraps, logical shifts emulated) are checked against each
other in tests/test_digest.py.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "digests.json")

_C1, _C2, _C3 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB
_M64 = (1 << 64) - 1


def _mix_np(z):
    z = z + np.uint64(_C1)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(_C2)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(_C3)
    return z ^ (z >> np.uint64(31))


def frame_hash_np(idx: np.ndarray, verdicts: np.ndarray) -> np.ndarray:
    """H(i, v) for frame indices idx (int/uint64) and verdicts (n x 16 bytes)"""
    v = np.ascontiguousarray(verdicts).view(np.uint8).reshape(-1, 16).view(np.uint64)
    i = np.asarray(idx, np.uint64)
    with np.errstate(over="ignore"):
        h = _mix_np(v[:, 0] ^ _mix_np(i))
        return _mix_np(h ^ v[:, 1])


def frame_digest_np(idx, verdicts) -> int:
    with np.errstate(over="ignore"):
        return int(frame_hash_np(idx, verdicts).sum(dtype=np.uint64))


def _s64(c: int) -> int:
    return c - (1 << 64) if c >= 1 << 63 else c


def _srl(x, s: int):
    """logical right shift of int64 tensor x"""
    return (x >> s) & ((1 << (64 - s)) - 1)


def _mix_t(z):
    z = z + _s64(_C1)
    z = (z ^ _srl(z, 30)) * _s64(_C2)
    z = (z ^ _srl(z, 27)) * _s64(_C3)
    return z ^ _srl(z, 31)


def frame_digest_torch(idx, verdicts) -> int:
    """the same digest on the device: idx int64 tensor (global frame indices),
    verdicts a uint8 tensor of len(idx) x 16 bytes on the same device"""
    v = verdicts.reshape(-1, 16).view(dtype=__import__("torch").int64)
    h = _mix_t(v[:, 0] ^ _mix_t(idx))
    h = _mix_t(h ^ v[:, 1])
    return int(h.sum().item()) & _M64  # int64 sum wraps like u64


def verdict8_torch(verdicts):
    """rxgpu.verdict8_of on the device: a uint8 tensor of n x 16 verdict bytes
    -> n x 8 bytes (rxg_verdict8)"""
    import torch
    v = verdicts.reshape(-1, 16).view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    x, y, z, w = v[:, 0], v[:, 1], v[:, 2], v[:, 3]
    hi = ((y >> 16) | ((y & 0x7F) << 16) | ((w & 0x200) << 14) | (((z >> 16) & 7) << 24)
          | (((z >> 24) & 7) << 27) | ((w & 1) << 30) | ((w & 0x100) << 23))
    return (x | (hi << 32)).contiguous().view(torch.uint8)


def sha256_bytes(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def counts_sha256(counts: np.ndarray) -> str:
    return sha256_bytes(np.ascontiguousarray(counts, "<u8"))


def load_golden() -> dict:
    with open(GOLDEN) as f:
        return json.load(f)
