#!/usr/bin/env python3
"""Whole-burst oracle digests of every BASELINE config (tests/golden/digests.json).

For each config the full per-GPU burst (frames 0..n-1 of the deterministic
pktgen, the burst bench.py and the -m gpu digest test classify) is generated on
the host chunk by chunk, classified by the oracle (oracle/ref_cpu.c: the
reference's list-scan lookups and DPDK checksum, test infrastructure) on
`--threads` host threads, and reduced to:

  verdict_sha256  SHA-256 of the n x 16 verdict bytes in frame order
  verdict8_sha256 SHA-256 of the n x 8 compact verdicts (rxg_verdict8: the
                  16-B verdicts projected by rxgpu.verdict8_of, as
                  rxg_classify_dev8 writes them)
  frame_digest    sum over frames of H(i, verdict_i) mod 2**64 (tests/digest.py)
  counts_sha256   SHA-256 of the burst's per-flow histogram (u64 LE, UDP then TCP)
  rc / cls        verdict histograms (for reading)

Run once in the container (cfg4 and cfg5 take minutes to most of an hour: the
O(N) list scans over 65,536 and 1,048,576 control blocks), e.g.

    python tests/golden/make_digests.py cfg1 cfg2 cfg3 cfg4 --threads 8
    python tests/golden/make_digests.py cfg5 --threads 6

Entries are merged into digests.json with the wall time and thread count.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import digest as D  # noqa: E402
import oracle_bind as O  # noqa: E402
import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

CHUNK = {"cfg1": 1 << 16, "cfg2": 1 << 18, "cfg3": 1 << 15, "cfg4": 1 << 12, "cfg5": 1 << 10}


def digest_config(name: str, threads: int, n: int | None = None) -> dict:
    w = rxdist.WORKLOADS[name]
    cfg = rxdist.gen_cfg(name)
    ul = w["unit_log2"]
    n = w["n"] if n is None else n
    udp, tcb = R.gen_flows(cfg)
    tb = O.Tables(udp, tcb)
    nflows = len(udp) + len(tcb)
    step = CHUNK[name]
    starts = list(range(0, n, step))

    def work(s):
        k = min(step, n - s)
        pk, off, ln = R.gen_host(cfg, s, k, ul)
        v, cnt = tb.classify(pk, off, ln, ul, counts=True)
        return v, cnt

    sha = hashlib.sha256()
    sha8 = hashlib.sha256()
    fd = 0
    counts = np.zeros(max(nflows, 1), np.uint64)[:nflows]
    rc = {}
    cls = {}
    t0 = time.perf_counter()
    done = 0
    with cf.ThreadPoolExecutor(threads) as ex:
        for s, (v, cnt) in zip(starts, ex.map(work, starts)):  # results in frame order
            sha.update(v.tobytes())
            sha8.update(R.verdict8_of(v).tobytes())
            fd = (fd + D.frame_digest_np(np.arange(s, s + len(v), dtype=np.uint64), v)) & D._M64
            counts += cnt
            for key, hist in (("rc", rc), ("cls", cls)):
                u, c = np.unique(v[key], return_counts=True)
                for a, b in zip(u.tolist(), c.tolist()):
                    hist[str(a)] = hist.get(str(a), 0) + int(b)
            done += len(v)
            if done * 20 // n != (done - len(v)) * 20 // n:
                el = time.perf_counter() - t0
                print(f"{name}: {done}/{n} frames, {el:.0f} s", file=sys.stderr, flush=True)
    el = time.perf_counter() - t0
    return dict(workload=name, desc=w["desc"], frames=n, flows=nflows,
                verdict_sha256=sha.hexdigest(), verdict8_sha256=sha8.hexdigest(), frame_digest=f"{fd:016x}",
                counts_sha256=D.counts_sha256(counts), counted=int(counts.sum()),
                rc=rc, cls=cls, seconds=round(el, 1), threads=threads,
                host=platform.processor() or platform.machine(),
                how="oracle/ref_cpu.c -O2 over the pktgen burst (rxg_gen_host), frames 0..n-1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=D.GOLDEN)
    a = ap.parse_args()
    for nm in a.configs:
        r = digest_config(nm, a.threads)
        print(json.dumps(r), flush=True)
        cur = {}
        if os.path.exists(a.out):
            with open(a.out) as f:
                cur = json.load(f)
        cur[nm] = r
        with open(a.out, "w") as f:
            json.dump(dict(sorted(cur.items())), f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
