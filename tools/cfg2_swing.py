#!/usr/bin/env python3
"""Why does cfg2 run ~9% slower in some bench processes?

One process, one context, the cfg2 burst (16M x 64 B, 1 GiB) built K times
into separately allocated buffers (identical bytes).  Then:
  - the kernel timed on copy 0 first (as bench.py does, after its 200-ms ramp);
  - every copy timed interleaved over R rounds (W warmup + S timed steps
    each, HIP events), with the shader clock sampled by a one-wave probe
    (tools/libceiling.so clock_probe_*) on a second stream across each timed
    window;
  - the buffers' device addresses printed (virtual; the physical placement
    is the driver's).
If the copies differ from each other, placement is the cause; if copy 0's
first window differs from its later ones, the time since start (clocks) is.
Prints one JSON object on stdout.  Diagnostics only."""
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402


def smi():
    try:
        r = subprocess.run(["amd-smi", "metric", "-g", "0", "-c", "-p", "-t"],
                           capture_output=True, text=True, timeout=30)
        return r.stdout[-1500:]
    except Exception as e:  # diagnostics: report, do not fail
        return repr(e)


def main():
    K = int(os.environ.get("COPIES", "4"))
    RND = int(os.environ.get("ROUNDS", "5"))
    S = int(os.environ.get("STEPS", "50"))
    W = 5
    t_start = time.perf_counter()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = C.CDLL(os.path.join(ROOT, "tools", "libceiling.so"))
    probe_state = C.c_void_p(0)
    ps = torch.cuda.Stream(dev)

    def probe_start(ms):
        rc = lib.clock_probe_launch(0, C.c_void_p(ps.cuda_stream), C.c_double(ms),
                                    C.byref(probe_state))
        assert rc == 0, rc

    def probe_read():
        ps.synchronize()
        m = C.c_double(0)
        lib.clock_probe_read(0, probe_state, C.byref(m))
        return round(m.value, 1)

    out = dict(smi_start=smi())
    ctx = R.Context(0)
    name = "cfg2"
    w = rxdist.WORKLOADS[name]
    udp, tcb = R.gen_flows(rxdist.gen_cfg(name))
    ctx.flows_sync(udp, tcb)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ul, lh = w["unit_log2"], w["len_hint"]

    def build():
        pk, off, ln, n, _, _ = rxdist.build_shard(ctx, name, 0, 1, dev, stream)
        o = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        c = torch.zeros(len(udp) + len(tcb), dtype=torch.int64, device=dev)
        return dict(pk=pk, off=off, ln=ln, n=n, out=o, cnt=c, addr=hex(pk.data_ptr()))

    def timed(b, steps=S, probe=True):
        for _ in range(W):
            ctx.classify_dev(b["pk"], b["off"], b["ln"], b["n"], ul, lh, b["out"], b["cnt"],
                             stream=sh)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        if probe:
            probe_start(steps * 0.2)
        a.record(stream)
        for _ in range(steps):
            ctx.classify_dev(b["pk"], b["off"], b["ln"], b["n"], ul, lh, b["out"], b["cnt"],
                             stream=sh)
        e.record(stream)
        torch.cuda.synchronize(dev)
        return round(a.elapsed_time(e) / steps, 4), (probe_read() if probe else None)

    copies = [build()]
    # as bench.py: 200 ms ramp without counts, then warmup + timed
    b = copies[0]
    t_r = time.perf_counter() + 0.2
    while time.perf_counter() < t_r:
        for _ in range(8):
            ctx.classify_dev(b["pk"], b["off"], b["ln"], b["n"], ul, lh, b["out"], None,
                             stream=sh)
        torch.cuda.synchronize(dev)
    out["first_windows_copy0"] = [timed(b) for _ in range(3)]
    out["t_first_s"] = round(time.perf_counter() - t_start, 1)
    # a 6 GiB block allocated and freed between copies shifts where the next land
    for k in range(1, K):
        if k == K // 2:
            big = torch.empty(6 << 30, dtype=torch.uint8, device=dev)
            big.fill_(1)
            del big
        copies.append(build())
    out["addr"] = [c["addr"] for c in copies]
    per = {k: [] for k in range(K)}
    clk = {k: [] for k in range(K)}
    for r in range(RND):
        for k in range(K):
            ms, mhz = timed(copies[k])
            per[k].append(ms)
            clk[k].append(mhz)
    out["interleaved_ms"] = {k: v for k, v in per.items()}
    out["interleaved_median_ms"] = {k: sorted(v)[len(v) // 2] for k, v in per.items()}
    out["sclk_mhz"] = clk
    # the verdicts of every copy are the same bytes
    ref = copies[0]["out"]
    out["copies_equal"] = all(bool(torch.equal(ref, c["out"])) for c in copies[1:])
    out["last_windows_copy0"] = [timed(copies[0]) for _ in range(3)]
    out["smi_end"] = smi()
    out["t_total_s"] = round(time.perf_counter() - t_start, 1)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
