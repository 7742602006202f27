#!/usr/bin/env python3
"""Which per-process state makes cfg2 ~5-9% slower in some processes?
(follows tools/cfg2_swing.py, which found every burst
copy inside one process equally fast.)

Run this several times as separate processes.  Each process times the cfg2
classify launch (16M x 64 B, 1024 UDP sockets, per-socket counts) on:
  A  context 1, the default stream (as bench.py)
  B  context 1, a second stream (another hardware queue)
  C  context 1, a high-priority stream
  D  context 2 (its own flow tables, workspace, code objects), default stream
  E  context 1, default stream, a burst copy allocated behind a 6 GiB spacer
interleaved over ROUNDS rounds of STEPS launches (HIP events on the stream
the launch runs on).  If A..E agree within a process while processes differ,
the cause is below everything a process can re-create (the box, its queues'
placement or the driver's page mapping), not our tables or buffers.
Prints one JSON object.  Diagnostics only."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))
import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402


def main():
    RND = int(os.environ.get("ROUNDS", "5"))
    S = int(os.environ.get("STEPS", "40"))
    W = 5
    t0 = time.perf_counter()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    name = "cfg2"
    w = rxdist.WORKLOADS[name]
    ul, lh = w["unit_log2"], w["len_hint"]
    udp, tcb = R.gen_flows(rxdist.gen_cfg(name))
    NCTX = int(os.environ.get("NCTX", "2"))
    ctxs = []
    for _ in range(NCTX):
        c = R.Context(0)
        c.flows_sync(udp, tcb)
        ctxs.append(c)
    ctx1, ctx2 = ctxs[0], ctxs[1]
    dflt = torch.cuda.current_stream(dev)
    s1 = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev, priority=-1)

    def burst(ctx):
        pk, off, ln, n, _, _ = rxdist.build_shard(ctx, name, 0, 1, dev, dflt)
        return dict(pk=pk, off=off, ln=ln, n=n,
                    out=torch.empty(n * 16, dtype=torch.uint8, device=dev),
                    cnt=torch.zeros(len(udp) + len(tcb), dtype=torch.int64, device=dev))

    b1 = burst(ctx1)
    spacer = torch.empty(6 << 30, dtype=torch.uint8, device=dev)
    spacer.fill_(1)
    b2 = burst(ctx1)
    del spacer
    torch.cuda.synchronize(dev)
    cases = dict(A=(ctx1, dflt, b1), B=(ctx1, s1, b1), C=(ctx1, s2, b1), D=(ctx2, dflt, b1),
                 E=(ctx1, dflt, b2))
    for j in range(2, NCTX):  # more contexts (their own tables), default stream
        cases["D%d" % j] = (ctxs[j], dflt, b1)
    launches = []  # (case, classify launches) in launch order: maps a kernel trace

    def timed(ctx, st, b, steps, tag="ramp"):
        launches.append((tag, W + steps))
        sh = st.cuda_stream
        for _ in range(W):
            ctx.classify_dev(b["pk"], b["off"], b["ln"], b["n"], ul, lh, b["out"], b["cnt"],
                             stream=sh)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        a.record(st)
        for _ in range(steps):
            ctx.classify_dev(b["pk"], b["off"], b["ln"], b["n"], ul, lh, b["out"], b["cnt"],
                             stream=sh)
        e.record(st)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(e) / steps

    # the bench's ramp: ~200 ms on case A first
    t_r = time.perf_counter() + 0.2
    while time.perf_counter() < t_r:
        timed(*cases["A"], 8)
    per = {k: [] for k in cases}
    for _ in range(RND):
        for k, c in cases.items():
            per[k].append(round(timed(*c, S, tag=k), 4))
    med = {k: sorted(v)[len(v) // 2] for k, v in per.items()}
    ref = b1["out"].clone()
    timed(*cases["D"], 1, tag="check")
    same = bool(torch.equal(ref, b1["out"]))
    # the launch log, run-length encoded
    rle = []
    for t, n in launches:
        if rle and rle[-1][0] == t:
            rle[-1][1] += n
        else:
            rle.append([t, n])
    print(json.dumps(dict(pid=os.getpid(), median_ms=med, rounds=per, d_equal_a=same,
                          launches=rle, steps=S, warmup=W,
                          addr=dict(b1=hex(b1["pk"].data_ptr()), b2=hex(b2["pk"].data_ptr())),
                          t_s=round(time.perf_counter() - t0, 1))), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
