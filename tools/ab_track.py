#!/usr/bin/env python3
"""A/B in one process: the per-burst tracking event (rx_api.hip burst_end)
on vs off (RXG_TT_NO_TRACK), interleaved rounds of back-to-back bursts.
    python tools/ab_track.py [cfg2,cfg4] [rounds] [bursts]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))
import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

names = (sys.argv[1] if len(sys.argv) > 1 else "cfg2").split(",")
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 7
bursts = int(sys.argv[3]) if len(sys.argv) > 3 else 100
dev = torch.device("cuda", 0)
ctx = R.Context(0)
for nm in names:
    w = rxdist.WORKLOADS[nm]
    cfg = rxdist.gen_cfg(nm)
    udp, tcb = R.gen_flows(cfg)
    ctx.flows_sync(udp, tcb)
    n, ul = w["n"], w["unit_log2"]
    pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n, dtype=torch.int32, device=dev)
    ln = torch.empty(n, dtype=torch.int16, device=dev)
    st = torch.cuda.current_stream(dev)
    R.gen_dev(cfg, 0, n, pk, off, ln, ul, stream=st.cuda_stream)
    out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(max(ctx.num_flows, 1), dtype=torch.int64, device=dev)
    res = {0: [], R.TT_NO_TRACK: []}
    for _ in range(30):
        ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, cnt, stream=st.cuda_stream)
    for r in range(rounds):
        for flag in res:
            ctx.tune_tables(flag)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(bursts):
                ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, cnt, stream=st.cuda_stream)
            b.record(st)
            torch.cuda.synchronize(dev)
            res[flag].append(a.elapsed_time(b) / bursts)
    ctx.tune_tables(0)
    for flag, t in res.items():
        t = sorted(t)
        print(f"{nm} {'no-track' if flag else 'track   '}: median {t[len(t) // 2]:.4f} ms "
              f"min {t[0]:.4f} ms  {['%.4f' % x for x in t]}", flush=True)
    del pk, off, ln, out
    torch.cuda.empty_cache()
