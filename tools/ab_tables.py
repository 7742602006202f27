#!/usr/bin/env python3
"""A/B of flow-table layouts on one burst, interleaved in one process (GPU).

For each workload: the burst is generated once in HBM; each round re-syncs
the flow tables with every layout in turn (rxg_tune_tables flags x
rxg_tune_flow_load) and times K1 back to back (HIP events), without and with
per-flow counts.  Median and min over rounds.  Verdicts are checked equal
across layouts (they must not depend on the layout).

    python tools/ab_tables.py [cfg4,cfg5] [rounds] [layout,layout...]

count4B = the default layout with 4-B count indices (the round-1 count
path), against which the counts columns of port+1/4 compare.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

LAYOUTS = [("port+1/4", 0, 0), ("hash+1/4", R.TT_NO_UDP_PORT, 0), ("port+1/2", 0, 1),
           ("port+1/8", 0, 3), ("count4B", R.TT_COUNT_4B, 0)]


def main():
    names = (sys.argv[1] if len(sys.argv) > 1 else "cfg4").split(",")
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    pick = sys.argv[3].split(",") if len(sys.argv) > 3 else None
    layouts = [lay for lay in LAYOUTS if pick is None or lay[0] in pick]
    dev = torch.device("cuda", 0)
    ctx = R.Context(0)
    sh = torch.cuda.current_stream(dev).cuda_stream
    for nm in names:
        w = rxdist.WORKLOADS[nm]
        cfg = rxdist.gen_cfg(nm)
        n = w["n"]
        udp, tcb = R.gen_flows(cfg)
        pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(n, dtype=torch.int32, device=dev)
        ln = torch.empty(n, dtype=torch.int16, device=dev)
        R.gen_dev(cfg, 0, n, pk, off, ln, w["unit_log2"], stream=sh)
        torch.cuda.synchronize(dev)
        alg = int(ln.to(torch.int64).bitwise_and(0xFFFF).sum().item()) + 22 * n
        out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        ref = None
        cnt = torch.zeros(len(udp) + len(tcb), dtype=torch.int64, device=dev)
        times = {(lay[0], c): [] for lay in layouts for c in (False, True)}
        for r in range(rounds):
            for name, flags, load in layouts:
                ctx.tune_tables(flags)
                ctx.tune_flow_load(load)
                ctx.flows_sync(udp, tcb)
                for with_counts in (False, True):
                    c = cnt if with_counts else None
                    for _ in range(30 if r == 0 else 5):
                        ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, c,
                                         stream=sh)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(10):
                        ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, c,
                                         stream=sh)
                    b.record()
                    torch.cuda.synchronize(dev)
                    times[(name, with_counts)].append(a.elapsed_time(b) / 10)
                    if ref is None:
                        ref = out.clone()
                    elif not torch.equal(ref, out):
                        raise SystemExit(f"{nm} {name}: verdicts differ between layouts")
        for (name, wc), t in times.items():
            t = sorted(t)
            med = t[len(t) // 2]
            print(f"{nm} {name:9s} {'+counts' if wc else 'K1 only'}: median {med:.4f} ms min "
                  f"{t[0]:.4f} ms -> {alg / med / 1e6:.0f} GB/s ({alg / med / 8e9 * 100:.1f}% of 8 TB/s)",
                  flush=True)
        del pk, off, ln, out
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
