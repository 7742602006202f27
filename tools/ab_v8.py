#!/usr/bin/env python3
"""A/B of the verdict format, interleaved in one process (GPU): the bench's
step (classify with per-flow counts; above 8192 flows the count passes on a
second stream) writing 16-B verdicts (rxg_classify_dev_cs) against 8-B ones
(rxg_classify_dev8).  Median and min over rounds.  The 8-B verdicts of the
last round are checked against the projection of the 16-B ones, every frame.

    python tools/ab_v8.py [cfg2,cfg3,cfg4,cfg5] [rounds] [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402


def main():
    names = (sys.argv[1] if len(sys.argv) > 1 else "cfg2,cfg3,cfg4,cfg5").split(",")
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    dev = torch.device("cuda", 0)
    ctx = R.Context(0)
    for nm in names:
        w = rxdist.WORKLOADS[nm]
        cfg = rxdist.gen_cfg(nm)
        n, ul = w["n"], w["unit_log2"]
        udp, tcb = R.gen_flows(cfg)
        ctx.flows_sync(udp, tcb)
        st = torch.cuda.current_stream(dev)
        cs = torch.cuda.Stream(dev)
        csh = cs.cuda_stream if ctx.num_flows >= R.SLAB_MIN_FLOWS else None
        pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(n, dtype=torch.int32, device=dev)
        ln = torch.empty(n, dtype=torch.int16, device=dev)
        out16 = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        out8 = torch.empty(n * 8, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
        R.gen_dev(cfg, 0, n, pk, off, ln, ul, stream=st.cuda_stream)
        torch.cuda.synchronize(dev)
        frame_bytes = int(ln.to(torch.int64).bitwise_and(0xFFFF).sum().item())
        modes = [("16-B verdicts", ctx.classify_dev, out16, 22),
                 ("8-B verdicts", ctx.classify_dev8, out8, 14)]
        times = {m[0]: [] for m in modes}
        # clock ramp
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            for _ in range(8):
                ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out16, None,
                                 stream=st.cuda_stream)
            torch.cuda.synchronize(dev)
        for rnd in range(rounds):
            for name, fn, out, _ in modes:
                for _ in range(5):
                    fn(pk, off, ln, n, ul, w["len_hint"], out, cnt, stream=st.cuda_stream,
                       count_stream=csh)
                torch.cuda.synchronize(dev)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(steps):
                    fn(pk, off, ln, n, ul, w["len_hint"], out, cnt, stream=st.cuda_stream,
                       count_stream=csh)
                st.wait_stream(cs)
                b.record(st)
                torch.cuda.synchronize(dev)
                times[name].append(a.elapsed_time(b) / steps)
        v16 = out16.cpu().numpy().view(R.VERDICT_DTYPE)
        same = R.verdict8_of(v16).tobytes() == out8.cpu().numpy().tobytes()
        base = sorted(times[modes[0][0]])[rounds // 2]
        for name, _, _, vb in modes:
            t = sorted(times[name])
            med = t[rounds // 2]
            alg = frame_bytes + vb * n
            print(f"{nm} {name}: step median {med:.4f} ms min {t[0]:.4f} ms "
                  f"({(med / base - 1) * 100:+.1f}%), {n / med / 1e3:,.0f} Mpps, "
                  f"{alg / med / 1e6:,.0f} GB/s algorithmic ({alg / med / 1e6 / 8000:.1%} of 8 TB/s)"
                  f"  {['%.4f' % x for x in times[name]]}", flush=True)
        print(f"{nm} 8-B verdicts == projection of the 16-B ones, all {n} frames: {same}", flush=True)
        if not same:
            sys.exit(3)
        del pk, off, ln, out16, out8, cnt
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
