#!/usr/bin/env python3
"""A/B of the per-flow count passes above 8192 flows, interleaved in one
process (GPU): the bench's step loop (classify on the main stream, the count
passes of burst k on a second stream beside burst k+1's classify) and the
same with every pass on one stream, against the classify kernel alone
without counts.  Median and min over rounds; the counts
of each mode are checked against the verdicts.  "K1" is the classify
dispatch alone (a HIP event pair around each launch on the main stream, the
count passes on the count stream), summed over the steps.

    python tools/ab_counts.py [cfg4] [rounds] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))

import torch  # noqa: E402

import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

# (name, count stream?, rxg_tune_tables flags).  profiles/r03d/ also holds a
# run with two count variants since removed: a "lite" slab pass (16384-flow
# ranges in 32 KiB of LDS, to share CUs with the classify kernel) and count
# indices stored write-through; neither was faster
MODES = [("no counts", None, 0), ("count stream", True, 0), ("one stream", False, 0)]


def main():
    names = (sys.argv[1] if len(sys.argv) > 1 else "cfg4").split(",")
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
        pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
        off = torch.empty(n, dtype=torch.int32, device=dev)
        ln = torch.empty(n, dtype=torch.int16, device=dev)
        out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(ctx.num_flows, dtype=torch.int64, device=dev)
        R.gen_dev(cfg, 0, n, pk, off, ln, ul, stream=st.cuda_stream)
        torch.cuda.synchronize(dev)
        times = {m[0]: [] for m in MODES}
        k1 = {m[0]: [] for m in MODES}
        n_ok = None
        for rnd in range(rounds):
            for name, mode, flags in MODES:
                ctx.tune_tables(flags)
                c = cnt if mode is not None else None
                csh = cs.cuda_stream if mode else None
                cnt.zero_()
                for _ in range(5):
                    ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, c,
                                     stream=st.cuda_stream, count_stream=csh)
                torch.cuda.synchronize(dev)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                for _ in range(steps):
                    ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, c,
                                     stream=st.cuda_stream, count_stream=csh)
                st.wait_stream(cs)
                b.record(st)
                torch.cuda.synchronize(dev)
                times[name].append(a.elapsed_time(b) / steps)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(steps)]
                for e0, e1 in evs:
                    e0.record(st)
                    ctx.classify_dev(pk, off, ln, n, ul, w["len_hint"], out, c,
                                     stream=st.cuda_stream, count_stream=csh)
                    e1.record(st)
                st.wait_stream(cs)
                torch.cuda.synchronize(dev)
                k1[name].append(sum(e0.elapsed_time(e1) for e0, e1 in evs) / steps)
                if n_ok is None:
                    v = out.view(n, 16)
                    n_ok = int((v[:, 11].view(torch.int8) == 0).sum().item())
                if mode is not None:
                    got = int(cnt.sum().item())
                    assert got == n_ok * (2 * steps + 5), (nm, name, got, n_ok * (2 * steps + 5))
        ctx.tune_tables(0)
        base = sorted(times["no counts"])[rounds // 2]
        for name, _, _ in MODES:
            t = sorted(times[name])
            med = t[rounds // 2]
            k = sorted(k1[name])[rounds // 2]
            print(f"{nm} {name:>22}: step median {med:.4f} ms min {t[0]:.4f} ms "
                  f"({(med / base - 1) * 100:+.1f}% vs no counts), K1 median {k:.4f} ms "
                  f"(step {(med / k - 1) * 100:+.1f}% vs K1)  {['%.4f' % x for x in times[name]]}",
                  flush=True)
        del pk, off, ln, out, cnt
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
