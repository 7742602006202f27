"""K2 (TX checksum) variant sweep: times every tx_cksum variant (rxg_tune_tx)
on the bench workloads, interleaved over rounds in one process.  Tuning only.
    python tools/tx_sweep.py cfg2,cfg3,cfg5 [variants] [bpc list]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))
import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["cfg2", "cfg3", "cfg5"]
variants = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(range(13))
bpcs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
dev = torch.device("cuda:0")
ctx = R.Context(0, max_pkts=1024, max_bytes=1 << 20)
for nm in names:
    w = rxdist.WORKLOADS[nm]
    cfg = rxdist.gen_cfg(nm)
    n = w["n"]
    sh = torch.cuda.current_stream(dev).cuda_stream
    pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n, dtype=torch.int32, device=dev)
    ln = torch.empty(n, dtype=torch.int16, device=dev)
    R.gen_dev(cfg, 0, n, pk, off, ln, w["unit_log2"], stream=sh)
    torch.cuda.synchronize(dev)
    fb = int(ln.to(torch.int64).bitwise_and(0xFFFF).sum().item())
    txb = fb + 10 * n
    times = {(v, b): [] for v in variants for b in bpcs}
    for rnd in range(5):
        for v, b in times:
            ctx.tune_tx(v, b)
            for _ in range(3):
                ctx.tx_cksum_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], stream=sh)
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                ctx.tx_cksum_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], stream=sh)
            e.record()
            torch.cuda.synchronize(dev)
            times[(v, b)].append(a.elapsed_time(e) / 10)
    for (v, b), t in times.items():
        t = sorted(t)
        print(f"tx {nm} variant={v} bpc={b}: median {t[2]:.4f} ms min {t[0]:.4f} -> "
              f"{n / t[2] / 1e3:.0f} Mpps {txb / t[2] / 1e6:.0f} GB/s ({txb / t[2] / 8e9:.3f} of 8 TB/s)",
              flush=True)
    del pk, off, ln
    torch.cuda.empty_cache()
ctx.tune_tx(R.TX_AUTO)
ctx.close()
