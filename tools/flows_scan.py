"""Flow-count scan (diagnostics): K1 time on a workload's frame mix at several
flow-table sizes, to separate table locality (L2 / Infinity Cache / HBM) from
the byte stream.  python tools/flows_scan.py cfg4 "512,512;4096,4095;32768,32767" """
import sys

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..",
                                              "dpdk-tcp-udp_protocol_stack_amd"))
import rxdist  # noqa: E402
import rxgpu as R  # noqa: E402

name = sys.argv[1]
sets = [tuple(int(x) for x in s.split(",")) for s in sys.argv[2].split(";")]
w = rxdist.WORKLOADS[name]
dev = torch.device("cuda:0")
ctx = R.Context(0)
sh = torch.cuda.current_stream(dev).cuda_stream
n = w["n"]
for nu, nt in sets:
    cfg = rxdist.gen_cfg(name, n_udp=nu, n_tcp=nt)
    udp, tcb = R.gen_flows(cfg)
    ctx.flows_sync(udp, tcb)
    pk = torch.empty(n * cfg.slot_bytes + 64, dtype=torch.uint8, device=dev)
    off = torch.empty(n, dtype=torch.int32, device=dev)
    ln = torch.empty(n, dtype=torch.int16, device=dev)
    out = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    R.gen_dev(cfg, 0, n, pk, off, ln, w["unit_log2"], stream=sh)
    ts = []
    for rnd in range(4):
        for _ in range(3):
            ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, None, stream=sh)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            ctx.classify_dev(pk, off, ln, n, w["unit_log2"], w["len_hint"], out, None, stream=sh)
        b.record()
        torch.cuda.synchronize(dev)
        ts.append(a.elapsed_time(b) / 10)
    ts.sort()
    print(f"flows {name} udp={nu} tcp={nt}: median {ts[len(ts) // 2]:.4f} ms", flush=True)
    del pk, off, ln, out
    torch.cuda.empty_cache()
ctx.close()
