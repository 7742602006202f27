import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "dpdk-tcp-udp_protocol_stack_amd")
import numpy as np, torch
import rxgpu as R, oracle_bind as O
from test_tx import _fuzz_burst
buf, off, lens = _fuzz_burst()
want = O.tx_cksum(buf, off, lens, 4)
dev = torch.device("cuda", 0)
with R.Context(0, max_pkts=len(off), max_bytes=len(buf) + 64) as ctx:
    got = ctx.tx_cksum(buf, off, lens, 4)
    for name, g in [("host", got)] + [(h, None) for h in (64, 1500, 9000)]:
        if g is None:
            d = torch.from_numpy(buf.copy()).to(dev)
            ctx.tx_cksum_dev(d, torch.from_numpy(off.view(np.int32)).to(dev), torch.from_numpy(lens.view(np.int16)).to(dev), len(off), 4, name, torch.cuda.current_stream(dev).cuda_stream)
            torch.cuda.synchronize(dev); g = d.cpu().numpy()
        bad = np.nonzero(g != want)[0]
        fr = sorted(set(int(np.searchsorted((off.astype(np.int64) << 4), b, side="right") - 1) for b in bad))
        print(name, "bad bytes", len(bad), "frames", len(fr))
        for i in fr[:6]:
            s = int(off[i]) << 4; c = int(lens[i])
            pos = [int(b) - s for b in bad if s <= b < s + 2048][:8]
            print("  frame", i, "cap", c, "et", buf[s+12:s+14].tobytes().hex(), "proto", buf[s+23], "tl", int.from_bytes(buf[s+16:s+18].tobytes(), "big"), "pos", pos,
                  "got", [int(g[s+p]) for p in pos], "want", [int(want[s+p]) for p in pos], "orig", [int(buf[s+p]) for p in pos])
