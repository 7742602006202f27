#!/usr/bin/env python3
"""A/B of two builds of librxgpu across bench processes on one box,
interleaved: python tools/ab_lib.py <other.so> [workloads] [rounds]
Each round runs bench.py once per library (RXGPU_LIB selects the build) and
prints every workload's step and kernel-stream times."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
other = sys.argv[1]
wls = sys.argv[2] if len(sys.argv) > 2 else "cfg4,cfg2,cfg3,cfg5"
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
libs = {"default": "", os.path.basename(other): os.path.abspath(other)}
res = {k: {} for k in libs}
for r in range(rounds):
    for name, lib in libs.items():
        env = dict(os.environ)
        if lib:
            env["RXGPU_LIB"] = lib
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", wls, "--no-cpu",
               "--no-cfg1", "--no-sockrate", "--no-tx", "--no-v8", "--parity-sample", "256", "--steps", "50"]
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            print(p.stderr[-3000:])
            raise SystemExit(p.returncode)
        line = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
        first = wls.split(",")[0]
        per = {first: line}
        for w in wls.split(",")[1:]:
            per[w] = line[w]
        for w, d in per.items():
            res[name].setdefault(w, []).append((d["ms_per_step"], d["kernel_ms_avg"]))
            print(f"round {r} {name:>18} {w}: step {d['ms_per_step']:.4f} ms kernel-stream "
                  f"{d['kernel_ms_avg']:.4f} ms digest_ok {d['digest']['digest_ok']}", flush=True)
for name in libs:
    for w, v in res[name].items():
        st = sorted(x[0] for x in v)
        print(f"{name:>18} {w}: median step {st[len(st) // 2]:.4f} ms  {['%.4f' % x for x in st]}")
