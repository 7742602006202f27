#!/usr/bin/env python3
"""K2 (TX checksum) write-back per write mode, from rocprofv3 WRITE_SIZE.

The TX kernel patches 4 bytes per frame (the IPv4 and L4 checksum fields).
Its variants differ in how those bytes reach memory (tx_cksum.hip WB): 0 =
two 2-B stores, 1 = the 16-B chunk holding each field, 2 = the whole 64-B
head.  One counter pass (WRITE_SIZE only, nothing else collected) over
tools/tx_sweep.py runs each variant on the same burst; WRITE_SIZE per dispatch
is summarised by kernel (= variant), next to the algorithmic write (4 B per
frame).  Run on the GPU box:  python tools/pmc_tx.py r02c
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (workload, frames, variants): cfg2 64 B (WB 2 / 1 / 0 at G=4), cfg3 1500 B (G=8)
RUNS = [("cfg2", 16 << 20, "0,6,7"), ("cfg3", 4 << 20, "2,8,9")]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    outdir = os.path.join(ROOT, "gpurun_out")
    res = {"tag": tag, "method": "rocprofv3 --pmc WRITE_SIZE over tools/tx_sweep.py; median "
           "WRITE_SIZE (KiB) per dispatch of each tx_cksum_kernel instantiation", "runs": {}}
    for wl, n, variants in RUNS:
        d = os.path.join(outdir, f"pmc_tx_{wl}")
        cmd = ["rocprofv3", "--pmc", "WRITE_SIZE", "--output-format", "csv", "-d", d, "-o", "run",
               "--", sys.executable, os.path.join(ROOT, "tools", "tx_sweep.py"), wl, variants]
        r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, TMPDIR="/tmp"), capture_output=True,
                           text=True, timeout=240)
        if r.returncode != 0:
            sys.stderr.write(r.stdout[-3000:] + r.stderr[-3000:])
            raise SystemExit(r.returncode)
        vals = defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if row.get("Counter_Name") == "WRITE_SIZE" and "tx_cksum" in row["Kernel_Name"]:
                    k = row["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
                    vals[k].append(float(row["Counter_Value"]))
        out = {}
        for k, v in vals.items():
            v = sorted(v)
            kb = v[len(v) // 2]
            out[k] = {"write_size_kb": kb, "bytes_per_frame": round(kb * 1024 / n, 2),
                      "algorithmic_bytes_per_frame": 4, "dispatches": len(v)}
        res["runs"][wl] = out
        print(wl, json.dumps(out, indent=1), flush=True)
    with open(os.path.join(outdir, f"pmc_tx_{tag}.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
