#!/usr/bin/env python3
"""SQ/TCC counter passes over bench.py for the classify kernel (diagnostics).

  python tools/pmc_counters.py <tag> <workload> "<bench extra args>" "CNT1 CNT2 ..." ["CNT ..."]
Each quoted counter list is one rocprofv3 --pmc pass (counters only, no
traces).  Prints the median per-dispatch value of every counter for the
rx_classify* kernel; raw CSVs stay under gpurun_out/.
"""
import csv
import glob
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, wl, extra = sys.argv[1], sys.argv[2], sys.argv[3].split()
    passes = sys.argv[4:]
    res = {}
    for i, group in enumerate(passes):
        d = os.path.join(ROOT, "gpurun_out", f"pmcx_{tag}_{wl}_{i}")
        cmd = ["rocprofv3", "--pmc", *group.split(), "--output-format", "csv", "-d", d, "-o", "run",
               "--", sys.executable, os.path.join(ROOT, "bench.py"), "--workload", wl, "--steps",
               "3", "--warmup", "1", "--no-cpu", *extra]
        r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, TMPDIR="/tmp"),
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-2000:])
            raise SystemExit(r.returncode)
        vals = defaultdict(list)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "rx_classify" in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, v in vals.items():
            v.sort()
            res[k] = v[len(v) // 2]
    for k in sorted(res):
        print(f"{tag} {wl} {' '.join(extra)} {k} = {res[k]:.6g}", flush=True)


if __name__ == "__main__":
    main()
