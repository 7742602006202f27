#!/usr/bin/env python3
"""L2 (TCC) hits of the flow-table probes: the TCC request / hit / miss
counters of the classify kernel with the probe (SH, pipe 64) and without it
(the no-probe ablation, pipe 160: the flow id from the port, wrong verdicts
by construction), one rocprofv3 --pmc pass each, nothing else collected.
The differences are the probes' own requests, hits and misses.
Run on the GPU box:  python tools/pmc_probe_hits.py [workload] [tag] [ablation pipe]
(ablation pipe 264: without the partial-last-chunk load instead of the probe)"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNTERS = ["TCC_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum"]  # 3 of the 4 TCC slots


def collect(workload, variant, outdir):
    d = os.path.join(outdir, f"pmc_hits_{workload}_{variant.replace(',', '-')}")
    cmd = ["rocprofv3", "--pmc", *COUNTERS, "--output-format", "csv", "-d", d, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--steps", "3",
           "--warmup", "1", "--no-cpu", "--no-cfg1", "--no-sockrate", "--no-tx", "--no-v8",
           "--parity-sample", "0", "--variant", variant]
    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, TMPDIR="/tmp"), capture_output=True,
                       text=True, timeout=240)
    # the ablation's verdicts are wrong by construction: bench.py exits 3 on them
    if r.returncode not in ((0, 3) if int(variant.split(",")[-1]) >= 100 else (0,)):
        sys.stderr.write(r.stdout[-3000:] + r.stderr[-3000:])
        raise SystemExit(r.returncode)
    vals = {c: [] for c in COUNTERS}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            c = row.get("Counter_Name")
            if c in vals and "rx_classify" in row.get("Kernel_Name", ""):
                vals[c].append(float(row["Counter_Value"]))
    if not all(vals.values()):
        raise SystemExit(f"no rx_classify rows for {workload} {variant}")
    return {c: sorted(v)[len(v) // 2] for c, v in vals.items()}  # median over dispatches


def main():
    w = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    tag = sys.argv[2] if len(sys.argv) > 2 else "r03"
    outdir = os.path.join(ROOT, "gpurun_out")
    res = {"workload": w, "counters": COUNTERS, "per_dispatch_median": {}}
    abl = sys.argv[3] if len(sys.argv) > 3 else "160"
    for name, v in (("probe", "0,1,1,64"), ("no_probe", "0,1,1," + abl)):
        res["per_dispatch_median"][name] = collect(w, v, outdir)
        print(name, res["per_dispatch_median"][name], flush=True)
    a, b = res["per_dispatch_median"]["probe"], res["per_dispatch_median"]["no_probe"]
    dreq, dhit = a["TCC_REQ_sum"] - b["TCC_REQ_sum"], a["TCC_HIT_sum"] - b["TCC_HIT_sum"]
    res["probe_requests"] = dreq
    res["probe_hits"] = dhit
    res["probe_hit_rate"] = dhit / dreq if dreq > 0 else None
    res["kernel_hit_rate"] = a["TCC_HIT_sum"] / max(a["TCC_REQ_sum"], 1.0)
    print(json.dumps(res), flush=True)
    res["ablation_pipe"] = int(abl)
    with open(os.path.join(outdir, f"pmc_probe_hits_{w}_{tag}_{abl}.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
