#!/usr/bin/env python3
"""HBM traffic of the classify kernel from rocprofv3 PMC counters.

Two separate counter passes (TCC has 4 slots: FETCH_SIZE needs 3, WRITE_SIZE
2 — MI355X_MICROARCH.md §rocprofv3 PMC slots), each with nothing but the
counter collection, over `bench.py --workload <w> --no-cpu`.  Per dispatch of
rx_classify_kernel (and of K2 tx_cksum_kernel, the bench's TX leg): hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(gfx950 correction: FETCH_SIZE reports half the bytes of a wide coalesced
streaming read, MI355X_MICROARCH.md §HBM; WRITE_SIZE is exact for 16-B
stores).  Writes profiles/pmc_<tag>.json, which bench.py reads for
roofline.traffic.  Run on the GPU box:  python tools/pmc_traffic.py r01 cfg2,cfg3
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def collect(workload, counter, outdir, variant=""):
    d = os.path.join(outdir, f"pmc_{workload}_{counter}{'_' + variant.replace(',', '-') if variant else ''}")
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--steps", "3",
           "--warmup", "1", "--no-cpu", "--no-cfg1", "--no-sockrate", "--no-v8", "--parity-sample", "0"]
    if variant:  # a forced kernel variant (tuning comparisons)
        cmd += ["--variant", variant]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    if r.returncode != 0:
        sys.stderr.write(r.stdout[-3000:] + r.stderr[-3000:])
        raise SystemExit(r.returncode)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {"rx_classify": [], "tx_cksum": []}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            for k in vals:
                if k in row.get("Kernel_Name", ""):
                    vals[k].append(float(row["Counter_Value"]))
    return vals, files


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    wls = (sys.argv[2] if len(sys.argv) > 2 else "cfg2,cfg3").split(",")
    variant = sys.argv[3] if len(sys.argv) > 3 else ""  # e.g. 0,0,0,40
    outdir = os.path.join(ROOT, "gpurun_out")
    import hashlib
    sha = hashlib.sha256(open(os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd", "librxgpu.so"),
                              "rb").read()).hexdigest()
    # bench.py publishes roofline.traffic only from a summary of the same library
    res = {"tag": tag, "librxgpu_sha256": sha, "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
           "hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per rx_classify_kernel dispatch "
           "(median over dispatches)", "workloads": {}}
    for w in wls:
        fetch, ff = collect(w, "FETCH_SIZE", outdir, variant)
        write, wf = collect(w, "WRITE_SIZE", outdir, variant)
        if not fetch["rx_classify"] or not write["rx_classify"]:
            raise SystemExit(f"no rx_classify_kernel rows for {w}: {ff} {wf}")

        def summary(k):
            fe, wr = sorted(fetch[k]), sorted(write[k])
            fk, wk = fe[len(fe) // 2], wr[len(wr) // 2]
            return {"fetch_size_kb": fk, "write_size_kb": wk,
                    "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
                    "dispatches": len(fe)}
        res["workloads"][w] = summary("rx_classify")
        if fetch["tx_cksum"] and write["tx_cksum"]:  # K2 over the same burst (bench's TX leg)
            res["workloads"][w]["tx_cksum"] = summary("tx_cksum")
        print(w, res["workloads"][w], flush=True)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    if variant:
        res["variant"] = variant
    with open(os.path.join(outdir, f"pmc_{tag}.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
