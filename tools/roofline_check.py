#!/usr/bin/env python3
"""Ties a bench line's roofline to a kernel trace of the same run.

    python tools/roofline_check.py BENCH_JSON TRACE_CSV [PLAIN_BENCH_JSON]

BENCH_JSON: the JSON line printed by the bench process that rocprofv3 traced
(its roofline.kernel = per-dispatch HIP-event timing of the dominant kernel);
TRACE_CSV: that run's rocprofv3 --kernel-trace CSV; PLAIN_BENCH_JSON
(optional): the line of an unprofiled bench run on the same box.  For every
workload: the dispatches of roofline.kernel.name with the workload's grid,
their median / mean from the trace, the frac they give (algorithmic bytes /
duration / 8 TB/s), and the bench's own per-dispatch and per-step fracs, so
the agreement is a number and not a claim."""
import csv
import json
import statistics
import sys
from collections import defaultdict

PEAK = 8000.0  # GB/s


def workloads(line):
    out = {}
    head = line["config"]["workload"].split(":")[0]
    out[head] = dict(roofline=line["roofline"], ms_per_step=line["ms_per_step"],
                     kernel_ms_avg=line.get("kernel_ms_avg"))
    for k, v in line.items():
        if k.startswith("cfg") and isinstance(v, dict) and "roofline" in v:
            out[k] = dict(roofline=v["roofline"], ms_per_step=v["ms_per_step"],
                          kernel_ms_avg=v.get("kernel_ms_avg"))
    return out


def load(path):
    """a bench detail file (the full dict, bench.py write_detail) or a file
    whose last line is a full (round <= 4) bench line"""
    t = open(path).read().strip()
    try:
        return json.loads(t)
    except ValueError:
        return json.loads(t.splitlines()[-1])


def main():
    line = load(sys.argv[1])
    plain = load(sys.argv[3]) if len(sys.argv) > 3 else None
    rows = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[2])):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
        short = name.split("<")[0].split("(")[0]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # ms
        rows[short].append((int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0), d))
    wl = workloads(line)
    pw = workloads(plain) if plain else {}
    print("workload | kernel | trace dispatches | trace median ms | trace mean ms | trace frac "
          "| bench per-dispatch median ms | bench frac (dispatch) | agree | "
          "bench ms_per_step (profiled run) | plain run ms_per_step | plain frac (step)")
    for nm, w in wl.items():
        k = w["roofline"].get("kernel") or {}
        kn = k.get("name")
        alg = w["roofline"]["achieved"] * w["kernel_ms_avg"] * 1e-3 * 1e9 if w.get("kernel_ms_avg") \
            else None
        if not kn or alg is None:
            print(f"{nm} | (no roofline.kernel) |")
            continue
        # the workload's dispatches: the trace grid whose dispatch durations sit
        # nearest the bench's per-dispatch median (each workload has its own grid)
        by_grid = defaultdict(list)
        for g, d in rows.get(kn.split("+")[0], []):
            by_grid[g].append(d)
        if not by_grid:
            print(f"{nm} | {kn} | 0 |")
            continue
        g, ds = min(by_grid.items(),
                    key=lambda kv: abs(statistics.median(kv[1]) - k["median_ms"]))
        med, mean = statistics.median(ds), statistics.mean(ds)
        tf = alg / (med * 1e-3) / 1e9 / PEAK
        agree = tf / k["frac"] - 1.0 if k.get("frac") else float("nan")
        p = pw.get(nm)
        print(f"{nm} | {kn} grid {g} | {len(ds)} | {med:.4f} | {mean:.4f} | {tf:.4f} | "
              f"{k['median_ms']:.4f} | {k['frac']:.4f} | {agree * 100:+.1f}% | "
              f"{w['ms_per_step']:.4f} | "
              f"{p['ms_per_step']:.4f} | {p['roofline']['frac']:.4f}" if p else
              f"{nm} | {kn} grid {g} | {len(ds)} | {med:.4f} | {mean:.4f} | {tf:.4f} | "
              f"{k['median_ms']:.4f} | {k['frac']:.4f} | {agree * 100:+.1f}% | "
              f"{w['ms_per_step']:.4f} | - | -")


if __name__ == "__main__":
    main()
