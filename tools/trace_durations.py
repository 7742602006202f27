#!/usr/bin/env python3
"""Per-kernel, per-grid dispatch durations from a rocprofv3 --kernel-trace
CSV (diagnostics): one line per (kernel, grid size) with n / median / mean /
min / max in microseconds, so that the dispatches of each bench workload
(different grid sizes) are told apart.

    python tools/trace_durations.py gpurun_out/prof_r02t/run_kernel_trace.csv
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    rows = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"]
        if "rx_" not in name and "tx_" not in name:
            continue
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        rows[(short, grid)].append(d)
    for (name, grid), v in sorted(rows.items(), key=lambda kv: kv[0]):
        print(f"{name[:90]} grid {grid}: n={len(v)} median {statistics.median(v):.1f} us "
              f"mean {statistics.mean(v):.1f} min {min(v):.1f} max {max(v):.1f}")


if __name__ == "__main__":
    main()
