#!/usr/bin/env python3
"""Map a rocprofv3 kernel trace of tools/cfg2_proc.py back to its cases:
per case, the median classify-kernel duration (the kernel alone) and the
median gap between consecutive dispatches (what back-to-back HIP-event timing
adds).  A case slow in its durations is a slower kernel; one slow only in the
gaps is an extra operation between launches.
    python tools/proc_trace.py <cfg2_proc JSON line file> <run_kernel_trace.csv>"""
import csv
import json
import statistics
import sys


def main():
    info = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
    rows = []
    with open(sys.argv[2]) as f:
        for r in csv.DictReader(f):
            if "rx_classify_lane_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]))
    rows.sort()
    total = sum(n for _, n in info["launches"])
    print(f"lane dispatches in trace {len(rows)}, in the launch log {total}")
    if len(rows) != total:
        print("(counts differ: the mapping below is not trustworthy)")
    W = info["warmup"]
    dur, gap, q = {}, {}, {}
    i = 0
    for tag, n in info["launches"]:
        seg = rows[i:i + n]
        i += n
        if tag in ("ramp", "check"):
            continue
        # the run-length groups hold R rounds' (W + S) launches each when a
        # case repeats back to back; otherwise one round: skip each W warmup
        per = W + info["steps"]
        for k in range(0, len(seg), per):
            t = seg[k + W:k + per]
            dur.setdefault(tag, []).extend((e - s) / 1e6 for s, e, _ in t)
            gap.setdefault(tag, []).extend((t[j + 1][0] - t[j][1]) / 1e6 for j in range(len(t) - 1))
            q.setdefault(tag, set()).update(x for _, _, x in t)
    print("case | kernel median ms | gap median us | gap mean us | queues | HIP-event median ms")
    for tag in dur:
        print(f"{tag} | {statistics.median(dur[tag]):.4f} | {statistics.median(gap[tag]) * 1e3:.2f} | "
              f"{statistics.mean(gap[tag]) * 1e3:.2f} | {','.join(sorted(q[tag]))} | "
              f"{info['median_ms'].get(tag)}")


if __name__ == "__main__":
    main()
