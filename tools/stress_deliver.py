#!/usr/bin/env python3
"""Diagnostics: the GPU delivery scenario of tests/test_deliver_oracle.py over
many scenario seeds, a fresh NStack (so a fresh random table hash seed) each
time, in one process; prints every failure (first lines of its assertion).

    python tools/stress_deliver.py [first_seed] [n_seeds]
"""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "dpdk-tcp-udp_protocol_stack_amd"))

import rxgpu as R  # noqa: E402
import test_deliver_oracle as T  # noqa: E402


def main():
    s0 = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    ns_ = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    bad = 0
    for seed in range(s0, s0 + ns_):
        ns = R.NStack(0)
        try:
            T._run(ns, "gpu", seed)
        except AssertionError as e:
            bad += 1
            print(f"seed {seed} FAILED: {str(e)[:600]}", flush=True)
            traceback.print_exc(limit=3)
            # the TCP table and listener table: device image vs host image
            for which in (1, 2):
                hd, hi = ns.ft_dump(which, False)
                dd, di = ns.ft_dump(which, True)
                diff = np.nonzero(hd != dd)[0]
                print(f"  table {which}: info {list(hi)} (device call: {list(di)}), "
                      f"{len(diff)} words differ: {[(int(k), int(hd[k]), int(dd[k])) for k in diff[:24]]}",
                      flush=True)
                if which == 1:
                    print("  host slots:", [tuple(int(x) for x in hd[4 * k:4 * k + 4])
                                            for k in range(len(hd) // 4) if hd[4 * k + 3] != 0xFFFFFFFF],
                          flush=True)
        finally:
            ns.fini()
    print(f"{bad} of {ns_} seeds failed", flush=True)


if __name__ == "__main__":
    main()
