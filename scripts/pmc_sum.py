#!/usr/bin/env python3
"""Sums rocprofv3 --pmc counter CSVs under a directory per kernel and counter
(development aid): `pmc_sum.py DIR [KERNEL_SUBSTRING]` prints, for every
kernel whose name contains the substring (default "sdual"), the dispatch
count and each counter's total and per-dispatch mean, plus a few ratios
(instruction-cache miss rate, wait fractions) when their counters are there."""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "sdual"
    totals = collections.defaultdict(float)
    dispatches = collections.defaultdict(set)
    files = glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True)
    for f in sorted(files):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if want not in name:
                    continue
                c = row.get("Counter_Name")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                totals[c] += v
                dispatches[c].add((f, row.get("Dispatch_Id")))
    if not totals:
        print(f"no counters for kernels matching {want!r} in {len(files)} files")
        return
    for c in sorted(totals):
        n = len(dispatches[c])
        print(f"{c:32s} total {totals[c]:.6g}  dispatches {n}  mean {totals[c] / max(1, n):.6g}")
    t = totals
    if t.get("SQC_ICACHE_REQ"):
        print(f"icache miss rate {t.get('SQC_ICACHE_MISSES', 0) / t['SQC_ICACHE_REQ']:.4f}")
    if t.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_IFETCH"):
            if k in t:
                print(f"{k} / SQ_WAVE_CYCLES {t[k] / t['SQ_WAVE_CYCLES']:.4f}")


if __name__ == "__main__":
    main()
