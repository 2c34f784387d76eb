#!/usr/bin/env python3
"""Slice a rocprofv3 kernel trace (CSV) to the probe's timed window
(scripts/probe.py records the window's CLOCK_MONOTONIC and CLOCK_BOOTTIME
marks) and split it: per-kernel totals, and each triangular solve (the
launches from tri_copy_in or tri_init to tri_copy_out on one queue) as its
span, the kernels' busy time and the gaps between them."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(trace_dir):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"], r.get("Queue_Id", r.get("Stream_Id", ""))))
    rows.sort()
    return rows


def short(name):
    n = name.split("(")[0]
    return n.replace("milp_kernels::", "")


def main():
    rows = load(sys.argv[1])
    probe = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    res = next(iter(probe["gpu"].values()))
    clocks = res["window_clock_ns"]
    best = max(clocks, key=lambda k: sum(1 for r in rows if clocks[k][0] <= r[0] <= clocks[k][1]))
    t0, t1 = clocks[best]
    win = [r for r in rows if t0 <= r[0] and r[1] <= t1]
    its = res["gpu_iterations"]
    print(f"clock {best}; window {(t1 - t0) / 1e6:.1f} ms, {its} iterations, {len(win)} kernels "
          f"(trace {len(rows)})")
    busy = defaultdict(float)
    count = defaultdict(int)
    for s, e, n, q in win:
        busy[short(n)] += (e - s) / 1e3
        count[short(n)] += 1
    total = sum(busy.values())
    print(f"kernel time {total / 1e3:.1f} ms = {total / max(its, 1):.1f} us/iteration "
          f"(window {(t1 - t0) / 1e3 / max(its, 1):.1f} us/iteration)")
    for n in sorted(busy, key=busy.get, reverse=True)[:20]:
        print(f"  {n:40s} {count[n]:7d} launches {busy[n] / 1e3:9.2f} ms "
              f"{busy[n] / count[n]:8.1f} us avg {busy[n] / max(its, 1):8.1f} us/it")
    # Triangular solves: per queue, from a copy-in (or an init without one) to
    # the next copy-out.
    by_q = defaultdict(list)
    for r in win:
        by_q[r[3]].append(r)
    solves = []
    for q, rs in by_q.items():
        cur = None
        for s, e, n, _ in rs:
            k = short(n)
            if k in ("tri_copy_in_kernel",) or (k == "tri_init_kernel" and cur is None):
                cur = {"start": s, "busy": 0.0, "n": 0, "parts": defaultdict(float)}
            if cur is None:
                continue
            cur["busy"] += (e - s) / 1e3
            cur["n"] += 1
            cur["parts"][k] += (e - s) / 1e3
            if k == "tri_copy_out_kernel":
                cur["span"] = (e - cur["start"]) / 1e3
                solves.append(cur)
                cur = None
    if solves:
        sp = sum(x["span"] for x in solves) / len(solves)
        bz = sum(x["busy"] for x in solves) / len(solves)
        nk = sum(x["n"] for x in solves) / len(solves)
        print(f"triangular solves: {len(solves)} ({len(solves) / max(its, 1):.2f}/iteration); "
              f"span {sp:.1f} us, kernels {bz:.1f} us ({nk:.1f} launches), gaps {sp - bz:.1f} us")
        parts = defaultdict(float)
        for x in solves:
            for k, v in x["parts"].items():
                parts[k] += v / len(solves)
        for k, v in sorted(parts.items(), key=lambda kv: -kv[1]):
            print(f"  {k:40s} {v:8.1f} us per solve")
        spans = sorted(x["span"] for x in solves)
        print("  span p10 %.1f p50 %.1f p90 %.1f max %.1f us" % (
            spans[len(spans) // 10], spans[len(spans) // 2], spans[9 * len(spans) // 10], spans[-1]))


if __name__ == "__main__":
    main()
