"""Keep the last N dispatches of a rocprofv3 kernel-trace CSV (the probe's
timed window) and print the per-iteration kernel sequence with gaps."""
import csv
import sys

src, dst, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = list(csv.DictReader(open(src)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
with open(dst, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "start_us", "dur_us", "gap_us", "stream"])
    t0 = int(tail[0]["Start_Timestamp"])
    prev_end = None
    for r in tail:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1000 if prev_end is not None else 0.0
        w.writerow([r["Kernel_Name"][:60], f"{(s - t0) / 1000:.1f}", f"{(e - s) / 1000:.1f}",
                    f"{gap:.1f}", r.get("Stream_Id", r.get("Queue_Id", ""))])
        prev_end = max(prev_end or 0, e)
print(len(rows), "dispatches,", len(tail), "kept")
