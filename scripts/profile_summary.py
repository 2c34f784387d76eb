"""Summarise a rocprofv3 run of bench.py (kernel trace + FETCH_SIZE and
WRITE_SIZE passes, each its own run) into profiles/<tag>/:
  kernel_stats.csv   rocprofv3 --stats output, as produced
  summary.md         per kernel: calls, average duration, HBM bytes/launch
  traffic.json       per engine kernel id (bench.py names): HBM bytes per
                     logical launch, for bench.py --traffic-json

FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE reports half of
the bytes of a streaming read (MI355X_MICROARCH.md, HBM section); it is
doubled here. Usage: python scripts/profile_summary.py gpurun_out/prof <tag> [c2|c4|c5]
(writes profiles/<tag>/ and profiles/traffic_<c2|c5>.json for bench.py)
"""
import collections
import csv
import json
import os
import shutil
import sys

GROUPS = {  # HIP kernel name fragment -> engine kernel id (bench.py names)
    "dense_dot_kernel<1,": "pricing", "column_dot_kernel<1,": "pricing",
    "dense_dot_kernel<5,": "pricing", "column_dot_kernel<5,": "pricing",
    "dense_dot_kernel<0,": "update_row", "column_dot_kernel<0,": "update_row",
    "dense_dot_kernel<4,": "update_row", "column_dot_kernel<4,": "update_row",
    "row_wise_update_kernel": "update_row", "row_wise_by_column_kernel": "update_row",
    "tag_rows_kernel": "update_row", "row_wise_full_rows_kernel": "update_row",
    "compact_flags_kernel": "update_row", "compact_small_kernel": "update_row",
    "dual_ratio_bound_kernel": "dual_ratio", "dual_ratio_select_kernel": "dual_ratio",
    "dual_ratio_keys_kernel": "dual_ratio", "dual_flip_walk_kernel": "dual_ratio",
    "boxed_flips_kernel": "dual_ratio",
    "update_reduced_costs_kernel": "rc_update",
    "dense_dot_kernel<2,": "primal_norms", "column_dot_kernel<2,": "primal_norms",
    "row_sum_kernel": "spmv_rows", "column_squared_norm_kernel": "col_norms",
    # one-launch kernels of small LPs (N <= 8192)
    "row_wise_small_kernel": "update_row", "row_wise_small_by_column_kernel": "update_row",
    "column_wise_small_kernel": "update_row", "list_dots_small_kernel": "primal_norms",
    # dense L/U solves of FTRAN (tri_solve.hip): staging, permutes, levels or
    # the readiness-driven single launch
    "tri_gather_kernel": "tri_solve", "tri_scatter_kernel": "tri_solve",
    "tri_level_grid_kernel": "tri_solve", "tri_levels_cu_kernel": "tri_solve",
    "tri_copy_in_kernel": "tri_solve", "tri_copy_out_kernel": "tri_solve",
    "tri_init_kernel": "tri_solve", "tri_syncfree_kernel": "tri_solve",
}


# Kernels that define one logical launch of an engine id (the first list
# that has calls is used): e.g. a pricing pass is one dense-block launch plus
# one CSC launch over the remaining columns.
PRIMARY = {
    "pricing": [["dense_dot_kernel<5,", "dense_dot_kernel<1,"],
                ["column_dot_kernel<5,", "column_dot_kernel<1,"]],
    "dual_ratio": [["dual_ratio_bound_kernel"]],
    "rc_update": [["update_reduced_costs_kernel"]],
    "update_row": [["row_wise_update_kernel", "row_wise_by_column_kernel",
                    "row_wise_full_rows_kernel",
                    "dense_dot_kernel<0,", "dense_dot_kernel<4,",
                    "row_wise_small_kernel", "row_wise_small_by_column_kernel",
                    "column_wise_small_kernel"],
                   ["column_dot_kernel<0,", "column_dot_kernel<4,"]],
    "primal_norms": [["dense_dot_kernel<2,", "list_dots_small_kernel"],
                     ["column_dot_kernel<2,"]],
    "spmv_rows": [["row_sum_kernel"]],
    "col_norms": [["column_squared_norm_kernel"]],
    "tri_solve": [["tri_init_kernel", "tri_gather_kernel"]],
}


def group_of(name):
    for frag, g in GROUPS.items():
        if frag in name:
            return g
    return None


def main(src, tag, workload, lps=0):
    root = os.environ.get("PROFILE_OUT_ROOT") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    out = os.path.join(root, tag)
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(out, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    counters = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    for pas, cname in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        path = os.path.join(src, pas, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != cname:
                continue
            kib = float(r["Counter_Value"])
            counters[r["Kernel_Name"]][cname] += kib * 1024.0 * (2.0 if cname == "FETCH_SIZE" else 1.0)
            if pas == "fetch":
                calls[r["Kernel_Name"]] += 1
    lines = [f"# rocprofv3 summary: {tag}", "",
             "| kernel | calls | avg us | HBM read MB/launch (FETCH_SIZE x2) | write MB/launch |",
             "|---|---|---|---|---|"]
    groups = collections.defaultdict(lambda: [0.0, 0.0, None, 0])  # bytes, ns, anchor, calls
    primary_calls = collections.defaultdict(lambda: collections.defaultdict(int))
    for s in stats:
        name = s["Name"]
        c = counters.get(name, {})
        n = max(1, calls.get(name, 0))
        rd = c.get("FETCH_SIZE", 0.0) / n
        wr = c.get("WRITE_SIZE", 0.0) / n
        lines.append(f"| `{name[:90]}` | {s['Calls']} | {float(s['AverageNs']) / 1e3:.1f} | "
                     f"{rd / 1e6:.2f} | {wr / 1e6:.2f} |")
        g = group_of(name)
        if g:
            total_ns = float(s["TotalDurationNs"])
            gg = groups[g]
            gg[0] += (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0))
            if gg[2] is None or total_ns > gg[1]:
                gg[1], gg[2], gg[3] = total_ns, name, calls.get(name, int(s["Calls"]))
            for level, frags in enumerate(PRIMARY.get(g, [])):
                if any(f in name for f in frags):
                    primary_calls[g][level] += calls.get(name, int(s["Calls"]))
    def logical_launches(g, v):
        for level in sorted(primary_calls[g]):
            if primary_calls[g][level] > 0:
                return primary_calls[g][level]
        return v[3]

    traffic = {g: {"traffic_bytes_per_launch": v[0] / max(1, logical_launches(g, v)),
                   "anchor_kernel": v[2], "launches": logical_launches(g, v)}
               for g, v in groups.items()}
    if lps > 0:
        # Batched sections: every engine kernel of the run (the persistent
        # sdual pool kernel is one dispatch for the whole batch), per LP.
        total = sum(v[0] for v in groups.values())
        total += sum(c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)
                     for name, c in counters.items() if "sdual" in name or "sprimal" in name)
        traffic["_batch"] = {"bytes_total": total, "lps_in_run": lps,
                             "bytes_per_lp": total / lps}
    json.dump(traffic, open(os.path.join(out, "traffic.json"), "w"), indent=1)
    latest = dict(traffic, _source=f"profiles/{tag}")
    json.dump(latest, open(os.path.join(os.path.dirname(out), f"traffic_{workload}.json"), "w"),
              indent=1)
    lines += ["", "Per engine kernel id (bytes per logical launch, all HIP kernels of the id):", ""]
    for g, v in traffic.items():
        if g == "_batch":
            lines.append(f"- batch: {v['bytes_total'] / 1e9:.3f} GB over {v['lps_in_run']} LPs = "
                         f"{v['bytes_per_lp'] / 1e6:.3f} MB per LP")
            continue
        lines.append(f"- {g}: {v['traffic_bytes_per_launch'] / 1e9:.3f} GB/launch "
                     f"(anchor `{v['anchor_kernel'][:60]}`, {v['launches']} launches)")
    open(os.path.join(out, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "c2",
         int(sys.argv[4]) if len(sys.argv) > 4 else 0)
