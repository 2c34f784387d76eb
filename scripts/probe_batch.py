#!/usr/bin/env python3
"""Config-4 probe (development aid): children of one job-shop search node
solved by W GPU worker handles, and by W oracle workers, with per-worker
kernel stats. MILP_PHASE_TIMING=1 adds the dual-loop phase split (use a
small --lps then)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from mi_glop import abi, engine  # noqa: E402
import jobshop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=15)
    ap.add_argument("--machines", type=int, default=10)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--lps", type=int, default=128)
    ap.add_argument("--workers", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--node", action="store_true",
                    help="the node's BranchOnVar LPs (bench.py config 4) instead of random fixings")
    a = ap.parse_args()
    jobs = jobshop.random_instance(a.jobs, a.machines, a.seed)
    lp, ycols = jobshop.relaxation(jobs)
    root = engine.LpHandle(abi.default_params(use_dual_simplex=1))
    root.load(lp)
    root.solve()
    state = root.state()
    if a.node:
        from mi_glop import cpsat
        x = root.primal()
        cols = cpsat.fractional_columns(x, ycols, limit=a.lps // 2)
        lbs, ubs = cpsat.branch_lps(cpsat.IntegerTrail(lp.col_lb, lp.col_ub), x, cols)
        a.lps = len(lbs)
    else:
        lbs, ubs = jobshop.child_bounds(lp, ycols, a.lps, a.seed + 1000)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    out = {"m": lp.m, "n": lp.n, "lps": a.lps}
    gpu_res = {}
    for w in a.workers:
        hs = [engine.LpHandle(p) for _ in range(w)]
        for h in hs:
            h.load(lp)
        engine.batch_solve_bounds(hs, lbs[:w], ubs[:w], state)  # warm-up
        for h in hs:
            h.reset_kernel_stats()
        engine.lib().milp_sdual_profile_reset()
        t = time.perf_counter()
        c0 = time.process_time()
        m0 = time.monotonic_ns()
        res = engine.batch_solve_bounds(hs, lbs, ubs, state)
        dt = time.perf_counter() - t
        # The engine's host sampler (MILP_SAMPLE_PROFILE) reports this call.
        os.environ["MILP_SAMPLE_WINDOW"] = f"{m0},{time.monotonic_ns()}"
        cpu = time.process_time() - c0
        gpu_res[w] = res
        its = sum(r.iterations for r in res)
        agg = {}
        for h in hs:
            for k, v in h.kernel_stats().items():
                d = agg.setdefault(k, {"launches": 0, "call_ms": 0.0})
                d["launches"] += v["launches"]
                d["call_ms"] += v["call_ms"]
        out[f"gpu_w{w}"] = {"lps_per_s": a.lps / dt, "iterations": its,
                            "wall_s": dt, "host_cpu_s": cpu,
                            "us_per_iteration_per_worker": 1e6 * dt * w / max(1, its),
                            "kernels": {k: v for k, v in agg.items() if v["launches"] or v["call_ms"]}}
        print(f"[probe] w={w}: {a.lps / dt:.1f} LPs/s", file=sys.stderr, flush=True)
    if a.cpu:
        import oracle_lib
        for w in a.workers:
            ows = [oracle_lib.OracleLp(p) for _ in range(w)]
            for o in ows:
                o.load(lp)
            t = time.perf_counter()
            res = oracle_lib.batch_solve_bounds(ows, lbs, ubs, state)
            dt = time.perf_counter() - t
            same = all(g.problem_status == c.problem_status and g.iterations == c.iterations
                       and g.objective == c.objective for g, c in zip(gpu_res[w], res))
            out[f"parity_w{w}"] = bool(same)
            out[f"cpu_w{w}"] = {"lps_per_s": a.lps / dt,
                                "us_per_iteration_per_worker":
                                    1e6 * dt * w / max(1, sum(r.iterations for r in res))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
