#!/usr/bin/env python3
"""Config-3 probe (development aid): the Netlib-shaped suite solved by W GPU
worker threads from scratch, with aggregated per-kernel call stats, and by W
oracle threads."""
import argparse
import concurrent.futures
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from mi_glop import abi, engine  # noqa: E402
import lp_gen  # noqa: E402
import netlib_suite  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-rows", type=int, default=1000)
    ap.add_argument("--workers", type=int, nargs="*", default=[8])
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--single", type=int, nargs="*", default=[],
                    help="suite indices solved one at a time (GPU alone, then the oracle)")
    a = ap.parse_args()
    lps = netlib_suite.suite(max_rows=a.max_rows)
    p = abi.default_params()
    warm = engine.LpHandle(p)
    warm.load(lp_gen.random_sparse_lp(40, 100, 0.1, 1))
    warm.solve()
    out = {"lps": len(lps), "max_n": max(lp.n + lp.m for lp in lps)}
    for i in a.single:
        # The suite's critical path: one LP alone, per-iteration latency.
        lp = lps[i]
        h = engine.LpHandle(p)
        h.load(lp)
        t = time.perf_counter()
        r = h.solve()
        dt = time.perf_counter() - t
        ks = {k: {"launches": v["launches"], "call_ms": round(v["call_ms"], 3)}
              for k, v in h.kernel_stats().items() if v["launches"] or v["call_ms"]}
        h.close()
        rec = {"m": lp.m, "n": lp.n, "nnz": int(lp.nnz), "iterations": int(r.iterations),
               "gpu_s": dt, "gpu_us_per_iteration": 1e6 * dt / max(1, r.iterations),
               "kernels": ks}
        if a.cpu:
            import oracle_lib
            o = oracle_lib.OracleLp(p)
            o.load(lp)
            t = time.perf_counter()
            ro = o.solve()
            dt = time.perf_counter() - t
            rec.update(cpu_s=dt, cpu_us_per_iteration=1e6 * dt / max(1, ro.iterations),
                       same_iterations=int(ro.iterations) == int(r.iterations))
        out[f"single_{i}"] = rec
        print(f"[probe] single {i}: {rec}", file=sys.stderr, flush=True)
    for w in a.workers:
        hs = []
        for lp in lps:
            h = engine.LpHandle(p)
            h.load(lp)
            hs.append(h)
        t = time.perf_counter()
        res = engine.batch_solve(hs, num_threads=w)
        dt = time.perf_counter() - t
        its = sum(r.iterations for r in res)
        agg = {}
        for h in hs:
            for k, v in h.kernel_stats().items():
                d = agg.setdefault(k, {"launches": 0, "call_ms": 0.0})
                d["launches"] += v["launches"]
                d["call_ms"] += v["call_ms"]
            h.close()
        out[f"gpu_w{w}"] = {"lps_per_s": len(lps) / dt, "iterations": its,
                            "us_per_iteration_per_worker": 1e6 * dt * w / max(1, its),
                            "kernels": {k: v for k, v in agg.items() if v["launches"] or v["call_ms"]}}
        print(f"[probe] w={w}: {len(lps) / dt:.1f} LPs/s", file=sys.stderr, flush=True)
    if a.cpu:
        import oracle_lib

        def solve_one(lp):
            o = oracle_lib.OracleLp(p)
            o.load(lp)
            return o.solve().iterations

        for w in a.workers:
            t = time.perf_counter()
            with concurrent.futures.ThreadPoolExecutor(w) as ex:
                its = sum(ex.map(solve_one, lps))
            dt = time.perf_counter() - t
            out[f"cpu_w{w}"] = {"lps_per_s": len(lps) / dt,
                                "us_per_iteration_per_worker": 1e6 * dt * w / max(1, its)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
