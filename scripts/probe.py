#!/usr/bin/env python3
"""Engine probe (development aid, not part of the bench contract).

Times one iteration window of the MI355X engine on config 2 (dense, primal)
or config 5 (sparse 100k x 1M, dual steepest edge), optionally next to the
CPU oracle on the same LP, and prints one JSON line with the rate, the setup
time and the per-kernel stats. MILP_PHASE_TIMING=1 adds the host phase split
on stderr.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from mi_glop import abi, engine  # noqa: E402
import lp_gen  # noqa: E402


def log(msg):
    print(f"[probe {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def make_lp(a):
    if a.config == "c2":
        return lp_gen.dense_box_lp(a.m, a.n, a.seed), abi.default_params()
    lp = lp_gen.sparse_c5_lp(a.m, a.n, a.per_col, a.seed)
    return lp, abi.default_params(use_dual_simplex=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["c2", "c5"], default="c2")
    ap.add_argument("--m", type=int, default=10000)
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--per-col", type=int, default=10)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--cpu-steps", type=int, default=0)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--variants", nargs="*", default=None,
                    help="env settings per GPU run, e.g. MILP_DENSE_UNROLL=8,MILP_DEFER_NORMS=0")
    a = ap.parse_args()
    t = time.perf_counter()
    lp, p = make_lp(a)
    out = {"config": a.config, "m": a.m, "n": a.n, "nnz": int(lp.nnz),
           "gen_s": round(time.perf_counter() - t, 2)}
    log(f"generated {a.config} {a.m}x{a.n} nnz={lp.nnz} in {out['gen_s']}s")
    for variant in ([] if a.no_gpu else (a.variants or [""])):
        env = dict(kv.split("=", 1) for kv in variant.split(",") if kv)
        os.environ.update(env)
        log(f"gpu variant {env}")
        h = engine.LpHandle(p)
        h.load(lp)
        t = time.perf_counter()
        h.begin(a.warmup)
        res = {"gpu_setup_s": round(time.perf_counter() - t, 3)}
        log(f"gpu warm-up done in {res['gpu_setup_s']}s")
        h.reset_kernel_stats()
        # Timing brackets every kernel with events (one sync each); the rate
        # is measured with it off, then the kernel split with it on.
        t = time.perf_counter()
        clk0 = {"monotonic": time.monotonic_ns(), "boottime": time.clock_gettime_ns(time.CLOCK_BOOTTIME)}
        fin, it = h.run_until(a.warmup + a.steps)
        dt = time.perf_counter() - t
        clk1 = {"monotonic": time.monotonic_ns(), "boottime": time.clock_gettime_ns(time.CLOCK_BOOTTIME)}
        # The engine's host sampler (MILP_SAMPLE_PROFILE) reports this window.
        os.environ["MILP_SAMPLE_WINDOW"] = f"{clk0['monotonic']},{clk1['monotonic']}"
        done = it - a.warmup
        res.update(gpu_iterations=done, gpu_s=round(dt, 4),
                   gpu_it_per_s=done / dt if dt > 0 else None, finished=fin,
                   window_clock_ns={k: [clk0[k], clk1[k]] for k in clk0})
        h.reset_kernel_stats()
        h.set_kernel_timing(True)
        fin2, it2 = h.run_until(it + a.steps)
        st = h.kernel_stats()
        res["timed_kernel_window"] = [it, it2]
        res["kernels"] = {k: {"launches": v["launches"], "device_ms": round(v["device_ms"], 3),
                              "call_ms": round(v["call_ms"], 3), "GB": round(v["bytes"] / 1e9, 4)}
                          for k, v in st.items() if v["launches"] or v["call_ms"]}
        log(f"gpu: {done} iterations in {dt:.3f}s ({res['gpu_it_per_s']} it/s)")
        h.stop()
        r = h.finish()
        res["status"] = int(r.problem_status)
        res["error_code"] = int(r.error_code)
        res["iterations_total"] = int(r.iterations)
        if fin or fin2:
            log(f"solve ended early: status {r.problem_status} error {r.error_code} after {r.iterations} iterations, "
                f"error: {h.last_error() if hasattr(h, 'last_error') else ''}")
        del h
        for k in env:
            os.environ.pop(k, None)
        out.setdefault("gpu", {})[variant or "default"] = res
    if a.cpu_steps > 0:
        import oracle_lib
        p2 = abi.default_params(use_dual_simplex=p.use_dual_simplex,
                                max_number_of_iterations=a.warmup + a.cpu_steps)
        o = oracle_lib.OracleLp(p2)
        o.record_iteration_times(True)
        o.load(lp)
        t = time.perf_counter()
        r = o.solve()
        total = time.perf_counter() - t
        ts = o.iteration_times()
        if len(ts) >= a.warmup + a.cpu_steps:
            w = ts[a.warmup - 1] if a.warmup > 0 else 0.0
            dt = ts[a.warmup + a.cpu_steps - 1] - w
            out.update(cpu_setup_s=round(w, 3), cpu_it_per_s=a.cpu_steps / dt)
        out.update(cpu_total_s=round(total, 3), cpu_iterations=int(r.iterations))
        log(f"cpu: {out.get('cpu_it_per_s')} it/s")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
