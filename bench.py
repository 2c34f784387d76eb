#!/usr/bin/env python3
"""Benchmark: simplex iterations/sec of the MI355X engine on BASELINE.json's
north-star workload, config 5 (synthetic sparse LP 100k x 1M, 0.01% dense,
dual simplex with dual steepest edge, 1 MI355X), with the dominant kernel's
roofline and the CPU oracle (Glop restatement) timed on the host in the same
run. Config 2 (dense 10k x 50k, primal), config 3 (Netlib-shaped suite) and
config 4 (CP-SAT-style children) follow as extra sections of the same line.

A "step" is one simplex iteration (RevisedSimplex::DualMinimize loop body,
revised_simplex.cc:3058-3367) at iteration 20 000 of the solve (--c5-window):
the solve runs untimed up to there (loading, factorizations, the hypersparse
early phase), then W more warm-up iterations, then exactly K iterations are
timed, bracketed by barrier + device synchronize, with HIP-event kernel
timing on (events are collected after the window, no per-kernel sync).

Multi-GPU: one process per GPU (torchrun). Config 5 runs one independent LP
per rank (seed + rank; replicas, "scaling": "weak", no collective in the data
path): value = all ranks' iterations / max wall time over ranks. One LP does
not divide usefully: its iteration is a chain of dependent host decisions and
triangular solves that every rank would replicate.
--c5-split runs ONE LP split across the ranks by column blocks instead (SURVEY
8(e), mi_lp_set_exchange): every rank runs the same host control flow, owns
one block of [A | I] on its GPU, and the per-column results are joined through
an all-gather every iteration ("scaling": "strong").
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "or-tools_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from mi_glop import abi, distributed, engine  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
COLL_DEVICE = "cuda"  # RCCL collectives on device tensors ("cpu" under gloo)
METRIC = "simplex iterations/sec + batched LPs/sec, 1/2/4/8 MI355X vs Glop CPU"


_T0 = time.perf_counter()


def log(msg):
    """Progress on stderr (keeps long runs visibly alive)."""
    print(f"[bench {time.perf_counter() - _T0:8.1f}s] {msg}", file=sys.stderr, flush=True)


def dense_box_lp(m, n, seed):
    import lp_gen
    return lp_gen.dense_box_lp(m, n, seed)


def cpu_baseline(lp, warm, iters):
    """Oracle (CPU restatement of Glop, single thread) on the same LP: time of
    iterations warm..warm+iters from per-iteration timestamps."""
    import oracle_lib
    p = abi.default_params(max_number_of_iterations=warm + iters)
    o = oracle_lib.OracleLp(p)
    o.record_iteration_times(True)
    o.load(lp)
    t0 = time.perf_counter()
    r = o.solve()
    total = time.perf_counter() - t0
    ts = o.iteration_times()
    if len(ts) >= warm + iters and iters > 0:
        dt = ts[warm + iters - 1] - (ts[warm - 1] if warm > 0 else 0.0)
        rate = iters / dt
    else:
        rate = r.iterations / max(total, 1e-9)
    return rate, dict(iterations=int(r.iterations), wall_s=total,
                      timed_iterations=iters, warm_iterations=warm)


def _solution_digests(h, r):
    """sha256 of everything the drop-in contract names, from an engine handle
    or an oracle handle after a solve (same getters on both)."""
    import hashlib

    def digest(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()

    var, cons = h.statuses()
    return {"iterations": str(int(r.iterations)), "problem_status": str(int(r.problem_status)),
            "error_code": str(int(r.error_code)), "objective": float(r.objective).hex(),
            "basis": digest(h.basis()), "state": digest(h.state()),
            "var_status": digest(var), "cons_status": digest(cons),
            "primal": digest(h.primal()), "duals": digest(h.duals()),
            "reduced_costs": digest(h.reduced_costs())}


def kernel_roofline(stats, traffic_json=None):
    """Roofline of the dominant kernel id of a timed window: algorithmic bytes
    per launch / HIP-event time per launch, against the HBM peak."""
    dom = max(stats, key=lambda k: stats[k]["device_ms"])
    ds = stats[dom]
    launches = max(1, ds["launches"])
    bytes_per_launch = ds["bytes"] / launches
    ms_per_launch = ds["device_ms"] / launches if ds["device_ms"] > 0 else float("nan")
    achieved = bytes_per_launch / (ms_per_launch * 1e-3) / 1e9 if ds["device_ms"] > 0 else 0.0
    traffic = None
    traffic_src = None
    if traffic_json and os.path.exists(traffic_json):
        tj = json.load(open(traffic_json))
        if dom in tj:
            traffic = tj[dom]["traffic_bytes_per_launch"]
            traffic_src = tj.get("_source", traffic_json)
    return {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": traffic_src, "bytes_per_launch": bytes_per_launch,
            "ms_per_launch": ms_per_launch, "launches": ds["launches"]}


def window_stats(ts, start, done, before, after):
    """Per-iteration statistics of a timed window [start, start + done):
    p50/p90/max of the iteration times (from the engine's per-iteration
    timestamps) and the LU refactorizations that fell inside it, so that a
    short window is interpretable (a refactorization costs many iterations)."""
    out = {"refactorizations_in_window": after["factorizations"] - before["factorizations"],
           "u_schedule_levels": after.get("u_levels", 0),
           "u_schedule_outputs": after.get("u_outputs", 0),
           "refactorization_ms_in_window": round(
               1000.0 * (after["factorization_seconds"] - before["factorization_seconds"]), 3)}
    if done > 0 and len(ts) >= start + done and start > 0:
        per = np.diff(np.asarray(ts[start - 1:start + done])) * 1000.0
        out.update(iteration_ms_p50=round(float(np.percentile(per, 50)), 4),
                   iteration_ms_p90=round(float(np.percentile(per, 90)), 4),
                   iteration_ms_max=round(float(per.max()), 4))
    return out


def kernel_table(stats):
    return {k: {"launches": v["launches"], "device_ms": round(v["device_ms"], 3),
                "call_ms": round(v["call_ms"], 3), "GB": round(v["bytes"] / 1e9, 4)}
            for k, v in stats.items() if v["launches"] or v["call_ms"]}


def run_c5(args, rank, world, local_rank, dist, barrier, sync):
    """Config 5: synthetic sparse LP 100k x 1M, 0.01% nnz,
    dual simplex with dual steepest edge. One LP per rank (replicas, seed +
    rank). The solve runs untimed to iteration c5_window + warmup; then
    exactly `steps` iterations are timed with the kernel timing on."""
    import lp_gen
    split = world > 1 and args.c5_split
    lp = lp_gen.sparse_c5_lp(args.c5_m, args.c5_n, 10, args.seed + (0 if split else rank))
    start = args.c5_window + args.warmup
    # The solve is capped where the timed windows end, so that its final
    # state is the one the oracle reaches with the same cap (oracle_check).
    end = start + max(args.steps, args.c5_amortized)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=end)
    h = engine.LpHandle(p, device=local_rank)
    if split:
        # The exchange runs on a gloo group: the joined messages are host
        # bytes the engine's host control flow consumes.
        # The joins run through the engine's C++ same-node exchange
        # (engine/exchange.cc); a gloo group only distributes its name.
        _, _, xchg = distributed.attach_column_split(h, dist, dist.new_group(backend="gloo"),
                                                     transport=args.c5_transport)
    h.load(lp)
    h.record_iteration_times(True)  # per-iteration timestamps (window statistics)
    t = time.perf_counter()
    h.begin(start)
    setup = time.perf_counter() - t
    log(f"c5: solve ran to iteration {start} in {setup:.1f}s (untimed)")
    h.reset_kernel_stats()
    # HIP events bracket the dominant kernels only (two event records per
    # launch of every other kernel cost ~9 % of the window, profiles/r05_tri).
    timed = None if args.c5_timed_kernels == "all" else args.c5_timed_kernels.split(",")
    h.set_kernel_timing(True, kernels=timed)
    before = h.run_counters()
    barrier()
    sync()
    t0 = time.perf_counter()
    fin, it = h.run_until(start + args.steps)
    sync()
    barrier()
    elapsed = distributed.max_over_ranks(time.perf_counter() - t0, dist, COLL_DEVICE)
    stats = h.kernel_stats()
    after = h.run_counters()
    done = it - start
    window = window_stats(h.iteration_times(), start, done, before, after)
    roof = kernel_roofline(stats, args.c5_traffic_json)
    if roof["kernel"] in ("tri_solve", "tri_solve_tau") and after.get("u_levels", 0) > 0:
        # The U solve is a dependency chain: each level is a hand-off between
        # workgroups (MI355X_MICROARCH.md handoff-1to1: ~1 us idle, 2.5-5 us
        # with the waves of a loaded CU). Time per level of the schedule in use.
        roof["latency"] = {"levels": after["u_levels"],
                           "us_per_level": 1000.0 * roof["ms_per_launch"] / after["u_levels"],
                           "handoff_us_idle": 1.0}
    # Split: every rank ran the same iterations of one LP; replicas: sum.
    total_done = done if split else distributed.sum_over_ranks(done, dist, COLL_DEVICE)
    log(f"c5: timed {done} iterations in {elapsed:.3f}s")
    # The refactorization-amortized rate: the headline window continued to
    # args.c5_amortized iterations (the headline's own iterations included),
    # so a short --steps window cannot hide the LU refactorizations.
    amortized = None
    span = max(args.c5_amortized, done)
    if not fin and span > done:
        before_a = h.run_counters()
        barrier()
        sync()
        t1 = time.perf_counter()
        fin_a, it_a = h.run_until(start + span)
        sync()
        barrier()
        more = distributed.max_over_ranks(time.perf_counter() - t1, dist, COLL_DEVICE)
        done_a = it_a - start
        amortized = {"timed_iterations": [start, it_a],
                     "value": done_a / (elapsed + more) if elapsed + more > 0 else 0.0,
                     "ms_per_step": 1000.0 * (elapsed + more) / max(1, done_a),
                     "window": window_stats(h.iteration_times(), start, done_a, before,
                                            h.run_counters())}
        log(f"c5: amortized {start}..{it_a}: {amortized['value']:.1f} it/s")
    elif span <= done:
        amortized = {"timed_iterations": [start, start + done], "value": total_done / elapsed
                     if elapsed > 0 else 0.0, "ms_per_step": 1000.0 * elapsed / max(1, done),
                     "window": window}
    # Run on to the cap (untimed): the final state is compared with the
    # oracle's at the same iteration below.
    h.run_until(end + 1)
    final = h.finish()
    digests = _solution_digests(h, final) if rank == 0 and world == 1 else None
    del h
    out = {
        "value": total_done / elapsed if elapsed > 0 else 0.0,
        "ms_per_step": 1000.0 * elapsed / max(1, done),
        "timed_iterations": [start, start + done],
        "finished_early": bool(fin), "setup_and_warmup_s": round(setup, 2),
        "nnz": int(lp.nnz),
        "roofline": roof,
        "kernels": kernel_table(stats),
        "host_ms_per_step": round((1000.0 * elapsed - sum(v["call_ms"] for v in stats.values()))
                                  / max(1, done), 3),
        "device_call_ms_per_step": round(sum(v["call_ms"] for v in stats.values())
                                         / max(1, done), 3),
        "window": window,
        "amortized": amortized,
        "split": split,
        "event_timed_kernels": timed or "all",
    }
    if split:
        ex = stats.get("exchange", {})
        out["exchange"] = {"transport": args.c5_transport,
                           "allgathers_per_step": ex.get("launches", 0) / max(1, done),
                           "us_per_step": 1000.0 * ex.get("call_ms", 0.0) / max(1, done),
                           "bytes_per_step": ex.get("bytes", 0.0) / max(1, done)}
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle_lib
        # The oracle runs the same solve with the same cap; its per-iteration
        # timestamps give its rate on exactly the GPU's headline window and
        # on the amortized window, and its final state must equal the
        # engine's bit for bit (oracle_check).
        log(f"c5: cpu baseline (oracle) to iteration {end}")
        po = abi.default_params(use_dual_simplex=1, max_number_of_iterations=end)
        o = oracle_lib.OracleLp(po)
        o.record_iteration_times(True)
        o.load(lp)
        t = time.perf_counter()
        ro = o.solve()
        wall = time.perf_counter() - t
        ref = _solution_digests(o, ro)
        bad = sorted(k for k in ref if ref[k] != digests[k])
        out["oracle_check"] = {"iteration": int(ro.iterations), "fields": sorted(ref),
                               "mismatches": len(bad), "differing": bad,
                               "digest": ref["primal"][:16]}
        if bad:
            FAILURES.append(f"config 5 at iteration {ro.iterations}: {bad} differ from the oracle")
        log(f"c5: oracle_check at iteration {ro.iterations}: {len(bad)} mismatches")
        ts = o.iteration_times()
        if len(ts) >= start + done and done > 0:
            dt = ts[start + done - 1] - ts[start - 1]
            out["cpu_baseline"] = {
                "value": done / dt, "unit": "iterations/s", "cores": 1, "kind": "port",
                "sample": (f"oracle (C++ restatement of Glop, -O3, 1 thread) on the same LP: "
                           f"iterations {start}..{start + done} of the same solve, the GPU's "
                           f"timed window ({wall:.1f}s wall incl. the untimed part)")}
            if amortized and len(ts) >= end:
                da = ts[end - 1] - ts[start - 1]
                out["cpu_baseline"]["amortized"] = {
                    "value": (end - start) / da, "timed_iterations": [start, end]}
    return out


def run_c2(args, rank, world, local_rank, dist, barrier, sync):
    """Config 2: dense random LP 10k x 50k, primal simplex, Glop defaults.
    Iterations c2_warmup..c2_warmup + c2_steps are timed (replicas per rank),
    then the solve runs on to c2_late and the same number of iterations is
    timed again (late_window). The CPU oracle (0.5 s per iteration here) is
    timed on the early window only."""
    lp = dense_box_lp(args.m, args.n, args.seed + rank)
    params = abi.default_params()  # Glop defaults: primal simplex, steepest edge
    h = engine.LpHandle(params, device=local_rank)
    h.load(lp)
    h.record_iteration_times(True)
    t_setup = time.perf_counter()
    h.begin(args.c2_warmup)  # load to HBM, factorize, first norms, warm-up iterations
    t_setup = time.perf_counter() - t_setup
    log(f"c2: warm-up done in {t_setup:.1f}s; timing {args.c2_steps} iterations")
    h.reset_kernel_stats()
    h.set_kernel_timing(True)
    before = h.run_counters()
    barrier()
    sync()
    t0 = time.perf_counter()
    finished, it = h.run_until(args.c2_warmup + args.c2_steps)
    sync()
    barrier()
    elapsed = distributed.max_over_ranks(time.perf_counter() - t0, dist, COLL_DEVICE)
    stats = h.kernel_stats()
    done = it - args.c2_warmup
    window = window_stats(h.iteration_times(), args.c2_warmup, done, before, h.run_counters())
    total_done = distributed.sum_over_ranks(done, dist, COLL_DEVICE)
    # A late window of the same length: the host LU solves grow as dense
    # columns enter the basis, so the early rate overstates the solve.
    late = None
    if args.c2_late > args.c2_warmup + args.c2_steps and not finished:
        t = time.perf_counter()
        fin_l, it_l = h.run_until(args.c2_late)
        reach_s = time.perf_counter() - t
        if not fin_l:
            sync()
            before_l = h.run_counters()
            t0l = time.perf_counter()
            fin_l, it_l2 = h.run_until(it_l + args.c2_steps)
            sync()
            el = distributed.max_over_ranks(time.perf_counter() - t0l, dist, COLL_DEVICE)
            late = {"timed_iterations": [it_l, it_l2], "reached_in_s": round(reach_s, 2),
                    "value": distributed.sum_over_ranks(it_l2 - it_l, dist, COLL_DEVICE) / el
                    if el > 0 else 0.0,
                    "ms_per_step": 1000.0 * el / max(1, it_l2 - it_l),
                    "window": window_stats(h.iteration_times(), it_l, it_l2 - it_l, before_l,
                                           h.run_counters())}
            log(f"c2: late window {it_l}..{it_l2}: {late['value']:.1f} it/s")
    h.stop()
    h.finish()
    del h
    out = {
        "metric": "simplex iterations/sec", "unit": "iterations/s",
        "value": total_done / elapsed if elapsed > 0 else 0.0,
        "late_window": late,
        "ms_per_step": 1000.0 * elapsed / max(1, done),
        "timed_iterations": [args.c2_warmup, args.c2_warmup + done],
        "finished_early": bool(finished), "setup_and_warmup_s": round(t_setup, 3),
        "workload": (f"config 2: dense random LP {args.m}x{args.n} (nnz={int(lp.nnz)}), "
                     f"primal simplex, Glop defaults"),
        "roofline": kernel_roofline(stats, args.traffic_json),
        "kernels": kernel_table(stats),
        "host_ms_per_step": round((1000.0 * elapsed - sum(v["call_ms"] for v in stats.values()))
                                  / max(1, done), 3),
        "window": window,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        log("c2: cpu baseline (oracle)")
        rate, info = cpu_baseline(lp, args.cpu_warmup, args.cpu_iters)
        out["cpu_baseline"] = {
            "value": rate, "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": (f"oracle (C++ restatement of Glop, -O3, 1 thread) on the same "
                       f"{args.m}x{args.n} LP: iterations {args.cpu_warmup}.."
                       f"{args.cpu_warmup + args.cpu_iters} timed "
                       f"({info['wall_s']:.1f}s wall incl. setup)"),
            "late_window": "not timed: the oracle needs ~10 min to reach iteration 1500"}
    return out


def run_c3(args, rank, world, local_rank, dist, barrier, sync):
    """Config 3: a suite of 94 Netlib-shaped LPs solved
    concurrently (tests/netlib_suite.py; the Netlib files are not available
    offline). Unit of work = one LP solved from scratch, device upload
    included. The suite is split across ranks by LPT (strong scaling, no
    collective); value = suite size / slowest rank's time."""
    import concurrent.futures
    import netlib_suite
    import lp_gen
    suite = netlib_suite.suite(max_rows=args.c3_max_rows)
    # The suite is sharded across ranks by LPT (longest processing time
    # first, weight nnz x rows): strong scaling, no collective.
    mine = distributed.lpt_partition([distributed.lp_cost(lp) for lp in suite], world)[rank]
    lps = [suite[i] for i in mine]
    p = abi.default_params()
    warm = engine.LpHandle(p, device=local_rank)  # module load / first launches
    warm.load(lp_gen.random_sparse_lp(40, 100, 0.1, 1))
    warm.solve()
    handles = []
    for lp in lps:
        h = engine.LpHandle(p, device=local_rank)
        h.load(lp)
        handles.append(h)
    log(f"c3: {len(lps)} LPs loaded (largest {max(lp.m for lp in lps)} rows)")

    def progress(done, elapsed):
        # Per-LP progress on stderr: a long or stuck member shows by name.
        left = [lps[i] for i in range(len(lps)) if i not in set(done)]
        big = ", ".join(f"{lp.m}x{lp.n}" for lp in sorted(left, key=lambda q: -q.m)[:3])
        log(f"c3: {len(done)}/{len(lps)} LPs done after {elapsed:.1f}s"
            + (f"; largest running: {big}" if left else ""))

    barrier()
    sync()
    t0 = time.perf_counter()
    res = engine.batch_solve(handles, num_threads=args.c3_workers, progress=progress,
                             progress_s=10.0)
    sync()
    barrier()
    elapsed = distributed.max_over_ranks(time.perf_counter() - t0, dist, COLL_DEVICE)
    statuses = [r.problem_status for r in res]
    slow = sorted(range(len(lps)), key=lambda i: -res[i].solve_seconds)[:5]
    log("c3: slowest LPs: " + ", ".join(
        f"{lps[i].m}x{lps[i].n} {res[i].iterations} it {res[i].solve_seconds:.2f}s" for i in slow))
    out = {
        "metric": "batched LPs/sec", "unit": "LPs/s", "scaling": "strong",
        "value": len(suite) / elapsed, "lps": len(suite), "lps_this_rank": len(lps),
        "seconds": elapsed,
        "workers_per_gpu": args.c3_workers,
        "iterations": int(sum(r.iterations for r in res)),
        "optimal": int(sum(s == abi.OPTIMAL for s in statuses)),
        "workload": (f"config 3: {len(lps)} Netlib-shaped seeded LPs (tests/netlib_suite.py, "
                     f"m 27..{args.c3_max_rows}, 1.5-4 columns per row, all bound types), "
                     f"primal simplex, Glop defaults, solved from scratch"),
    }
    stats = _agg_stats(handles)
    for h in handles:
        h.close()
    # The same batch again on fresh handles with event timing on: the
    # dominant kind's device time (the timed pass above runs without events).
    timed_pass = None
    try:
        if args.profile_batch:
            raise RuntimeError("skipped (--profile-batch)")
        th = []
        for lp in lps:
            h = engine.LpHandle(p, device=local_rank)
            h.load(lp)
            h.set_kernel_timing(True)
            th.append(h)
        engine.batch_solve(th, num_threads=args.c3_workers)
        timed_pass = _agg_stats(th)
        for h in th:
            h.close()
    except Exception as e:  # a report, never a reason to fail the bench
        log(f"c3: event-timed pass unavailable: {e}")
    out["roofline"] = batched_roofline_from(stats, elapsed, timed_pass, args.c3_traffic_json,
                                            len(lps))
    if args.profile_batch:
        log(f"c3: LPs solved in this process: {len(lps) + 1}")
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle_lib
        log("c3: cpu baseline (oracle)")

        def solve_one(lp):
            o = oracle_lib.OracleLp(p)
            o.load(lp)
            return o.solve()

        t = time.perf_counter()
        with concurrent.futures.ThreadPoolExecutor(args.c3_cpu_threads) as ex:
            ref = list(ex.map(solve_one, suite))
        dt = time.perf_counter() - t
        slow = sorted(range(len(suite)), key=lambda i: -ref[i].solve_seconds)[:5]
        log("c3: oracle's slowest LPs: " + ", ".join(
            f"{suite[i].m}x{suite[i].n} {ref[i].iterations} it {ref[i].solve_seconds:.2f}s"
            for i in slow))
        if world == 1:
            out["oracle_check"] = oracle_check(res, [ref[i] for i in mine])
        out["cpu_baseline"] = {
            "value": len(suite) / dt, "unit": "LPs/s", "cores": args.c3_cpu_threads,
            "kind": "port",
            "sample": f"oracle, {args.c3_cpu_threads} threads, the same {len(suite)} LPs"}
    return out


def oracle_check(got, ref):
    """Status, iteration count and objective of every GPU result against the
    oracle's for the same LP (bit-equal objective). Mismatches are reported
    in the line and make bench.py exit non-zero after printing it."""
    bad = []
    for i, (a, b) in enumerate(zip(got, ref)):
        same_obj = a.objective == b.objective or (np.isnan(a.objective) and np.isnan(b.objective))
        if (a.error_code, a.problem_status, a.iterations) != \
                (b.error_code, b.problem_status, b.iterations) or not same_obj:
            bad.append(i)
    if bad:
        FAILURES.append(f"{len(bad)} of {len(ref)} batched LPs differ from the oracle")
    return {"lps": len(ref), "mismatches": len(bad), "first": bad[:8]}


FAILURES = []


def _agg_stats(handles):
    agg = {}
    for h in handles:
        for k, v in h.kernel_stats().items():
            a = agg.setdefault(k, {"launches": 0, "bytes": 0.0, "device_ms": 0.0, "call_ms": 0.0})
            for f in a:
                a[f] += v[f]
    return agg


def batched_roofline(handles, wall_s, timed_pass=None, traffic_json=None, lps=0):
    return batched_roofline_from(_agg_stats(handles), wall_s, timed_pass, traffic_json, lps)


def batch_traffic(traffic_json, lps):
    """HBM bytes of a batch of `lps` LPs from a profiled run of the same
    section (scripts/profile_bench.sh: FETCH_SIZE x2 + WRITE_SIZE of every
    engine kernel of the run, per LP solved in it), or (None, None)."""
    if not traffic_json or not os.path.exists(traffic_json) or lps <= 0:
        return None, None
    tj = json.load(open(traffic_json))
    b = tj.get("_batch")
    if not b:
        return None, None
    return b["bytes_per_lp"] * lps, tj.get("_source", traffic_json)


def batched_roofline_from(agg, wall_s, timed_pass=None, traffic_json=None, lps=0):
    """Roofline of the batch's dominant kernel kind, summed over the handles
    of the timed batch: algorithmic bytes (the engine's per-kind formulas,
    DESIGN.md section 4; for the device dual segments 12 bytes per operation
    of Glop's own deterministic-time counts plus the arena bytes moved) over
    the batch's wall time: the LPs run concurrently, so that is the rate the
    GPU sustained. The kind's summed per-LP time is reported beside it
    (device time where the engine measured it, else its callers' waits).
    `timed_pass`: the kernel stats of a second run of the same batch with
    event timing on (HIP events on each handle's stream), whose device time
    then picks and times the dominant kind."""
    try:
        timed = {k: a for k, a in agg.items()
                 if a["launches"] > 0 and a["bytes"] > 0 and k != "exchange"}
        if not timed or wall_s <= 0:
            return None
        source = "device"
        if timed_pass:
            dev = {k: v for k, v in timed_pass.items() if k in timed and v["device_ms"] > 0}
            if dev:
                kind = max(dev, key=lambda k: dev[k]["device_ms"])
                a = dict(timed[kind])
                a["device_ms"] = dev[kind]["device_ms"]
                source = "device (event-timed second pass)"
            else:
                timed_pass = None
        if not timed_pass:
            kind, a = max(timed.items(),
                          key=lambda kv: max(kv[1]["device_ms"], kv[1]["call_ms"]))
        per_lp_ms = a["device_ms"] if a["device_ms"] > 0 else a["call_ms"]
        traffic, traffic_src = batch_traffic(traffic_json, lps)
        # The segment's op-count model (12 B per Glop operation) also counts
        # operands that stay in LDS or L2; when the profiled HBM bytes of the
        # whole batch are below it, the counters are the honest numerator.
        basis = "algorithmic bytes (engine per-kind model)"
        numerator = a["bytes"]
        if traffic is not None and traffic < numerator:
            numerator = traffic
            basis = ("HBM counter bytes of the batch (FETCH_SIZE + WRITE_SIZE, "
                     f"{traffic_src}): the op-count model ({a['bytes'] / 1e9:.2f} GB) exceeds them")
        achieved = numerator / wall_s / 1e9
        return {"kernel": kind, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "achieved_basis": basis,
                "traffic": traffic,
                "traffic_unit": "HBM bytes of the whole batch (all engine kernels)",
                "traffic_source": traffic_src, "algorithmic_bytes": a["bytes"],
                "launches": int(a["launches"]), "bytes_per_launch": a["bytes"] / a["launches"],
                "timing": "batch wall", "wall_s": wall_s,
                "summed_kind_ms": per_lp_ms,
                "summed_kind_timing": source if a["device_ms"] > 0 else "call",
                "ms_per_launch": per_lp_ms / a["launches"]}
    except Exception as e:  # the roofline is a report, never a reason to fail the bench
        log(f"batched roofline unavailable: {e}")
        return None


def run_batched(args, rank, world, local_rank, dist, barrier, sync):
    """Config 4: one CP-SAT search node's branching LPs
    (mi_glop.cpsat: BranchOnVar, linear_programming_constraint.cc:485-584).
    The node LP is solved, its fractional order variables (most fractional
    first) each give a down branch (y <= floor) and an up branch (y >= ceil),
    all warm-started from the node's basis state (SolveLpForBranching,
    :443-464). The variables are sharded across ranks (both branches of a
    variable on one rank; strong scaling by default: the node's batch_lps
    LPs split over the ranks, --batch-scaling weak: batch_lps per rank), solved by
    `workers` GPU handles per rank, and folded with BranchOnVar's decisions.
    The only collective: all-reduce(max) of the node's objective lower bound
    (each variable's min over its branches is a valid bound), the cross-GPU
    analogue of SharedResponseManager::UpdateInnerObjectiveBounds."""
    import math
    import jobshop
    from mi_glop import cpsat
    jobs = jobshop.random_instance(args.batch_jobs, args.batch_machines, args.seed)
    lp, ycols = jobshop.relaxation(jobs)
    root = engine.LpHandle(abi.default_params(use_dual_simplex=1), device=local_rank)
    root.load(lp)
    root_res = root.solve()
    state = root.state()
    x = root.primal()
    node = cpsat.IntegerTrail(lp.col_lb, lp.col_ub,
                              obj_lb=math.ceil(root_res.objective - cpsat.K_CP_EPSILON))
    # Strong scaling (BASELINE config 4: one node's ~1k LPs sharded over the
    # GPUs): --batch-lps is the node's total; weak: --batch-lps per GPU.
    strong = args.batch_scaling == "strong"
    per_node = args.batch_lps // 2 if strong else (args.batch_lps // 2) * world
    cols_all = cpsat.fractional_columns(x, ycols, limit=per_node)
    b, e = distributed.shard(len(cols_all), rank, world)
    cols = cols_all[b:e]
    lbs, ubs = cpsat.branch_lps(node, x, cols)
    p = abi.default_params(use_dual_simplex=1, max_number_of_iterations=1000)
    n_workers = max(1, min(args.batch_workers, len(lbs)))
    workers = [engine.LpHandle(p, device=local_rank) for _ in range(n_workers)]
    for w in workers:
        w.load(lp)
    # Warm-up batch (not timed): first-touch allocations on every worker.
    if not args.profile_batch:
        engine.batch_solve_bounds(workers, lbs[:n_workers], ubs[:n_workers], state)
    else:
        log(f"batched: LPs solved in this process: {len(lbs) + 1}")
    for w in workers:
        w.reset_kernel_stats()
    # The bound share goes through the engine's C ABI (mi_lp_share_bound:
    # ncclAllReduce on a device buffer, engine/comm.hip), as a C++ CP-SAT host
    # would call it; the unique id travels over the process group. Rehearsals
    # with every rank on one GPU (RCCL refuses that) use the process group.
    comm, share = None, "torch.distributed all_reduce (" + ("gloo" if COLL_DEVICE == "cpu"
                                                            else "rccl") + ")"
    if COLL_DEVICE != "cpu":
        try:
            comm = distributed.NativeComm(rank, world, local_rank, dist=dist)
            share = "mi_lp_share_bound (RCCL ncclAllReduce max, float64, device buffer)"
        except Exception as e:  # reported in the line, never a reason to fail
            log(f"batched: native RCCL communicator unavailable: {e}")
    barrier()
    sync()
    t0 = time.perf_counter()
    res = engine.batch_solve_bounds(workers, lbs, ubs, state)
    summary = cpsat.fold_node(cpsat.IntegerTrail(node.lb, node.ub, node.obj_lb), x, cols, res)
    if comm is not None:
        node_lb = comm.share_bound(summary["obj_lb"], distributed.NativeComm.MAX)
    else:
        node_lb = -distributed.share_bound(-summary["obj_lb"], dist, COLL_DEVICE)
    sync()
    barrier()
    elapsed = distributed.max_over_ranks(time.perf_counter() - t0, dist, COLL_DEVICE)
    total = distributed.sum_over_ranks(len(lbs), dist, COLL_DEVICE)
    out = {
        "metric": "batched LPs/sec", "value": total / elapsed, "unit": "LPs/s",
        "scaling": args.batch_scaling, "lps_this_rank": len(lbs),
        "lps": int(total), "seconds": elapsed, "workers_per_gpu": n_workers,
        "host_threads_per_gpu": min(n_workers, 16),
        "mean_iterations": float(np.mean([r.iterations for r in res])) if res else 0.0,
        "root_objective": float(root_res.objective), "root_iterations": int(root_res.iterations),
        "node_obj_lb": node_lb, "bound_share": share, "deductions": int(summary["deductions"]),
        "speculative_lps": int(summary["speculative"]),
        "workload": (f"config 4: job-shop {args.batch_jobs}x{args.batch_machines} (seeded "
                     f"Taillard-style instance; ta041 itself is 50x10) big-M LP relaxation, m={lp.m} n={lp.n}; one search "
                     f"node's BranchOnVar LPs: {len(cols_all)} fractional order variables x 2 "
                     f"branches, dual simplex warm-started from the node basis, cap 1000 "
                     f"iterations"),
    }
    out["roofline"] = batched_roofline(workers, elapsed, None, args.c4_traffic_json, len(lbs))
    if comm is not None:
        comm.close()
    if rank == 0 and world == 1 and args.batch_share_lps > 0:
        # One GPU's share of an 8-way split of the node (BASELINE config 4 at
        # 8 GPUs): the first batch_share_lps children on as many handles.
        k = min(args.batch_share_lps, len(lbs))
        sub = workers[:k]
        t1 = time.perf_counter()
        res_k = engine.batch_solve_bounds(sub, lbs[:k], ubs[:k], state)
        dt_k = time.perf_counter() - t1
        out["share_8way"] = {"lps": k, "workers": len(sub), "value": k / dt_k, "seconds": dt_k,
                             "unit": "LPs/s"}
        log(f"batched: {k} LPs on {len(sub)} handles: {k / dt_k:.1f} LPs/s")
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle_lib
        ows = [oracle_lib.OracleLp(p) for _ in range(args.batch_cpu_threads)]
        for w in ows:
            w.load(lp)
        n_cpu = min(len(lbs), args.batch_cpu_lps)
        t0 = time.perf_counter()
        ref = oracle_lib.batch_solve_bounds(ows, lbs[:n_cpu], ubs[:n_cpu], state)
        dt = time.perf_counter() - t0
        out["oracle_check"] = oracle_check(res[:n_cpu], ref)
        if "share_8way" in out:
            k = out["share_8way"]["lps"]
            out["share_8way"]["oracle_check"] = oracle_check(res_k, ref[:k]) if k <= n_cpu \
                else None
            t1 = time.perf_counter()
            oracle_lib.batch_solve_bounds(ows, lbs[:k], ubs[:k], state)
            out["share_8way"]["cpu_baseline"] = {
                "value": k / (time.perf_counter() - t1), "unit": "LPs/s",
                "cores": args.batch_cpu_threads, "kind": "port",
                "sample": f"oracle, {args.batch_cpu_threads} threads, the same {k} LPs"}
        out["cpu_baseline"] = {
            "value": n_cpu / dt, "unit": "LPs/s", "cores": args.batch_cpu_threads, "kind": "port",
            "sample": f"oracle, {args.batch_cpu_threads} threads, the first {n_cpu} of the same "
                      f"branch LPs"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000,
                    help="timed config-5 iterations (the headline)")
    ap.add_argument("--warmup", type=int, default=20,
                    help="untimed config-5 iterations after --c5-window")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--c5-m", type=int, default=100000)
    ap.add_argument("--c5-n", type=int, default=1000000)
    ap.add_argument("--c5-window", type=int, default=20000,
                    help="config-5 iteration where the timed window starts")
    ap.add_argument("--c5-amortized", type=int, default=1000,
                    help="config-5 iterations of the refactorization-amortized window "
                         "(starts with the headline window)")
    ap.add_argument("--c5-timed-kernels", default="tri_solve,tri_solve_tau",
                    help="kernel ids bracketed with HIP events in the config-5 windows "
                         "(comma-separated, or 'all')")
    ap.add_argument("--c5-transport", default="shm", choices=["shm", "gloo"],
                    help="N > 1: the split's join transport (C++ shared memory, or gloo)")
    ap.add_argument("--c5-split", action="store_true",
                    help="N > 1: one config-5 LP split by column blocks over the ranks "
                         "(strong scaling) instead of one independent LP per rank")
    ap.add_argument("--c5-replicas", action="store_true",
                    help="N > 1: one independent config-5 LP per rank (the default)")
    ap.add_argument("--c5-traffic-json",
                    default=os.path.join(REPO, "profiles", "traffic_c5.json"),
                    help="per-launch HBM bytes of the config-5 kernels (profiles/)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the config-5 headline (profiling runs of the other sections)")
    ap.add_argument("--no-c2", action="store_true", help="skip the config-2 section")
    ap.add_argument("--m", type=int, default=10000, help="config-2 rows")
    ap.add_argument("--n", type=int, default=50000, help="config-2 columns")
    ap.add_argument("--c2-steps", type=int, default=64)
    ap.add_argument("--c2-warmup", type=int, default=3)
    ap.add_argument("--c2-late", type=int, default=1500,
                    help="config-2 iteration where a second (late) window starts (0: none)")
    ap.add_argument("--cpu-iters", type=int, default=None,
                    help="config-2 CPU baseline iterations (default: the GPU's --c2-steps)")
    ap.add_argument("--cpu-warmup", type=int, default=None,
                    help="config-2 CPU baseline start (default: the GPU's --c2-warmup)")
    ap.add_argument("--traffic-json",
                    default=os.path.join(REPO, "profiles", "traffic_c2.json"),
                    help="per-launch HBM bytes of the config-2 dominant kernel from a "
                         "separate rocprofv3 --pmc pass (profiles/)")
    ap.add_argument("--batch-lps", type=int, default=1024,
                    help="config-4 branch LPs of the search node (strong) or per GPU (weak); "
                         "0 disables the batched section")
    ap.add_argument("--batch-scaling", default="strong", choices=["strong", "weak"],
                    help="config 4 over N GPUs: one node's LPs split over the ranks (strong, "
                         "BASELINE config 4) or --batch-lps per rank (weak)")
    ap.add_argument("--batch-workers", type=int, default=1024,
                    help="config-4 solver handles per GPU (LPs in flight); the engine runs "
                         "them on at most 16 host threads as fibers with batched launches")
    ap.add_argument("--batch-cpu-threads", type=int, default=16)
    ap.add_argument("--batch-jobs", type=int, default=15)
    ap.add_argument("--batch-machines", type=int, default=10)
    ap.add_argument("--batch-cpu-lps", type=int, default=512)
    ap.add_argument("--batch-share-lps", type=int, default=128,
                    help="N=1: also time this many children on as many handles (one GPU's "
                         "share of an 8-way split of the node); 0 disables")
    ap.add_argument("--no-c3", action="store_true", help="skip the config-3 section")
    ap.add_argument("--profile-batch", action="store_true",
                    help="profiling runs (scripts/profile_bench.sh): config 3 without its "
                         "event-timed second pass, config 4 without its warm-up batch, so "
                         "that the process solves each batch once")
    ap.add_argument("--c3-traffic-json", default=os.path.join(REPO, "profiles", "traffic_c3.json"))
    ap.add_argument("--c4-traffic-json", default=os.path.join(REPO, "profiles", "traffic_c4.json"))
    ap.add_argument("--c3-max-rows", type=int, default=16000,
                    help="largest config-3 member (SURVEY 8(c): m from 27 to ~16k)")
    ap.add_argument("--c3-workers", type=int, default=16)
    ap.add_argument("--c3-cpu-threads", type=int, default=16)
    args = ap.parse_args()
    # The config-2 CPU baseline times the GPU's own early window by default.
    if args.cpu_iters is None:
        args.cpu_iters = args.c2_steps
    if args.cpu_warmup is None:
        args.cpu_warmup = args.c2_warmup

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` on its own: start the N ranks (one process
        # per GPU, torch.distributed.run) before anything touches a GPU, as a
        # child process, and exit with its status.
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
               f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the multi-rank path on a one-GPU box: every rank on GPU 0.
    one_gpu = os.environ.get("MILP_BENCH_ONE_GPU") == "1"
    if one_gpu:
        local_rank = 0
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        if one_gpu:  # RCCL refuses two ranks on one GPU: gloo for the rehearsal
            global COLL_DEVICE
            COLL_DEVICE = "cpu"
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()

    if args.no_c5:  # profiling runs of the other sections only
        c5 = {"value": 0.0, "ms_per_step": 0.0, "timed_iterations": [0, 0], "finished_early": False,
              "setup_and_warmup_s": 0.0, "nnz": 0, "roofline": None, "kernels": {},
              "event_timed_kernels": None, "host_ms_per_step": None,
              "device_call_ms_per_step": None, "window": None, "split": False}
    else:
        log(f"config-5 headline: {args.c5_m}x{args.c5_n}")
        c5 = run_c5(args, rank, world, local_rank, dist, barrier, sync)
        log(f"c5: {c5['value']:.1f} iterations/s")
    c2 = None
    if not args.no_c2:
        log(f"config-2 section: {args.m}x{args.n} dense")
        c2 = run_c2(args, rank, world, local_rank, dist, barrier, sync)
        log(f"c2: {c2['value']:.1f} iterations/s")
    c3 = None
    if not args.no_c3:
        log("config-3 section: Netlib-shaped suite")
        c3 = run_c3(args, rank, world, local_rank, dist, barrier, sync)
        log(f"c3: {c3['value']:.1f} LPs/s")
    batched = None
    if args.batch_lps > 0:
        log(f"batched section: {args.batch_lps} children ({args.batch_scaling} scaling)")
        batched = run_batched(args, rank, world, local_rank, dist, barrier, sync)
        log(f"batched: {batched['value']:.1f} LPs/s")
    if rank != 0:
        return
    line = {
        "metric": METRIC,
        "value": c5["value"],
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": c5["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong" if c5["split"] else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded sparse LP, BASELINE.json config 5 generator, tests/lp_gen.py)",
        "config": {
            "workload": (f"config 5: sparse LP {args.c5_m}x{args.c5_n}, 10 nnz/column "
                         f"(nnz={c5['nnz']}), dual simplex, dual steepest edge, Glop defaults; "
                         f"iterations {c5['timed_iterations'][0]}..{c5['timed_iterations'][1]}"),
            "m": args.c5_m, "n": args.c5_n, "seed": args.seed,
            "timed_iterations": c5["timed_iterations"],
            "finished_early": c5["finished_early"],
            "setup_and_warmup_s": c5["setup_and_warmup_s"],
            "parallelism": f"column_split{world}" if c5["split"] else f"replicas{world}",
        },
        "roofline": c5["roofline"],
        "kernels": c5["kernels"],
        "event_timed_kernels": c5["event_timed_kernels"],
        "host_ms_per_step": c5["host_ms_per_step"],
        "device_call_ms_per_step": c5["device_call_ms_per_step"],
        "window": c5["window"],
        "cpu_baseline": c5.get("cpu_baseline"),
        "oracle_check": c5.get("oracle_check"),
        "amortized": c5.get("amortized"),
        "exchange": c5.get("exchange"),
        "c2": c2,
        "c3": c3,
        "batched": batched,
    }
    print(json.dumps(line), flush=True)
    if FAILURES:
        log("PARITY FAILURES: " + "; ".join(FAILURES))
        sys.exit(3)


if __name__ == "__main__":
    main()
