#!/usr/bin/env python3
"""Development aid: the smallest programs that end under `rocprofv3 --pmc`,
to tell a profiler teardown crash from one of the engine's.
  torch   -- one torch kernel, no engine
  single  -- one small LP through one engine handle
  batch   -- a few branch LPs through the batch API (MILP_SDUAL_POOL as set)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "or-tools_amd"), os.path.join(REPO, "tests")]

what = sys.argv[1]
if what == "torch":
    import torch
    x = torch.ones(4, device="cuda")
    print("torch", float((x * 2).sum()))
elif what == "torch_thread":
    # HIP work from short-lived threads that exit before the process does.
    import threading
    import torch
    x = torch.ones(4, device="cuda")

    def work():
        y = x * 3
        torch.cuda.synchronize()
        print("thread", float(y.sum()))

    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
else:
    from mi_glop import abi, engine
    import lp_gen
    if what == "single":
        h = engine.LpHandle(abi.default_params(use_dual_simplex=1))
        h.load(lp_gen.random_sparse_lp(60, 200, 0.06, 2))
        print("single", h.solve().objective)
    else:
        import jobshop
        lp, _ = jobshop.relaxation(jobshop.FT06)
        root = engine.LpHandle(abi.default_params(use_dual_simplex=1))
        root.load(lp)
        root.solve()
        lbs, ubs = jobshop.child_bounds(lp, _, 8, 3)
        ws = [engine.LpHandle(abi.default_params(use_dual_simplex=1)) for _ in range(4)]
        for w in ws:
            w.load(lp)
        print("batch", [r.objective for r in engine.batch_solve_bounds(ws, lbs, ubs, root.state())])
