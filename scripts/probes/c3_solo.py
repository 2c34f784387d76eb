"""Config 3's largest members solved one at a time (no batch) on the GPU
engine and by the oracle: per-iteration time of the host-driven engine
without batch contention. Usage: python scripts/probes/c3_solo.py [k]"""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "or-tools_amd"), os.path.join(R, "tests")]
from mi_glop import abi, engine  # noqa: E402
import netlib_suite  # noqa: E402
import oracle_lib  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 2
suite = netlib_suite.suite(max_rows=16000)
big = sorted(range(len(suite)), key=lambda i: -suite[i].m * suite[i].n)[:k]
p = abi.default_params()
for i in big:
    lp = suite[i]
    h = engine.LpHandle(p, 0)
    h.load(lp)
    t = time.perf_counter()
    r = h.solve()
    dt = time.perf_counter() - t
    o = oracle_lib.OracleLp(p)
    o.load(lp)
    t = time.perf_counter()
    ro = o.solve()
    do = time.perf_counter() - t
    print(f"{lp.m}x{lp.n}: engine {r.iterations} it {dt:.2f}s ({1e3 * dt / max(1, r.iterations):.3f} ms/it),"
          f" oracle {ro.iterations} it {do:.2f}s ({1e3 * do / max(1, ro.iterations):.3f} ms/it)",
          flush=True)
    h.close()
