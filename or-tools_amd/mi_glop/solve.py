"""`solve --solver=glop` for the MI355X engine: linear_solver/solve.cc:261-398.

    python -m mi_glop.solve --input model.mps [--params "use_preprocessing: true"]
                            [--params_file F] [--time_limit SECONDS]
                            [--output_csv F] [--sol_file F] [--device N]

Reads the model (mi_mps_*: fixed or free MPS), builds the
MPSolver mirror (mi_glop.linear_solver.Solver, GLOP_LINEAR_PROGRAMMING), sets
the GlopParameters text (SetSolverSpecificParametersAsString) and solves it
through the engine's LPSolver layer on the GPU, then prints the reference's
report lines (File, Solver, Parameters, Dimension, Status, Objective,
BestBound, StatusString, Time) and writes the .sol / .csv files the same way.
There is no CPU fallback: without a usable MI355X it exits with an error.
"""
import argparse
import math
import sys
import time

from . import engine, linear_solver, mps

# MPSolverResponseStatus names (linear_solver.proto) of MPSolver::ResultStatus.
_RESPONSE = {0: "MPSOLVER_OPTIMAL", 1: "MPSOLVER_FEASIBLE", 2: "MPSOLVER_INFEASIBLE",
             3: "MPSOLVER_UNBOUNDED", 4: "MPSOLVER_ABNORMAL", 5: "MPSOLVER_MODEL_INVALID",
             6: "MPSOLVER_NOT_SOLVED"}


def build_solver(lp, device=0):
    """MPModelProto -> MPSolver (the model LocalSolve receives)."""
    s = linear_solver.Solver(lp.name or "model", device=device)
    col_names = getattr(lp, "col_names", None) or [f"x{j}" for j in range(lp.n)]
    row_names = getattr(lp, "row_names", None) or [f"c{i}" for i in range(lp.m)]
    xs = [s.NumVar(lp.col_lb[j], lp.col_ub[j], col_names[j]) for j in range(lp.n)]
    cons = [s.Constraint(lp.row_lb[i], lp.row_ub[i], row_names[i]) for i in range(lp.m)]
    for j in range(lp.n):
        for k in range(lp.col_starts[j], lp.col_starts[j + 1]):
            cons[lp.row_idx[k]].SetCoefficient(xs[j], float(lp.vals[k]))
    obj = s.Objective()
    for j in range(lp.n):
        if lp.obj[j] != 0.0:
            obj.SetCoefficient(xs[j], float(lp.obj[j]))
    obj.SetOffset(float(lp.obj_offset))
    obj.SetOptimizationDirection(bool(lp.maximize))
    return s, xs


def parse_args(argv):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--input", required=True, help="REQUIRED: input file name (.mps)")
    ap.add_argument("--solver", default="glop", help="only glop is backed by this engine")
    ap.add_argument("--params", default="", help="GlopParameters in text format")
    ap.add_argument("--params_file", default="", help="GlopParameters text file")
    ap.add_argument("--time_limit", type=float, default=math.inf, help="seconds")
    ap.add_argument("--output_csv", default="", help="write 'name,value' lines")
    ap.add_argument("--sol_file", default="", help="write the solution in .sol format")
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args(argv)
    if args.solver.lower() != "glop":
        ap.error(f"unsupported --solver: {args.solver}")
    if args.params_file and args.params:
        ap.error("--params and --params_file are incompatible")
    if not args.time_limit > 0:
        ap.error("--time_limit must be given a positive duration")
    return args


def main(argv=None):
    args = parse_args(sys.argv[1:] if argv is None else argv)
    lp = mps.read_mps(args.input, with_names=True)
    params = args.params
    if args.params_file:
        with open(args.params_file) as f:
            params = f.read()
    print("%-12s: '%s'" % ("File", args.input))
    s, xs = build_solver(lp, device=args.device)
    if params and not s.SetSolverSpecificParametersAsString(params):
        print(f"invalid --params: {params!r}", file=sys.stderr)
        return 2
    if math.isfinite(args.time_limit):
        s.SetTimeLimit(int(args.time_limit * 1000))
    print("%-12s: %s" % ("Solver", "GLOP_LINEAR_PROGRAMMING"))
    print("%-12s: %s" % ("Parameters", args.params))
    print("%-12s: %d x %d" % ("Dimension", lp.m, lp.n))
    t0 = time.perf_counter()
    try:
        status = s.Solve()
    except engine.EngineUnavailable as exc:
        print(f"error: {exc}", file=sys.stderr)
        return 3
    elapsed = time.perf_counter() - t0
    has_solution = status in (0, 1)
    value = s.Objective().Value() if has_solution else 0.0
    print("%-12s: %s" % ("Status", _RESPONSE.get(status, "MPSOLVER_ABNORMAL")))
    print("%-12s: %15.15e" % ("Objective", value))
    print("%-12s: %15.15e" % ("BestBound", value))
    print("%-12s: %s" % ("StatusString", ""))
    print("%-12s: %-6.4g s" % ("Time", elapsed))
    if args.sol_file and has_solution:
        with open(args.sol_file, "w") as f:
            f.write(f"=obj= {value!r}\n")
            for x in xs:
                f.write(f"{x.name()} {x.solution_value()!r}\n")
    if args.output_csv and has_solution:
        with open(args.output_csv, "w") as f:
            for x in xs:
                f.write("%s,%e\n" % (x.name(), x.solution_value()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
