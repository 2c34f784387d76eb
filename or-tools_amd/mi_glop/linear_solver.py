"""MPSolver-shaped front end over the MI355X engine (config 1 plumbing).

Mirrors the subset of or-tools' pywraplp / MPSolver that an LP user of the
GLOP backend touches (linear_solver/linear_solver.h:199, 451-466, 691-697,
1583-1867; the GLOP interface linear_solver/glop_interface.cc:37-431):

    solver = Solver.CreateSolver("GLOP")        # or Solver("name", GLOP_LINEAR_PROGRAMMING)
    x = solver.NumVar(0, 10, "x")
    c = solver.Constraint(-solver.infinity(), 14, "c")
    c.SetCoefficient(x, 2.0)
    solver.Objective().SetCoefficient(x, 3.0)
    solver.Objective().SetMaximization()
    status = solver.Solve()                     # Solver.OPTIMAL ...
    x.solution_value(), x.reduced_cost(), c.dual_value(), x.basis_status()

Model -> LinearProgram follows GLOPInterface::ExtractModel + LinearProgram::
CleanUp: one coefficient per (row, column), the last SetCoefficient wins as in
MPConstraint; entries of a column sorted by row, zeros dropped (the
IsCleanedUp precondition of lp_solver.cc:185-191).
Status maps are glop_utils.cc:18-125. Solve() goes through the engine's
LPSolver layer (mi_lp_solver_solve: Glop's presolve passes and scaling
preprocessor, the simplex on the presolved and scaled LP, RecoverSolution,
the postsolve and LoadAndVerifySolution, lp_solver.cc:150-790), with Glop's
defaults (use_preprocessing on, parameters.proto:326).
Integer variables are rejected (GLOP is an LP solver: IsMIP() is false).
"""
import math

import numpy as np

from . import abi, engine, lp

# MPSolver::OptimizationProblemType (linear_solver.h:199)
GLOP_LINEAR_PROGRAMMING = 2


class Variable:
    def __init__(self, solver, index, lb, ub, name):
        self._solver = solver
        self._index = index
        self._lb = float(lb)
        self._ub = float(ub)
        self._name = name

    def name(self):
        return self._name

    def index(self):
        return self._index

    def lb(self):
        return self._lb

    def ub(self):
        return self._ub

    def SetBounds(self, lb, ub):
        self._lb, self._ub = float(lb), float(ub)
        self._solver._changed()

    def SetLb(self, lb):
        self.SetBounds(lb, self._ub)

    def SetUb(self, ub):
        self.SetBounds(self._lb, ub)

    def solution_value(self):
        return self._solver._value("x", self._index)

    def reduced_cost(self):
        return self._solver._value("rc", self._index)

    def basis_status(self):
        return self._solver._value("vstat", self._index)

    SolutionValue = solution_value
    ReducedCost = reduced_cost


class Constraint:
    def __init__(self, solver, index, lb, ub, name):
        self._solver = solver
        self._index = index
        self._lb = float(lb)
        self._ub = float(ub)
        self._name = name
        self._coefs = {}

    def name(self):
        return self._name

    def index(self):
        return self._index

    def lb(self):
        return self._lb

    def ub(self):
        return self._ub

    def SetBounds(self, lb, ub):
        self._lb, self._ub = float(lb), float(ub)
        self._solver._changed()

    def SetCoefficient(self, var, coef):
        self._coefs[var.index()] = float(coef)
        self._solver._changed()

    def GetCoefficient(self, var):
        return self._coefs.get(var.index(), 0.0)

    def dual_value(self):
        return self._solver._value("y", self._index)

    def activity(self):
        return self._solver._value("act", self._index)

    def basis_status(self):
        return self._solver._value("cstat", self._index)

    DualValue = dual_value


class Objective:
    def __init__(self, solver):
        self._solver = solver
        self._coefs = {}
        self._offset = 0.0
        self._maximize = False

    def SetCoefficient(self, var, coef):
        self._coefs[var.index()] = float(coef)
        self._solver._changed()

    def GetCoefficient(self, var):
        return self._coefs.get(var.index(), 0.0)

    def SetOffset(self, value):
        self._offset = float(value)
        self._solver._changed()

    def offset(self):
        return self._offset

    def SetMaximization(self):
        self._maximize = True
        self._solver._changed()

    def SetMinimization(self):
        self._maximize = False
        self._solver._changed()

    def SetOptimizationDirection(self, maximize):
        self._maximize = bool(maximize)
        self._solver._changed()

    def maximization(self):
        return self._maximize

    def Value(self):
        return self._solver._objective_value()


class Solver:
    # MPSolver::ResultStatus (linear_solver.h:451-466)
    OPTIMAL, FEASIBLE, INFEASIBLE, UNBOUNDED, ABNORMAL, MODEL_INVALID = range(6)
    NOT_SOLVED = 6
    # MPSolver::BasisStatus (linear_solver.h:691-697)
    FREE, AT_LOWER_BOUND, AT_UPPER_BOUND, FIXED_VALUE, BASIC = range(5)
    GLOP_LINEAR_PROGRAMMING = GLOP_LINEAR_PROGRAMMING

    # glop_utils.cc:18-49 GlopToMPSolverResultStatus
    _STATUS = {
        abi.OPTIMAL: 0, abi.PRIMAL_FEASIBLE: 1,
        3: 2, abi.PRIMAL_INFEASIBLE: 2, abi.DUAL_UNBOUNDED: 2,   # INFEASIBLE_OR_UNBOUNDED = 3
        abi.DUAL_INFEASIBLE: 3, abi.PRIMAL_UNBOUNDED: 3,
        abi.DUAL_FEASIBLE: 6, 6: 6,                               # INIT = 6
        abi.ABNORMAL: 4, abi.IMPRECISE: 4, abi.INVALID_PROBLEM: 4,
    }
    # glop::VariableStatus -> MPSolver::BasisStatus (glop_utils.cc:51-66)
    _BASIS = {0: 4, 1: 3, 2: 1, 3: 2, 4: 0}

    def __init__(self, name="", problem_type=GLOP_LINEAR_PROGRAMMING, device=0):
        if problem_type != GLOP_LINEAR_PROGRAMMING:
            raise ValueError("only GLOP_LINEAR_PROGRAMMING is backed by this engine")
        self._name = name
        self._device = device
        self._vars = []
        self._cons = []
        self._objective = Objective(self)
        self._params = abi.default_params()
        self._solver_params = abi.default_solver_params()
        self._time_limit_ms = 0
        self._handle = None
        self._sol = None
        self._iterations = 0

    @staticmethod
    def CreateSolver(solver_id):
        """linear_solver.cc:563 name "glop" (case-insensitive), as in
        MPSolver::CreateSolver; any other backend returns None."""
        if solver_id.upper() in ("GLOP", "GLOP_LINEAR_PROGRAMMING"):
            return Solver("glop", GLOP_LINEAR_PROGRAMMING)
        return None

    @staticmethod
    def infinity():
        return math.inf

    Infinity = infinity

    # --- model ------------------------------------------------------------
    def NumVar(self, lb, ub, name=""):
        v = Variable(self, len(self._vars), lb, ub, name or f"x{len(self._vars)}")
        self._vars.append(v)
        self._changed()
        return v

    def IntVar(self, lb, ub, name=""):
        raise ValueError("GLOP solves LPs only (MPSolverInterface::IsMIP() is false)")

    BoolVar = IntVar

    def Constraint(self, lb=-math.inf, ub=math.inf, name=""):
        c = Constraint(self, len(self._cons), lb, ub, name or f"c{len(self._cons)}")
        self._cons.append(c)
        self._changed()
        return c

    RowConstraint = Constraint
    # C++ MPSolver spellings (linear_solver.h)
    MakeNumVar = NumVar
    MakeRowConstraint = Constraint

    def MutableObjective(self):
        return self._objective

    def Objective(self):
        return self._objective

    def Minimize(self, expr):
        self._set_objective(expr, False)

    def Maximize(self, expr):
        self._set_objective(expr, True)

    def _set_objective(self, terms, maximize):
        self._objective._coefs = {}
        for var, coef in dict(terms).items():
            self._objective._coefs[var.index()] = float(coef)
        self._objective._maximize = maximize
        self._changed()

    def variables(self):
        return list(self._vars)

    def constraints(self):
        return list(self._cons)

    def NumVariables(self):
        return len(self._vars)

    def NumConstraints(self):
        return len(self._cons)

    def SetTimeLimit(self, ms):
        self._time_limit_ms = int(ms)

    def SetNumThreads(self, n):
        return n == 1

    def EnableOutput(self):
        pass

    def SuppressOutput(self):
        pass

    def SolverVersion(self):
        return "MI355X revised simplex (Glop drop-in)"

    def iterations(self):
        return self._iterations

    def nodes(self):
        return 0  # MPSolverInterface::nodes() is 0 for an LP solver

    def IsMip(self):
        return False

    def _changed(self):
        self._sol = None

    # --- extraction (GLOPInterface::ExtractModel + LinearProgram::CleanUp) --
    def to_linear_program(self):
        n, m = len(self._vars), len(self._cons)
        cols = [[] for _ in range(n)]
        for c in self._cons:
            for j, v in c._coefs.items():
                if v != 0.0:
                    cols[j].append((c.index(), v))
        col_starts = np.zeros(n + 1, np.int64)
        rows, vals = [], []
        for j in range(n):
            entries = sorted(cols[j])
            rows.extend(r for r, _ in entries)
            vals.extend(v for _, v in entries)
            col_starts[j + 1] = len(rows)
        obj = np.zeros(n)
        for j, v in self._objective._coefs.items():
            obj[j] = v
        return lp.LinearProgram(
            m, n, col_starts, np.asarray(rows, np.int32), np.asarray(vals, np.float64),
            np.array([v.lb() for v in self._vars]), np.array([v.ub() for v in self._vars]),
            np.array([c.lb() for c in self._cons]), np.array([c.ub() for c in self._cons]),
            obj, self._objective.offset(), 1.0, self._objective.maximization(), self._name)

    # --- solve (GLOPInterface::Solve, glop_interface.cc:104-169) ----------
    def Solve(self, params=None):
        model = self.to_linear_program()
        p = params if params is not None else self._params
        if self._time_limit_ms:
            # A copy: the caller's params (and the solver's own) keep their
            # time limit, as MPSolver's do.
            p = type(p).from_buffer_copy(p)
            p.max_time_in_seconds = self._time_limit_ms / 1000.0
        if self._handle is None:
            self._handle = engine.LpHandle(p, device=self._device)
        self._handle.set_params(p)
        r, sol = self._handle.solve_lp(model, self._solver_params)
        self._iterations = int(r.iterations)
        status = self._STATUS.get(int(r.problem_status), 4)
        self._sol = {"status": status, "objective": r.objective}
        if r.error_code == 0 and r.problem_status != abi.INVALID_PROBLEM:
            self._sol["x"] = sol["x"]
            self._sol["rc"] = sol["rc"]
            self._sol["y"] = sol["y"]
            self._sol["act"] = sol["act"]
            self._sol["vstat"] = [self._BASIS[int(s)] for s in sol["vstat"]]
            self._sol["cstat"] = [self._BASIS[int(s)] for s in sol["cstat"]]
        return status

    # GlopParameters enum value names (parameters.proto:34-92, 194-210, 42-46).
    _ENUM_VALUES = {
        "DANTZIG": 0, "STEEPEST_EDGE": 1, "DEVEX": 2,
        "NONE": 0, "BIXBY": 1, "TRIANGULAR": 2, "MAROS": 3,
        "DEFAULT": 0, "EQUILIBRATION": 1, "LINEAR_PROGRAM": 2,
        "NO_COST_SCALING": 0, "CONTAIN_ONE_COST_SCALING": 1, "MEAN_COST_SCALING": 2,
        "MEDIAN_COST_SCALING": 3,
        "ALWAYS_DO": 0, "NEVER_DO": 1, "LET_SOLVER_DECIDE": 2,
    }

    def SetSolverSpecificParametersAsString(self, text):
        """GLOPInterface::SetSolverSpecificParametersAsString (glop_interface.cc:
        397-411) reads a GlopParameters text proto; the fields of mi_glop_params
        and of the LPSolver layer are accepted as `name: value` pairs."""
        tokens = text.replace(":", " : ").split()
        i = 0
        while i < len(tokens):
            name = tokens[i]
            if i + 2 >= len(tokens) or tokens[i + 1] != ":":
                return False
            value = tokens[i + 2]
            i += 3
            v = {"true": 1, "false": 0}.get(value.lower(), None)
            if v is None:
                v = self._ENUM_VALUES.get(value)
            if v is None:
                try:
                    v = float(value) if any(ch in value for ch in ".eE") else int(value)
                except ValueError:
                    return False
            if name in dict(abi.MiLpSolverParams._fields_):
                setattr(self._solver_params, name, v)
            elif name in dict(abi.MiGlopParams._fields_):
                setattr(self._params, name, v)
            else:
                return False
        return True

    def _value(self, key, index):
        if self._sol is None or key not in self._sol:
            raise RuntimeError("no solution: call Solve() after the last model change")
        return self._sol[key][index]

    def _objective_value(self):
        if self._sol is None:
            raise RuntimeError("no solution: call Solve() after the last model change")
        return self._sol["objective"]
