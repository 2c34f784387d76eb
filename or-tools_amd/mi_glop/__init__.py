"""MI355X-native revised-simplex LP engine (drop-in for OR-Tools' Glop).

Modules:
  abi            ctypes structs of include/mi_lp.h
  lp             LinearProgram container (glop::LinearProgram subset)
  engine         handle over the HIP engine (libmi_lp.so)
  linear_solver  pywraplp-style Solver front end (MPSolver GLOP mirror)
"""
from . import abi, lp  # noqa: F401
