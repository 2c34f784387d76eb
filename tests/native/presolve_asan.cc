#include <cstdio>
#include <random>
// Memory/UB check of the presolve passes and their postsolve (host code):
// random LPs of every bound type, random solutions of the presolved LP.
// Built and run by tests/test_presolve_native.py with ASan + UBSan.
#include "presolve.h"
using namespace milp::presolve;
int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937_64 rng(7);
  auto U = [&](double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); };
  auto I = [&](int a, int b) { return std::uniform_int_distribution<int>(a, b)(rng); };
  const double inf = std::numeric_limits<double>::infinity();
  long total_passes = 0;
  for (int t = 0; t < N; ++t) {
    Lp lp;
    const int m = I(1, 14), n = I(1, 16);
    lp.num_rows = m;
    lp.cols.resize(n);
    for (int c = 0; c < n; ++c) {
      for (int r = 0; r < m; ++r) if (U(0, 1) < 0.35) lp.cols[c].push_back({r, double(I(-3, 3)) + (I(0, 1) ? 0.0 : 0.5)});
      auto& v = lp.cols[c]; size_t w = 0; for (auto& e : v) if (e.coeff != 0) v[w++] = e; v.resize(w);
    }
    if (n > 1 && I(0, 2) == 0) { lp.cols[n - 1] = lp.cols[0]; for (auto& e : lp.cols[n - 1]) e.coeff *= -2; }
    auto bounds = [&](std::vector<double>& lb, std::vector<double>& ub, int k) {
      lb.resize(k); ub.resize(k);
      for (int i = 0; i < k; ++i) { double a = I(-3, 3), b = a + I(0, 3); int ty = I(0, 5);
        lb[i] = (ty == 1 || ty == 3) ? -inf : a; ub[i] = (ty == 2 || ty == 3) ? inf : (ty == 4 ? a : b); }
    };
    bounds(lp.col_lb, lp.col_ub, n); bounds(lp.row_lb, lp.row_ub, m);
    lp.obj.resize(n); for (auto& o : lp.obj) o = I(-3, 3);
    lp.maximize = I(0, 1); lp.offset = I(-2, 2);
    Params p; p.solve_dual_problem = I(0, 2);
    MainPresolve pre(p);
    Lp work = lp;
    const bool post = pre.Run(&work);
    total_passes += pre.applied().size();
    Solution s(work.num_rows, work.num_cols());
    s.status = pre.status() == kInit ? kOptimal : pre.status();
    for (auto& v : s.vstat) v = I(0, 4);
    for (auto& c : s.cstat) c = I(0, 4);
    for (auto& x : s.primal) x = U(-5, 5);
    for (auto& y : s.dual) y = U(-5, 5);
    if (post) pre.Recover(&s);
    if ((int)s.primal.size() != n || (int)s.dual.size() != m || (int)s.vstat.size() != n || (int)s.cstat.size() != m) {
      printf("size mismatch at %d\n", t); return 1;
    }
  }
  printf("ok %d LPs, %ld passes applied\n", N, total_passes);
  return 0;
}
