"""The engine's host fork-join helpers (or-tools_amd/csrc/engine/host_pool.h)
against their serial loops: ParallelAppendNonZeros must append exactly the
serial scan's indices, values and largest magnitude for any split. Compiled
here with g++ (host code only)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = r"""
#include "host_pool.h"
#include <cstdio>
#include <random>
int main() {
  std::mt19937_64 rng(7);
  const int sizes[] = {0, 1, 63, 64, 65, 1000, 65535, 65536, 65537, 100000, 300001};
  for (int n : sizes) {
    for (int density = 0; density < 4; ++density) {
      std::vector<double> v(n, 0.0);
      for (int i = 0; i < n; ++i) {
        const double u = std::uniform_real_distribution<double>(0, 1)(rng);
        if (u < (density == 0 ? 0.0 : density == 1 ? 0.01 : density == 2 ? 0.5 : 1.0))
          v[i] = std::uniform_real_distribution<double>(-5, 5)(rng);
      }
      for (int begin : {0, n / 3}) {
        std::vector<int> rows = {-1, -2}, srows = {-1, -2};
        std::vector<double> vals = {9.0}, svals = {9.0};
        double m = 0.5, sm = 0.5;
        milp::ParallelAppendNonZeros(v.data(), begin, n, &rows, &vals, &m);
        for (int i = begin; i < n; ++i) {
          if (v[i] != 0.0) {
            srows.push_back(i);
            svals.push_back(v[i]);
            sm = std::max(sm, std::fabs(v[i]));
          }
        }
        if (rows != srows || vals != svals || m != sm) {
          std::printf("mismatch n=%d density=%d begin=%d\n", n, density, begin);
          return 1;
        }
      }
    }
  }
  std::printf("ok\n");
  return 0;
}
"""


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_parallel_append_non_zeros_matches_serial(tmp_path, threads):
    src = tmp_path / "hp.cc"
    src.write_text(PROG)
    exe = tmp_path / "hp"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread",
                    "-I", os.path.join(REPO, "or-tools_amd", "csrc", "engine"),
                    str(src), "-o", str(exe)], check=True)
    env = dict(os.environ, MILP_HOST_THREADS=threads)
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
