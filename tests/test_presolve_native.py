"""Host sanitizers (AddressSanitizer + UndefinedBehaviorSanitizer, g++, host
code only) over the presolve passes (or-tools_amd/csrc/engine/presolve.cc)
and the whole LPSolver flow (lp_solver.cc, mi_lp_solver_solve_with):
20 000 random LPs of every bound type each, with random presolved solutions
or a fake simplex returning arbitrary statuses and values."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_presolve_under_asan_ubsan(tmp_path):
    exe = tmp_path / "presolve_asan"
    src = os.path.join(REPO, "tests", "native", "presolve_asan.cc")
    eng = os.path.join(REPO, "or-tools_amd", "csrc", "engine")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-ffp-contract=off",
                    "-I", eng, src, os.path.join(eng, "presolve.cc"), "-o", str(exe)],
                   check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok 20000 LPs")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_lp_solver_flow_under_asan_ubsan(tmp_path):
    exe = tmp_path / "lp_solver_asan"
    src = os.path.join(REPO, "tests", "native", "lp_solver_asan.cc")
    eng = os.path.join(REPO, "or-tools_amd", "csrc", "engine")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-ffp-contract=off",
                    "-I", eng, src, os.path.join(eng, "lp_solver.cc"),
                    os.path.join(eng, "presolve.cc"), "-o", str(exe)],
                   check=True, capture_output=True, text=True, timeout=300)
    r = subprocess.run([str(exe), "20000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok 20000 LPs")
