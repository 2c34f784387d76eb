import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "or-tools_amd"), os.path.join(REPO, "tests"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU oracle runs")


_TIMES = os.environ.get("MILP_TEST_TIMES")


def pytest_runtest_logreport(report):
    """MILP_TEST_TIMES=path: append each test's call duration as it ends (a
    suite cut off by a time limit still leaves its per-test times)."""
    if _TIMES and report.when == "call":
        with open(_TIMES, "a") as f:
            f.write(f"{report.duration:8.2f} {report.outcome} {report.nodeid}\n")
