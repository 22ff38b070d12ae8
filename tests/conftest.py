import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sgvamp-py_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def pytest_runtest_logreport(report):
    """SGV_TEST_TIMES=<file>: append each test's call time as it finishes (the
    GPU suite's budget is planned from these; a run cut off still leaves them)."""
    path = os.environ.get("SGV_TEST_TIMES")
    if path and report.when == "call":
        with open(path, "a") as f:
            f.write("%.2f %s %s\n" % (report.duration, report.outcome, report.nodeid))
