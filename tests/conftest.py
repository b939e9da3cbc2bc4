"""pytest configuration: the `gpu` marker and on-demand builds of the in-tree
libraries (product, oracle, generator) so the CPU suite works from a clean
checkout."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _make(subdir, target, always=False):
    # (always: small harnesses compiled against the library's headers — make
    # rebuilds them when a header they include changed, e.g. the Workspace
    # layout guard_test fills in)
    if always or not os.path.exists(os.path.join(ROOT, target)):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, subdir)])


_make("oracle", "oracle/_build/libmochi_ref.so")
_make("tools", "tools/_build/libmqgen.so")
_make("maxmq_amd/csrc", "maxmq_amd/_lib/libmqmatch.so")
_make("tests/harness", "tests/harness/_build/shim_harness")
_make("tests/harness", "tests/harness/_build/churn_harness")
_make("tests/harness", "tests/harness/_build/guard_test", always=True)
_make("tests/harness", "tests/harness/_build/tok_test")


@pytest.fixture(scope="session")
def kat():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as fh:
        return json.load(fh)


# A heartbeat for long GPU tests (the C4 shard test runs for minutes): every
# 30 s one line on the terminal (through pytest's terminal reporter, which
# writes past output capture) and into gpurun_out/pytest_heartbeat.log, so a
# runner that takes minutes of silence for a hang sees progress.
_current = {"test": None, "t0": 0.0}


def pytest_runtest_logstart(nodeid, location):
    import time

    _current["test"], _current["t0"] = nodeid, time.time()


@pytest.fixture(scope="session", autouse=True)
def _heartbeat(request):
    import threading
    import time

    tr = request.config.pluginmanager.get_plugin("terminalreporter")
    stop = threading.Event()
    path = os.path.join(ROOT, "gpurun_out", "pytest_heartbeat.log")

    def beat():
        while not stop.wait(30.0):
            t = _current["test"]
            if t is None:
                continue
            line = f"[heartbeat {time.strftime('%H:%M:%S')}] {t} running {time.time() - _current['t0']:.0f} s"
            try:
                if tr is not None:
                    tr.write_line(line)
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "a") as fh:
                    fh.write(line + "\n")
            except Exception:
                pass

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
