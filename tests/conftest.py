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


def _make(subdir, target):
    if not os.path.exists(os.path.join(ROOT, target)):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, subdir)])


_make("oracle", "oracle/_build/libmochi_ref.so")
_make("tools", "tools/_build/libmqgen.so")
_make("maxmq_amd/csrc", "maxmq_amd/_lib/libmqmatch.so")
_make("tests/harness", "tests/harness/_build/shim_harness")


@pytest.fixture(scope="session")
def kat():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as fh:
        return json.load(fh)
