"""The literal-edge table built on the device at upload (maxmq_amd/csrc/
edges.hip) must be byte-identical to the one the host builds
(flatten.cpp insert_edges_host, snapshot.h layout): a device index and a
host-only index of the same store have equal snapshot digests (the digest
covers every slot of the table).  Small tables have a few slots per
partition (kEdgeParts = 16384), so most edges run past their partition and
the run-past placement (k_edge_spill) is exercised as well as the
per-partition insertion.  Every other GPU test matches through the device
built table."""

import numpy as np
import pytest

import maxmq_amd
from tools import mqgen

pytestmark = pytest.mark.gpu


def _pair(build):
    out = []
    for dev in (0, None):
        idx = maxmq_amd.TopicsIndex(device=dev, autocommit=False)
        build(idx)
        idx.commit()
        out.append(idx)
    return out


@pytest.mark.parametrize("config,overrides", [(1, dict(n_filters=20000, n_topics=10)),
                                              (2, dict(n_filters=60000, n_topics=10)),
                                              (1, dict(n_filters=300000, n_topics=10))])
def test_device_edge_table_equals_host(config, overrides):
    w = mqgen.generate(config, **overrides)
    dev, host = _pair(lambda idx: idx.subscribe_workload(w))
    assert dev.snapshot_digest() == host.snapshot_digest()
    dev.close()
    host.close()


def test_device_edge_table_tiny_and_empty():
    for filters in ([], ["a"], ["a", "a/b", "a/+/c", "#", "$SYS/x", "x/" + "y" * 40]):
        def build(idx, fs=filters):
            for k, f in enumerate(fs):
                idx.subscribe(f"c{k}", maxmq_amd.Subscription(f))
        dev, host = _pair(build)
        assert dev.snapshot_digest() == host.snapshot_digest(), filters
        dev.close()
        host.close()


def test_device_edge_table_with_retained():
    """retained topics add their own trie nodes and edges (config 5's store)"""
    w = mqgen.generate(5, n_filters=2000, n_topics=30000)
    refs = np.arange(len(w.topics), dtype=np.uint64) * 7 + 3

    def build(idx):
        idx.subscribe_workload(w)
        idx.retain_many(w.topics, refs)
    dev, host = _pair(build)
    assert dev.snapshot_digest() == host.snapshot_digest()
    dev.close()
    host.close()
