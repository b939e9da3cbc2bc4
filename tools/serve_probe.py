"""tools/serve_probe.py — where a served per-publish call's time goes
(benchmark tooling, not product code).

Builds a config-3-shaped index (--filters, default 1M: the host-side costs do
not depend on the index size; the device walk does, and bench.py's latency leg
measures it on the full 10M), turns on MQM_CFG_SERVE and runs the native
driver (tools/conc_driver.cpp: one std::thread per connection, each calling
mqm_subscribers) for every (threads, grid) pair, printing one JSON line each:
throughput, p50/p99 and the host / device breakdown (mqm_serve_host_us,
mqm_serve_device_us)."""

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=100_000)
    ap.add_argument("--threads", default="1,8,16,32,64")
    ap.add_argument("--grids", default="64")
    ap.add_argument("--calls", type=int, default=300)
    a = ap.parse_args()

    import maxmq_amd
    from bench import _driver
    from tools import mqgen

    w = mqgen.generate(3, n_filters=a.filters, n_topics=a.topics)
    idx = maxmq_amd.TopicsIndex(device=0, serve=True)
    idx.subscribe_workload(w)
    idx.commit()
    D, api = _driver()
    n = len(w.topics)
    data = np.ascontiguousarray(w.topics.data[: int(w.topics.offs[n])])
    offs = np.ascontiguousarray(w.topics.offs[: n + 1].astype(np.uint64))

    def run(threads, calls):
        lat = np.zeros(threads * calls, np.uint64)
        dsum = C.c_uint64()
        ns = D.mqd_concurrent(C.byref(api), idx._h, data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                              n, threads, calls, lat.ctypes.data_as(C.c_void_p), C.byref(dsum))
        if ns < 0:
            raise RuntimeError("mqm_subscribers failed in the driver")
        us = lat.astype(np.float64) / 1e3
        return {"topics_per_s": threads * calls / (ns * 1e-9), "p50_us": float(np.median(us)),
                "p99_us": float(np.percentile(us, 99))}

    print(json.dumps({"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "filters": a.filters}),
          flush=True)
    for g in [int(x) for x in a.grids.split(",")]:
        idx.serve_policy(g, 20000)
        for t in [int(x) for x in a.threads.split(",")]:
            run(t, 20)  # warm (and the server launched)
            idx.serve_host_us()
            d0 = idx.serve_device_us()
            r = run(t, a.calls)
            r.update(threads=t, grid=g, host_us=idx.serve_host_us(), device_us_cumulative=d0["total"])
            print(json.dumps(r), flush=True)
    idx.close()


if __name__ == "__main__":
    main()
