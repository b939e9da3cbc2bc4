"""Sum rocprofv3 FETCH_SIZE / WRITE_SIZE over the match kernels of one batch.

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts exactly half the bytes of wide coalesced reads, so
read bytes = 2 * FETCH_SIZE * 1024 (our gathers are narrower than 16 B/lane and
uncalibrated: the doubled figure is an upper estimate of reads), write bytes =
WRITE_SIZE * 1024.  Infinity-Cache hits are counted too (same section).
usage: pmc_to_traffic.py <gpurun_out dir> <batches profiled>
"""
import csv
import glob
import json
import os
import sys

root, batches = sys.argv[1], int(sys.argv[2])
KERNELS = ("k_walk", "k_emit_small", "k_copy", "k_merge", "k_multi_part", "k_multi", "k_route", "k_chunks", "k_items",
           "k_dfs", "k_table_sizes")


def total(counter):
    per_kernel = {}
    for path in glob.glob(os.path.join(root, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != counter or not any(k in name for k in KERNELS):
                    continue
                k = next(k for k in KERNELS if k in name)
                per_kernel[k] = per_kernel.get(k, 0.0) + float(row["Counter_Value"])
    return per_kernel


fetch, write = total("FETCH_SIZE"), total("WRITE_SIZE")
kib = 1024.0
out = {
    "batches": batches,
    "read_bytes_per_batch_by_kernel": {k: 2 * v * kib / batches for k, v in fetch.items()},
    "write_bytes_per_batch_by_kernel": {k: v * kib / batches for k, v in write.items()},
}
out["hbm_bytes_per_batch"] = sum(out["read_bytes_per_batch_by_kernel"].values()) + sum(
    out["write_bytes_per_batch_by_kernel"].values())
out["note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; reads = 2 x FETCH_SIZE KiB "
               "(gfx950 correction, upper estimate for our narrow gathers), writes = WRITE_SIZE KiB; "
               "match kernels only (scans and copies excluded)")
print(json.dumps(out, indent=1))
